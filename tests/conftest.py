import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle_lib
    oracle_lib.build()
    return oracle_lib


@pytest.fixture(scope="session")
def gpu_ctx():
    """One context for the whole GPU session (one process on the card).

    torch is imported first so that libmsw.so binds to the same HIP runtime
    as torch (the bench and the device-resident tests share pointers/streams)."""
    import torch  # noqa: F401
    from mini_parallel_amd import Context, is_gpu_available
    if not is_gpu_available():
        pytest.fail("-m gpu tests need a GPU and the built libmsw.so (no CPU fallback)")
    ctx = Context(0)
    yield ctx
    ctx.close()


class FreshCtx:
    """A Context made at its first use, under the environment of that moment:
    the library reads its switches (MSW_LAYOUT, MSW_NO_F16, MSW_HOST_TRACE,
    ...) once, when a context is created, so a test that sets one uses a
    context of its own (closed at teardown)."""

    def __init__(self):
        self._c = None

    def __getattr__(self, k):
        if k.startswith("__"):
            raise AttributeError(k)
        if self._c is None:
            from mini_parallel_amd import Context
            self._c = Context(0)
        return getattr(self._c, k)

    def close(self):
        if self._c is not None:
            self._c.close()
            self._c = None


@pytest.fixture
def fresh_ctx():
    import torch  # noqa: F401  (as gpu_ctx: libmsw.so binds torch's HIP runtime)
    c = FreshCtx()
    yield c
    c.close()
