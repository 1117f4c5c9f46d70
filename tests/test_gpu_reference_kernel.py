"""Parity against the REFERENCE's own GPU kernel, executed on the MI355X.

`make -C oracle ref` compiles the reference's smith_waterman.cl (where it lies
under /root/reference) for gfx950; oracle/ref_cl.py runs its
`smith_waterman_align` through OpenCL with the reference host flow of
gpu_align (aligner.rs:410-532).  The legacy path of this framework
(msw_align_compat, kernel K0, = gpu_align) must return the same integer on
the same inputs and geometry, and so must the CPU restatement
(oracle_compat_align).  Work-group sizes stay <= 256: the reference's
local_scores[256] (smith_waterman.cl:23) makes larger groups undefined.
Run with -m gpu."""
import numpy as np
import pytest

from oracle import ref_cl

pytestmark = pytest.mark.gpu

ACGT = np.frombuffer(b"ACGT", np.uint8)


@pytest.fixture(scope="module")
def ref():
    if not ref_cl.available():
        pytest.fail("oracle/_ref not built: run __graft_entry__.build() where /root/reference exists")
    return ref_cl


def cases():
    rng = np.random.default_rng(2024)
    out = []
    for L in (1, 2, 63, 64, 65, 255, 256, 257, 1000, 4097, 65536, 1_500_000):
        a = rng.choice(ACGT, L).tobytes()
        b = rng.choice(ACGT, L).tobytes()
        out.append((f"random{L}", a, b))
    out.append(("identical", b"ACGT" * 300, b"ACGT" * 300))
    out.append(("all_mismatch", b"A" * 5000, b"C" * 5000))
    # sparse matches (the Kadane runs matter once positions are strided)
    a = bytearray(b"A" * 20000)
    b = bytearray(b"C" * 20000)
    for p in rng.integers(0, 20000, 300):
        b[p] = ord("A")
    out.append(("sparse", bytes(a), bytes(b)))
    # long matching runs broken by mismatches
    a = rng.choice(ACGT, 50000)
    b = a.copy()
    b[rng.integers(0, 50000, 2000)] = ord("N")
    out.append(("runs", a.tobytes(), b.tobytes()))
    out.append(("unequal_lengths", b"ACGTACGTAC" * 100, b"ACGTACGTAC" * 37 + b"TTT"))
    return out


@pytest.mark.parametrize("wg", [64, 128, 256])
@pytest.mark.parametrize("name,s1,s2", cases(), ids=[c[0] for c in cases()])
def test_compat_matches_reference_kernel(gpu_ctx, oracle, ref, name, s1, s2, wg):
    L = min(len(s1), len(s2))
    W, G = ref.gpu_align_geometry(L, max_wg=wg)
    want = ref.run_align(s1, s2, W, G)
    assert gpu_ctx.compat(s1, s2, wg=W, max_groups=1_000_000) == want
    assert oracle.compat_align(s1, s2, W, 1_000_000) == want


@pytest.mark.parametrize("max_groups", [1, 3, 7, 100])
def test_compat_strided_kadane_matches_reference_kernel(gpu_ctx, oracle, ref, max_groups):
    """Group count capped below ceil(L / W): each work item then scans a
    strided run of positions (the only case where Kadane state carries)."""
    rng = np.random.default_rng(max_groups)
    for L in (1000, 33333):
        a = rng.choice(ACGT, L)
        b = a.copy()
        b[rng.random(L) < 0.3] = ord("T")
        s1, s2 = a.tobytes(), b.tobytes()
        W = 64
        G = min((L + W - 1) // W, max_groups)
        want = ref.run_align(s1, s2, W, G)
        assert gpu_ctx.compat(s1, s2, wg=W, max_groups=max_groups) == want
        assert oracle.compat_align(s1, s2, W, max_groups) == want
