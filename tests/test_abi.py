"""The C ABI library: builds, loads, exports every declared symbol, and fails
loudly (no CPU fallback) when no GPU is present.  CPU only."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import mini_parallel_amd as mpa
from mini_parallel_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "msw.h")
FASTQ_HEADER = os.path.join(ROOT, "include", "msw_fastq.h")


def declared_symbols(header=None):
    if header is None:
        return declared_symbols(HEADER) | declared_symbols(FASTQ_HEADER)
    text = open(header).read()
    return set(re.findall(r"\b(msw_[a-z0-9_]+)\s*\(", text)) - {"msw_ctx", "msw_fastq"}


def test_header_matches_binding():
    assert declared_symbols(HEADER) == set(_lib.EXPORTED)
    assert declared_symbols(FASTQ_HEADER) == set(_lib.FASTQ_EXPORTED)


def test_library_exports_every_symbol():
    assert os.path.exists(_lib.LIB_PATH), "libmsw.so not built (run __graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (msw_[a-z0-9_]+)$", out, re.M))
    missing = declared_symbols() - exported
    assert not missing, f"missing exports: {missing}"
    L = _lib.lib()
    for name in declared_symbols():
        assert getattr(L, name) is not None


def test_lib_path_override(tmp_path):
    """MSW_LIB_PATH (A/B tooling) loads the named build instead of the
    in-tree one; without it the in-tree library loads."""
    import shutil
    import sys
    alt = tmp_path / "libmsw_alt.so"
    shutil.copy(_lib.LIB_PATH, alt)
    code = ("import sys; sys.path.insert(0, sys.argv[1]); from mini_parallel_amd import _lib; L = _lib.lib(); "
            "print(_lib.LIB_PATH); print(L._name)")
    env = dict(os.environ, MSW_LIB_PATH=str(alt))
    out = subprocess.run([sys.executable, "-c", code, ROOT], env=env, capture_output=True, text=True, check=True)
    assert out.stdout.split() == [str(alt), str(alt)]
    env.pop("MSW_LIB_PATH")
    out = subprocess.run([sys.executable, "-c", code, ROOT], env=env, capture_output=True, text=True, check=True)
    assert out.stdout.split()[0] == os.path.join(ROOT, "mini_parallel_amd", "libmsw.so")


def test_library_targets_gfx950():
    """The fat binary embeds a gfx950 code object (and nothing else)."""
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data))
    assert targets == {b"gfx950"}, targets


def test_version_string():
    assert b"gfx950" in _lib.lib().msw_version()


def test_struct_layout():
    # msw_device_info_t: 256 + 8 + 8 + 4 + 4 + 64
    assert ctypes.sizeof(_lib.DeviceInfoT) == 344
    assert ctypes.sizeof(_lib.ScoringT) == 24
    assert ctypes.sizeof(_lib.BatchT) == 48
    assert ctypes.sizeof(_lib.OutT) == 24
    assert ctypes.sizeof(_lib.ReadBatchT) == 48


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU present")
def test_no_gpu_fails_loudly():
    assert not mpa.is_gpu_available()
    with pytest.raises(mpa.MswError):
        mpa.Context(0)
    with pytest.raises(mpa.MswError):
        mpa.get_gpu_devices()


def test_chunk_size_env(monkeypatch):
    monkeypatch.delenv("GPU_CHUNK_SIZE_READS", raising=False)
    with pytest.raises(mpa.MswError, match="not set"):
        mpa.get_chunk_size_reads()
    monkeypatch.setenv("GPU_CHUNK_SIZE_READS", "12x")
    with pytest.raises(mpa.MswError, match="Invalid"):
        mpa.get_chunk_size_reads()
    monkeypatch.setenv("GPU_CHUNK_SIZE_READS", "10000")
    assert mpa.get_chunk_size_reads() == 10000


def test_pack_batch():
    R, rl, W, wl = mpa.pack_batch([b"ACGT", b""], [b"TTACGTTT", b"A" * 40])
    assert R.shape == (2, 16) and W.shape == (2, 48)
    assert list(rl) == [4, 0] and list(wl) == [8, 40]
    assert bytes(R[0, :4]) == b"ACGT" and not R[1].any()


def _build_c_consumer(tmp_path):
    """Compile tests/c/abi_c99.c as strict C99 against include/ and link it to
    libmsw.so (the header must be plain C; every entry point must link)."""
    exe = str(tmp_path / "abi_c99")
    src = os.path.join(ROOT, "tests", "c", "abi_c99.c")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-I",
                    os.path.join(ROOT, "include"), src, "-o", exe, "-L", libdir, "-lmsw",
                    "-Wl,-rpath," + libdir], check=True)
    return exe


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU present (the gpu variant runs there)")
def test_c99_consumer_no_gpu(tmp_path):
    r = subprocess.run([_build_c_consumer(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_c99 ok (no gpu)" in r.stdout


@pytest.mark.gpu
def test_c99_consumer_gpu():
    """The prebuilt C99 consumer (__graft_entry__.build()) scores a known-answer
    pair through the C ABI on the GPU."""
    exe = os.path.join(ROOT, "tests", "c", "abi_c99")
    assert os.path.exists(exe), "tests/c/abi_c99 not built: run __graft_entry__.build()"
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_c99 ok (gpu)" in r.stdout
