"""ctypes binding of oracle/_ref/libref_cl.so: the REFERENCE's own OpenCL
kernel (smith_waterman.cl, compiled for gfx950 by `make -C oracle ref`) run
on the GPU with the reference host geometry of gpu_align (aligner.rs:410-532).

TEST INFRASTRUCTURE ONLY (tests/ import it as the checker)."""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
CO = os.path.join(_HERE, "_ref", "smith_waterman_gfx950.co")
SO = os.path.join(_HERE, "_ref", "libref_cl.so")
_lib = None


def available() -> bool:
    return os.path.exists(CO) and os.path.exists(SO)


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(SO)
        L.ref_cl_run.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_uint32,
                                 ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                 ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p, ctypes.c_size_t]
        L.ref_cl_run.restype = ctypes.c_int
        _lib = L
    return _lib


def run_align(s1: bytes, s2: bytes, wg: int, groups: int) -> int:
    """smith_waterman_align(seq1, seq2, result, min(len)) over NDRange
    (groups * wg, wg); result starts at 0."""
    res = ctypes.c_int32(0)
    err = ctypes.create_string_buffer(256)
    rc = lib().ref_cl_run(CO.encode(), 0, s1, len(s1), s2, len(s2), wg, groups, ctypes.byref(res), err, 256)
    if rc != 0:
        raise RuntimeError(err.value.decode())
    return int(res.value)


def gpu_align_geometry(L: int, max_wg: int = 1024, max_groups: int = 1_000_000):
    """aligner.rs:422-424: W = min(max_wg, 1024), G = min(ceil(L / W), max_groups)."""
    W = min(max_wg, 1024)
    return W, min((L + W - 1) // W, max_groups)
