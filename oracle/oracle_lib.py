"""ctypes binding of oracle/libsw_oracle.so (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module -- as the checker, never as the measured or shipped path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "libsw_oracle.so")
_lib = None


def build() -> str:
    """Compile the C restatement (gcc) in place."""
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_sw_batch.argtypes = [
            u8p, u8p, ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(ctypes.c_uint16),
            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
            ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int16),
            ctypes.POINTER(ctypes.c_int16), ctypes.c_int]
        L.oracle_sw_batch.restype = None
        L.oracle_sw_batch_simd.argtypes = L.oracle_sw_batch.argtypes
        L.oracle_sw_batch_simd.restype = ctypes.c_int
        L.oracle_simd_isa.argtypes = []
        L.oracle_simd_isa.restype = ctypes.c_int
        L.oracle_compat_align.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t,
                                          ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_compat_align.restype = ctypes.c_int32
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def sw_batch(reads, read_len, wins, win_len, match=2, mismatch=-1, gap_open=0,
             gap_extend=2, affine=False, threads=1):
    """Score a padded SoA batch with the C oracle -> (score, end_i, end_j)."""
    reads = np.ascontiguousarray(reads, dtype=np.uint8)
    wins = np.ascontiguousarray(wins, dtype=np.uint8)
    read_len = np.ascontiguousarray(read_len, dtype=np.uint16)
    win_len = np.ascontiguousarray(win_len, dtype=np.uint16)
    B = reads.shape[0]
    score = np.zeros(B, np.int32)
    ei = np.zeros(B, np.int16)
    ej = np.zeros(B, np.int16)
    if B:
        lib().oracle_sw_batch(_p(reads, ctypes.c_uint8), _p(wins, ctypes.c_uint8),
                              _p(read_len, ctypes.c_uint16), _p(win_len, ctypes.c_uint16),
                              reads.shape[1], wins.shape[1], B, match, mismatch, gap_open,
                              gap_extend, 1 if affine else 0, _p(score, ctypes.c_int32),
                              _p(ei, ctypes.c_int16), _p(ej, ctypes.c_int16), threads)
    return score, ei, ej


def sw_batch_simd(reads, read_len, wins, win_len, match=2, mismatch=-1, gap_open=0,
                  gap_extend=2, affine=False, threads=1, coords=True):
    """Same results as sw_batch, by the inter-sequence SIMD restatement
    (oracle/sw_simd.c; AVX-512BW / AVX2).  coords=False skips the best-cell
    tracking (end_i / end_j then stay 0).  Returns (score, end_i, end_j, isa_bits)."""
    reads = np.ascontiguousarray(reads, dtype=np.uint8)
    wins = np.ascontiguousarray(wins, dtype=np.uint8)
    read_len = np.ascontiguousarray(read_len, dtype=np.uint16)
    win_len = np.ascontiguousarray(win_len, dtype=np.uint16)
    B = reads.shape[0]
    score = np.zeros(B, np.int32)
    ei = np.zeros(B, np.int16)
    ej = np.zeros(B, np.int16)
    isa = simd_isa()
    if B:
        isa = lib().oracle_sw_batch_simd(_p(reads, ctypes.c_uint8), _p(wins, ctypes.c_uint8),
                                         _p(read_len, ctypes.c_uint16), _p(win_len, ctypes.c_uint16),
                                         reads.shape[1], wins.shape[1], B, match, mismatch, gap_open,
                                         gap_extend, 1 if affine else 0, _p(score, ctypes.c_int32),
                                         _p(ei, ctypes.c_int16) if coords else None,
                                         _p(ej, ctypes.c_int16) if coords else None, threads)
    return score, ei, ej, isa


def simd_isa() -> int:
    """Vector width (bits) the SIMD restatement uses on this CPU (512, 256 or 0)."""
    return int(lib().oracle_simd_isa())


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def compat_align(s1: bytes, s2: bytes, wg: int = 1024, max_groups: int = 0) -> int:
    a = np.frombuffer(s1, np.uint8) if s1 else np.zeros(1, np.uint8)
    b = np.frombuffer(s2, np.uint8) if s2 else np.zeros(1, np.uint8)
    return int(lib().oracle_compat_align(_p(a, ctypes.c_uint8), len(s1), _p(b, ctypes.c_uint8),
                                         len(s2), wg, max_groups))
