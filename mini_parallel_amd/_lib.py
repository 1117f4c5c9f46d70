"""ctypes binding of the in-tree C ABI library ``libmsw.so`` (include/msw.h).

There is no CPU fallback: if the HIP library is missing or no GPU is present,
every call raises :class:`MswError` (the reference likewise refuses to run
without ``--gpu``, main.rs:160-163).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MSW_LIB_PATH lets A/B tooling (tools/sweep.py) load another in-tree build.
LIB_PATH = os.environ.get("MSW_LIB_PATH") or os.path.join(_HERE, "libmsw.so")

MSW_OK = 0
MSW_E_INVALID = -1
MSW_E_RANGE = -2
MSW_E_DEVICE = -3
MSW_E_NODEVICE = -4
MSW_E_NOMEM = -5

# Every symbol include/msw.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "msw_device_count", "msw_device_info", "msw_ctx_create", "msw_ctx_create_ex", "msw_ctx_destroy",
    "msw_align_batch", "msw_align_batch_async", "msw_wait", "msw_align_batch_device",
    "msw_align_compat", "msw_host_alloc", "msw_host_free", "msw_dev_alloc", "msw_dev_free",
    "msw_memcpy_h2d", "msw_memcpy_d2h", "msw_synchronize", "msw_last_error", "msw_version",
    "msw_plan_create", "msw_align_batch_planned", "msw_plan_destroy",
    "msw_genome_create", "msw_genome_destroy", "msw_genome_length", "msw_align_reads",
    "msw_align_reads_async", "msw_genome_cut_device", "msw_ctx_stats", "msw_align_reads_device",
    "msw_memcpy_d2h_async", "msw_fence_record", "msw_fence_wait", "msw_ctx_prepare",
    "msw_stream_create", "msw_stream_destroy",
)
# include/msw_fastq.h
FASTQ_EXPORTED = ("msw_fastq_open", "msw_fastq_close", "msw_fastq_next", "msw_fastq_next_packed",
                  "msw_fastq_stats", "msw_fastq_count_bases", "msw_is_bgzf", "msw_gfastq_open",
                  "msw_gfastq_next", "msw_gfastq_stats", "msw_gfastq_close", "msw_bgzf_inflate",
                  "msw_gfastq_reset", "msw_gfastq_prefetch")


class MswError(RuntimeError):
    """A failing msw_* call; mirrors the reference's ``Err(String)``."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


class ScoringT(ctypes.Structure):
    _fields_ = [("match", ctypes.c_int32), ("mismatch", ctypes.c_int32),
                ("gap_open", ctypes.c_int32), ("gap_extend", ctypes.c_int32),
                ("affine", ctypes.c_int32), ("want_coords", ctypes.c_int32)]


class BatchT(ctypes.Structure):
    _fields_ = [("reads", ctypes.c_void_p), ("wins", ctypes.c_void_p),
                ("read_len", ctypes.c_void_p), ("win_len", ctypes.c_void_p),
                ("read_stride", ctypes.c_uint32), ("win_stride", ctypes.c_uint32),
                ("n_pairs", ctypes.c_uint64)]


class ReadBatchT(ctypes.Structure):
    _fields_ = [("reads", ctypes.c_void_p), ("read_len", ctypes.c_void_p),
                ("read_stride", ctypes.c_uint32), ("win_pos", ctypes.c_void_p),
                ("win_len", ctypes.c_void_p), ("n_pairs", ctypes.c_uint64)]


class OutT(ctypes.Structure):
    _fields_ = [("score", ctypes.c_void_p), ("end_i", ctypes.c_void_p),
                ("end_j", ctypes.c_void_p)]


class DevReadsT(ctypes.Structure):
    _fields_ = [("reads", ctypes.c_void_p), ("read_len", ctypes.c_void_p), ("pos", ctypes.c_void_p),
                ("read_stride", ctypes.c_uint32), ("n", ctypes.c_uint64), ("first_read", ctypes.c_uint64),
                ("min_len", ctypes.c_uint32), ("max_len", ctypes.c_uint32)]


class DeviceInfoT(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 256), ("mem_bytes", ctypes.c_uint64),
                ("mem_free_bytes", ctypes.c_uint64), ("max_wg", ctypes.c_uint32),
                ("cu_count", ctypes.c_uint32), ("arch", ctypes.c_char * 64)]


class StatsT(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("launches", ctypes.c_uint64), ("pairs", ctypes.c_uint64),
                ("cells", ctypes.c_uint64), ("alg_bytes", ctypes.c_uint64)]


_lib = None


def _declare(L):
    P = ctypes.c_void_p
    I = ctypes.c_int
    sigs = {
        "msw_device_count": (I, [ctypes.POINTER(I)]),
        "msw_device_info": (I, [I, ctypes.POINTER(DeviceInfoT)]),
        "msw_ctx_create": (I, [I, ctypes.POINTER(P)]),
        "msw_ctx_create_ex": (I, [I, ctypes.c_uint, ctypes.POINTER(P)]),
        "msw_ctx_destroy": (None, [P]),
        "msw_align_batch": (I, [P, ctypes.POINTER(ScoringT), ctypes.POINTER(BatchT),
                                ctypes.POINTER(OutT), ctypes.c_uint64]),
        "msw_align_batch_async": (I, [P, ctypes.POINTER(ScoringT), ctypes.POINTER(BatchT),
                                      ctypes.POINTER(OutT), ctypes.c_uint64,
                                      ctypes.POINTER(ctypes.c_uint64)]),
        "msw_wait": (I, [P, ctypes.c_uint64]),
        "msw_align_batch_device": (I, [P, ctypes.POINTER(ScoringT), ctypes.POINTER(BatchT),
                                       ctypes.POINTER(OutT), ctypes.c_uint32, ctypes.c_uint32, P]),
        "msw_plan_create": (I, [P, ctypes.POINTER(ScoringT), P, P, ctypes.c_uint64, ctypes.POINTER(P)]),
        "msw_align_batch_planned": (I, [P, P, ctypes.POINTER(BatchT), ctypes.POINTER(OutT), P]),
        "msw_plan_destroy": (None, [P]),
        "msw_genome_create": (I, [P, P, ctypes.c_uint64, ctypes.POINTER(P)]),
        "msw_genome_destroy": (None, [P]),
        "msw_genome_length": (ctypes.c_uint64, [P]),
        "msw_genome_cut_device": (I, [P, P, P, P, ctypes.c_uint64, P, ctypes.c_uint32, P, P]),
        "msw_align_reads": (I, [P, ctypes.POINTER(ScoringT), P, ctypes.POINTER(ReadBatchT),
                                ctypes.POINTER(OutT), ctypes.c_uint64]),
        "msw_align_reads_async": (I, [P, ctypes.POINTER(ScoringT), P, ctypes.POINTER(ReadBatchT),
                                      ctypes.POINTER(OutT), ctypes.c_uint64,
                                      ctypes.POINTER(ctypes.c_uint64)]),
        "msw_align_reads_device": (I, [P, ctypes.POINTER(ScoringT), P, P, P, ctypes.c_uint32, P, ctypes.c_uint64,
                                       ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(OutT), P, P]),
        "msw_align_compat": (I, [P, P, ctypes.c_size_t, P, ctypes.c_size_t, ctypes.c_uint32,
                                 ctypes.c_uint32, ctypes.POINTER(ctypes.c_int32)]),
        "msw_host_alloc": (P, [ctypes.c_size_t]),
        "msw_host_free": (None, [P]),
        "msw_dev_alloc": (P, [P, ctypes.c_size_t]),
        "msw_dev_free": (None, [P, P]),
        "msw_memcpy_h2d": (I, [P, P, ctypes.c_size_t]),
        "msw_memcpy_d2h": (I, [P, P, ctypes.c_size_t]),
        "msw_memcpy_d2h_async": (I, [P, P, P, ctypes.c_size_t, P]),
        "msw_fence_record": (I, [P, P, ctypes.POINTER(ctypes.c_uint64)]),
        "msw_fence_wait": (I, [P, ctypes.c_uint64]),
        "msw_stream_create": (I, [P, ctypes.POINTER(P)]),
        "msw_stream_destroy": (I, [P, P]),
        "msw_synchronize": (I, [P]),
        "msw_ctx_stats": (I, [P, ctypes.POINTER(StatsT), I]),
        "msw_ctx_prepare": (I, [P, ctypes.POINTER(ScoringT)]),
        "msw_last_error": (ctypes.c_char_p, []),
        "msw_version": (ctypes.c_char_p, []),
        "msw_fastq_open": (I, [ctypes.c_char_p, ctypes.POINTER(P)]),
        "msw_fastq_close": (None, [P]),
        "msw_fastq_next": (I, [P, P, P, ctypes.c_uint32, ctypes.c_uint64,
                               ctypes.POINTER(ctypes.c_uint64), P]),
        "msw_fastq_next_packed": (I, [P, P, ctypes.c_uint64, P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
        "msw_fastq_stats": (None, [P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                   ctypes.POINTER(ctypes.c_uint64)]),
        "msw_fastq_count_bases": (I, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_uint64)]),
        "msw_is_bgzf": (I, [ctypes.c_char_p]),
        "msw_gfastq_open": (I, [P, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64, I, ctypes.c_uint64,
                                ctypes.POINTER(P)]),
        "msw_gfastq_next": (I, [P, P, ctypes.POINTER(DevReadsT)]),
        "msw_gfastq_stats": (None, [P] + [ctypes.POINTER(ctypes.c_uint64)] * 6),
        "msw_gfastq_close": (None, [P]),
        "msw_gfastq_reset": (I, [P, ctypes.c_char_p]),
        "msw_gfastq_prefetch": (I, [P, ctypes.c_char_p]),
        "msw_bgzf_inflate": (I, [P, P, ctypes.c_uint64, P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args


def lib():
    """Load libmsw.so (raises MswError if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MswError(MSW_E_NODEVICE,
                           f"{LIB_PATH} is not built: run `make -C mini_parallel_amd/csrc` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        _declare(L)
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != MSW_OK:
        msg = lib().msw_last_error()
        raise MswError(rc, msg.decode() if msg else f"msw error {rc}")
