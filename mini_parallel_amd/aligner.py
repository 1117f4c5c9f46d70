"""Host-side mirror of the reference's align/score API over the C ABI.

Reference interface (smith_waterman/src/), same names, argument meaning and
error behaviour (errors raise :class:`MswError`, the ``Err(String)`` analogue):

  gpu.rs:9-10        GPU_WORK_GROUP_SIZE, GPU_MAX_WORK_GROUPS
  gpu.rs:17-30       GpuDevice, GpuAlignmentResult
  gpu.rs:33-94       is_gpu_available, get_gpu_devices
  gpu.rs:97-109      get_opencl_context  -> get_context (one Context per GPU)
  aligner.rs:9-15    get_chunk_size_reads
  aligner.rs:365-373 gpu_align_chunk_self
  aligner.rs:410-532 gpu_align            (legacy kernel semantics, K0)

New batched API (north_star): ``Context.align_batch`` (host arrays, pinned
async staging) and ``Context.align_batch_device`` (HBM-resident batches), both
calling the hand-written gfx950 kernels through include/msw.h.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from ._lib import (MSW_E_INVALID, BatchT, DeviceInfoT, MswError, OutT, ReadBatchT, ScoringT, StatsT,
                   check, lib)

GPU_WORK_GROUP_SIZE = 1024          # gpu.rs:9
GPU_MAX_WORK_GROUPS = 1_000_000     # gpu.rs:10


@dataclass
class GpuDevice:
    """gpu.rs:17-22, plus the HIP ordinal / CU count / arch."""
    name: str
    memory_gb: float
    max_work_group_size: int
    ordinal: int = 0
    cu_count: int = 0
    arch: str = ""


@dataclass
class GpuAlignmentResult:
    """gpu.rs:25-30."""
    score: int
    processing_time_ms: float
    gpu_device: str


@dataclass(frozen=True)
class Scoring:
    """Scoring scheme (include/msw.h msw_scoring_t).

    Reference constants: match +2, mismatch -1, linear gap 2
    (smith_waterman.cl:5-7).  Affine: a gap of length k costs
    gap_open + k * gap_extend."""
    match: int = 2
    mismatch: int = -1
    gap_open: int = 0
    gap_extend: int = 2
    affine: bool = False
    want_coords: bool = False

    def to_c(self) -> ScoringT:
        return ScoringT(self.match, self.mismatch, self.gap_open, self.gap_extend,
                        1 if self.affine else 0, 1 if self.want_coords else 0)


LINEAR = Scoring()                                             # config 2
LINEAR_COORDS = Scoring(want_coords=True)
AFFINE = Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True)   # config 3


def is_gpu_available() -> bool:
    """gpu.rs:33-45."""
    try:
        n = ctypes.c_int(0)
        return lib().msw_device_count(ctypes.byref(n)) == 0 and n.value > 0
    except MswError:
        return False


def get_gpu_devices() -> list:
    """gpu.rs:48-94 (memory from hipMemGetInfo instead of nvidia-smi)."""
    n = ctypes.c_int(0)
    check(lib().msw_device_count(ctypes.byref(n)))
    out = []
    for i in range(n.value):
        info = DeviceInfoT()
        check(lib().msw_device_info(i, ctypes.byref(info)))
        out.append(GpuDevice(name=info.name.decode(), memory_gb=info.mem_bytes / 2**30,
                             max_work_group_size=int(info.max_wg), ordinal=i,
                             cu_count=int(info.cu_count), arch=info.arch.decode()))
    return out


_PTRS: dict = {}


def _ptr(a) -> int:
    """Data address of a numpy array.  ``a.ctypes.data`` costs ~2 us a call
    (a ctypes view object per call), a sizeable share of a 10k-pair async
    call, so the address is remembered per live array: keyed on id(), checked
    by a weak reference and the shape (an in-place resize changes the shape),
    dropped when the array is freed."""
    if a is None:
        return 0
    k = id(a)
    e = _PTRS.get(k)
    if e is not None and e[0]() is a and e[2] == a.shape:
        return e[1]
    p = a.ctypes.data
    try:
        _PTRS[k] = (weakref.ref(a, lambda _r, k=k: _PTRS.pop(k, None)), p, a.shape)
    except TypeError:  # not weak-referenceable: no caching
        pass
    return p


_SCORING_C: dict = {}


def _scoring_c(scoring: "Scoring"):
    """The C struct of a (frozen, hashable) Scoring, built once."""
    c = _SCORING_C.get(scoring)
    if c is None:
        c = _SCORING_C[scoring] = scoring.to_c()
    return c


def _outputs(n: int, coords: bool):
    """Result arrays of an n-pair call in ONE allocation (score int32, then
    end_i / end_j int16 when coords): one address lookup instead of three.
    Every element is written by the library before the call returns (or
    before wait()), so the buffer is not zeroed."""
    if not coords:
        score = np.empty(n, np.int32)
        return (score, None, None), OutT(_fresh_ptr(score), 0, 0)
    buf = np.empty(8 * n, np.uint8)
    base = _fresh_ptr(buf)
    score, ei, ej = buf[:4 * n].view(np.int32), buf[4 * n:6 * n].view(np.int16), buf[6 * n:].view(np.int16)
    return (score, ei, ej), OutT(base, base + 4 * n, base + 6 * n)


def _fresh_ptr(a) -> int:
    """Address of a just-allocated (writable, contiguous) array: through the
    buffer protocol, ~3x cheaper than a.ctypes.data."""
    return ctypes.addressof(ctypes.c_char.from_buffer(a)) if a.size else 0


class Context:
    """One GPU: compute + copy streams and double-buffered pinned staging
    (replaces the (Context, Queue, Device) singleton of gpu.rs:13-14)."""

    def __init__(self, ordinal: int = 0):
        self.ordinal = ordinal
        h = ctypes.c_void_p()
        check(lib().msw_ctx_create(ordinal, ctypes.byref(h)))
        self._h = h

    @property
    def handle(self) -> ctypes.c_void_p:
        if self._h is None:
            raise MswError(MSW_E_INVALID, "context is closed")
        return self._h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            lib().msw_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- batched scoring from host memory --------------------------------------------
    def align_batch(self, reads: np.ndarray, read_len: np.ndarray, wins: np.ndarray,
                    win_len: np.ndarray, scoring: Scoring = LINEAR, chunk_pairs: int = 0,
                    asynchronous: bool = False):
        """Score a padded SoA batch (uint8 [B, stride] reads / windows, uint16
        lengths).  Returns (score int32[B], end_i int16[B], end_j int16[B]);
        the coordinates are None unless ``scoring.want_coords``.  With
        ``asynchronous`` (msw_align_batch_async) it returns a :class:`Pending`
        whose ``wait()`` gives the same tuple."""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        wins = np.ascontiguousarray(wins, dtype=np.uint8)
        read_len = np.ascontiguousarray(read_len, dtype=np.uint16)
        win_len = np.ascontiguousarray(win_len, dtype=np.uint16)
        B = reads.shape[0]
        if wins.shape[0] != B or read_len.shape[0] != B or win_len.shape[0] != B:
            raise MswError(MSW_E_INVALID, "batch arrays disagree on the number of pairs")
        (score, ei, ej), out = _outputs(B, scoring.want_coords)
        batch = BatchT(_ptr(reads), _ptr(wins), _ptr(read_len), _ptr(win_len),
                       reads.shape[1] if reads.ndim == 2 else 0,
                       wins.shape[1] if wins.ndim == 2 else 0, B)
        sc = _scoring_c(scoring)
        if asynchronous:
            t = ctypes.c_uint64(0)
            check(lib().msw_align_batch_async(self.handle, ctypes.byref(sc), ctypes.byref(batch),
                                              ctypes.byref(out), chunk_pairs, ctypes.byref(t)))
            return Pending(self, t.value, (score, ei, ej), (reads, wins, read_len, win_len))
        check(lib().msw_align_batch(self.handle, ctypes.byref(sc), ctypes.byref(batch),
                                    ctypes.byref(out), chunk_pairs))
        return score, ei, ej

    # -- reads against an HBM-resident genome ------------------------------------------
    def load_genome(self, seq) -> "Genome":
        """Upload a reference genome (bytes / str / uint8 array) once; windows
        are then cut on the GPU (msw_genome_create)."""
        return Genome(self, seq)

    def align_reads(self, genome: "Genome", reads: np.ndarray, read_len: np.ndarray,
                    win_pos: np.ndarray, win_len: np.ndarray, scoring: Scoring = LINEAR,
                    chunk_pairs: int = 0, asynchronous: bool = False):
        """Score read p against genome[win_pos[p] : win_pos[p] + win_len[p]]
        (clipped at the genome end; positions outside it score 0).  Returns
        (score, end_i, end_j) like :meth:`align_batch` (a :class:`Pending`
        with ``asynchronous``, msw_align_reads_async)."""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        read_len = np.ascontiguousarray(read_len, dtype=np.uint16)
        win_pos = np.ascontiguousarray(win_pos, dtype=np.int64)
        win_len = np.ascontiguousarray(win_len, dtype=np.uint16)
        B = reads.shape[0]
        if read_len.shape[0] != B or win_pos.shape[0] != B or win_len.shape[0] != B:
            raise MswError(MSW_E_INVALID, "batch arrays disagree on the number of pairs")
        (score, ei, ej), out = _outputs(B, scoring.want_coords)
        batch = ReadBatchT(_ptr(reads), _ptr(read_len), reads.shape[1] if reads.ndim == 2 else 0,
                           _ptr(win_pos), _ptr(win_len), B)
        sc = _scoring_c(scoring)
        if asynchronous:
            t = ctypes.c_uint64(0)
            check(lib().msw_align_reads_async(self.handle, ctypes.byref(sc), genome.handle,
                                              ctypes.byref(batch), ctypes.byref(out), chunk_pairs,
                                              ctypes.byref(t)))
            return Pending(self, t.value, (score, ei, ej), (reads, read_len, win_pos, win_len, genome))
        check(lib().msw_align_reads(self.handle, ctypes.byref(sc), genome.handle, ctypes.byref(batch),
                                    ctypes.byref(out), chunk_pairs))
        return score, ei, ej

    # -- HBM-resident batches ----------------------------------------------------------
    def align_batch_device(self, reads_ptr: int, read_len_ptr: int, wins_ptr: int,
                           win_len_ptr: int, read_stride: int, win_stride: int, n_pairs: int,
                           score_ptr: int, max_read_len: int, max_win_len: int,
                           scoring: Scoring = LINEAR, end_i_ptr: int = 0, end_j_ptr: int = 0,
                           stream: int = 0) -> None:
        """Enqueue one scoring pass over device-resident arrays (raw device
        pointers) on ``stream`` (a hipStream_t handle, 0 = context stream)."""
        batch = BatchT(reads_ptr, wins_ptr, read_len_ptr, win_len_ptr, read_stride, win_stride,
                       n_pairs)
        out = OutT(score_ptr, end_i_ptr, end_j_ptr)
        sc = scoring.to_c()
        check(lib().msw_align_batch_device(self.handle, ctypes.byref(sc), ctypes.byref(batch),
                                           ctypes.byref(out), max_read_len, max_win_len,
                                           ctypes.c_void_p(stream or None)))

    def prepare_device_launch(self, reads_ptr: int, read_len_ptr: int, wins_ptr: int,
                              win_len_ptr: int, read_stride: int, win_stride: int, n_pairs: int,
                              score_ptr: int, max_read_len: int, max_win_len: int,
                              scoring: Scoring = LINEAR, end_i_ptr: int = 0, end_j_ptr: int = 0,
                              stream: int = 0):
        """Bind the arguments of align_batch_device once; returns a zero-argument
        callable that enqueues one pass (keeps per-launch host cost minimal)."""
        batch = BatchT(reads_ptr, wins_ptr, read_len_ptr, win_len_ptr, read_stride, win_stride,
                       n_pairs)
        out = OutT(score_ptr, end_i_ptr, end_j_ptr)
        sc = scoring.to_c()
        fn = lib().msw_align_batch_device
        args = (self.handle, ctypes.byref(sc), ctypes.byref(batch), ctypes.byref(out),
                max_read_len, max_win_len, ctypes.c_void_p(stream or None))
        keep = (batch, out, sc)

        def launch() -> None:
            _ = keep
            rc = fn(*args)
            if rc:
                check(rc)
        return launch

    def prepare_planned_launch(self, reads_ptr: int, read_len_ptr: int, wins_ptr: int,
                               win_len_ptr: int, read_stride: int, win_stride: int,
                               read_len, win_len, score_ptr: int, scoring: Scoring = LINEAR,
                               end_i_ptr: int = 0, end_j_ptr: int = 0, stream: int = 0):
        """Mixed-length device batch: build the length-bucketed plan once from the
        host length arrays (msw_plan_create), return a zero-argument callable that
        enqueues one single-launch pass (msw_align_batch_planned).  The plan is
        freed with the callable's ``close()``."""
        rl = np.ascontiguousarray(read_len, dtype=np.uint16)
        wl = np.ascontiguousarray(win_len, dtype=np.uint16)
        if rl.shape != wl.shape:
            raise ValueError("read_len / win_len shapes differ")
        sc = scoring.to_c()
        plan = ctypes.c_void_p()
        check(lib().msw_plan_create(self.handle, ctypes.byref(sc), rl.ctypes.data, wl.ctypes.data,
                                    rl.size, ctypes.byref(plan)))
        batch = BatchT(reads_ptr, wins_ptr, read_len_ptr, win_len_ptr, read_stride, win_stride, rl.size)
        out = OutT(score_ptr, end_i_ptr, end_j_ptr)
        fn = lib().msw_align_batch_planned
        args = (self.handle, plan, ctypes.byref(batch), ctypes.byref(out), ctypes.c_void_p(stream or None))
        keep = (batch, out, sc)

        class _Launch:
            def __call__(self_inner) -> None:
                _ = keep
                rc = fn(*args)
                if rc:
                    check(rc)

            def close(self_inner) -> None:
                if plan.value:
                    lib().msw_plan_destroy(plan)
                    plan.value = None

            def __del__(self_inner):
                try:
                    self_inner.close()
                except Exception:
                    pass
        return _Launch()

    def prepare(self, scoring: Scoring = LINEAR) -> None:
        """msw_ctx_prepare: load every scoring kernel module this scheme may
        use now (HIP loads a module at its first launch), so a short timed
        run does not pay for it."""
        check(lib().msw_ctx_prepare(self.handle, ctypes.byref(_scoring_c(scoring))))

    def synchronize(self) -> None:
        check(lib().msw_synchronize(self.handle))

    def stats(self, reset: bool = False) -> dict:
        """msw_ctx_stats: kernel time, launches, pairs, cells and algorithmic
        bytes of this context's host-batch calls (since creation / last reset)."""
        st = StatsT()
        check(lib().msw_ctx_stats(self.handle, ctypes.byref(st), 1 if reset else 0))
        return {"kernel_ms": st.kernel_ms, "launches": st.launches, "pairs": st.pairs, "cells": st.cells,
                "alg_bytes": st.alg_bytes}

    # -- legacy kernel ------------------------------------------------------------------
    def compat(self, s1: bytes, s2: bytes, wg: int = 0, max_groups: int = 0) -> int:
        """smith_waterman_align semantics (see gpu_align)."""
        res = ctypes.c_int32(0)
        b1 = ctypes.create_string_buffer(s1, len(s1)) if s1 else None
        b2 = ctypes.create_string_buffer(s2, len(s2)) if s2 else None
        check(lib().msw_align_compat(self.handle, b1, len(s1), b2, len(s2), wg, max_groups,
                                     ctypes.byref(res)))
        return int(res.value)


class Pending:
    """An asynchronous call in flight (msw_*_async ticket).  The input and
    output arrays are held until ``wait()``; ``wait()`` returns (score, end_i,
    end_j).  Waiting on a ticket also completes every earlier one (msw_wait).
    A Pending dropped without ``wait()`` waits in its finaliser: the runtime's
    staging slots still point at its arrays until the ticket drains."""

    def __init__(self, ctx: "Context", ticket: int, outs, keep):
        self.ctx, self.ticket, self._outs, self._keep = ctx, ticket, outs, keep

    def wait(self):
        if self._keep is not None:
            check(lib().msw_wait(self.ctx.handle, self.ticket))
            self._keep = None
        return self._outs

    def __del__(self):
        try:
            if self._keep is not None and getattr(self.ctx, "_h", None) is not None:
                lib().msw_wait(self.ctx._h, self.ticket)
        except Exception:
            pass
        self._keep = None


class Genome:
    """A reference genome resident in HBM on one context (msw_genome_*)."""

    def __init__(self, ctx: Context, seq):
        if isinstance(seq, str):
            seq = seq.encode()
        a = np.ascontiguousarray(np.frombuffer(bytes(seq), np.uint8) if isinstance(seq, (bytes, bytearray))
                                 else seq, dtype=np.uint8)
        h = ctypes.c_void_p()
        check(lib().msw_genome_create(ctx.handle, _ptr(a) if a.size else None, a.size, ctypes.byref(h)))
        self._h = h
        self.ctx = ctx  # keeps the context alive for as long as the genome

    @property
    def handle(self) -> ctypes.c_void_p:
        if self._h is None:
            raise MswError(MSW_E_INVALID, "genome is closed")
        return self._h

    def __len__(self) -> int:
        return int(lib().msw_genome_length(self.handle))

    def cut_device(self, pos_ptr: int, win_len_ptr: int, n: int, wins_ptr: int, win_stride: int,
                   win_len_out_ptr: int = 0, stream: int = 0) -> None:
        """msw_genome_cut_device: cut n windows (device arrays of positions and
        requested lengths) into a device slab, clipped lengths to
        win_len_out; enqueued on ``stream`` (0 = the context's stream)."""
        check(lib().msw_genome_cut_device(self.ctx.handle, self.handle, ctypes.c_void_p(pos_ptr),
                                          ctypes.c_void_p(win_len_ptr), n, ctypes.c_void_p(wins_ptr),
                                          win_stride, ctypes.c_void_p(win_len_out_ptr or None),
                                          ctypes.c_void_p(stream or None)))

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            lib().msw_genome_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pinned_empty(shape, dtype) -> np.ndarray:
    """A numpy array in page-locked host memory (msw_host_alloc): batches held
    in such arrays are copied to the GPU directly, without staging.  The
    memory is freed when the array (and every view of it) is collected."""
    dt = np.dtype(dtype)
    n = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
    p = lib().msw_host_alloc(max(n, 1))
    if not p:
        check(-5)
    buf = (ctypes.c_uint8 * max(n, 1)).from_address(p)
    arr = np.frombuffer(buf, dtype=np.uint8, count=n).view(dt).reshape(shape)

    class _Owner:
        def __del__(self_inner):
            lib().msw_host_free(p)
    # numpy keeps `buf` alive through arr.base; hang the owner on the ctypes buffer
    buf._owner = _Owner()
    return arr


_contexts: dict = {}
_ctx_lock = threading.Lock()


def get_context(device=0) -> Context:
    """Process-wide context per GPU (gpu.rs:97-109 get_opencl_context)."""
    ordinal = device.ordinal if isinstance(device, GpuDevice) else int(device)
    with _ctx_lock:
        ctx = _contexts.get(ordinal)
        if ctx is None:
            ctx = _contexts[ordinal] = Context(ordinal)
        return ctx


def gpu_align(seq1: str, seq2: str, device: GpuDevice) -> int:
    """aligner.rs:410-532: the score of the kernel the reference launches
    (smith_waterman_align), with its host geometry W = min(max_wg, 1024),
    G = min(ceil(L/W), 1e6); L == 0 -> 0; oversize -> MswError."""
    b1 = seq1.encode() if isinstance(seq1, str) else bytes(seq1)
    b2 = seq2.encode() if isinstance(seq2, str) else bytes(seq2)
    wg = min(int(device.max_work_group_size), GPU_WORK_GROUP_SIZE)
    return get_context(device).compat(b1, b2, wg, GPU_MAX_WORK_GROUPS)


def gpu_align_chunk_self(chunk: str, device: GpuDevice) -> int:
    """aligner.rs:365-373: chunks under 1000 bases score 0, else self-align."""
    if len(chunk) < 1000:
        return 0
    return gpu_align(chunk, chunk, device)


def get_chunk_size_reads() -> int:
    """aligner.rs:9-15: GPU_CHUNK_SIZE_READS is mandatory."""
    v = os.environ.get("GPU_CHUNK_SIZE_READS")
    if v is None:
        raise MswError(MSW_E_INVALID, "GPU_CHUNK_SIZE_READS not set in .env file")
    try:
        n = int(v)
        if n < 0:
            raise ValueError(v)
        return n
    except ValueError as e:
        raise MswError(MSW_E_INVALID, f"Invalid GPU_CHUNK_SIZE_READS value '{v}': {e}") from None


def pack_batch(reads: Sequence[bytes], wins: Sequence[bytes], read_stride: Optional[int] = None,
               win_stride: Optional[int] = None):
    """Lists of byte strings -> padded SoA arrays (reads, read_len, wins, win_len)."""
    B = len(reads)
    if len(wins) != B:
        raise MswError(MSW_E_INVALID, "reads and windows differ in count")
    rl = np.array([len(r) for r in reads], np.uint16)
    wl = np.array([len(w) for w in wins], np.uint16)
    rs = read_stride or max(16, (int(rl.max()) if B else 0) + 15) // 16 * 16
    ws = win_stride or max(16, (int(wl.max()) if B else 0) + 15) // 16 * 16
    R = np.zeros((B, rs), np.uint8)
    W = np.zeros((B, ws), np.uint8)
    for i, (r, w) in enumerate(zip(reads, wins)):
        R[i, :len(r)] = np.frombuffer(bytes(r), np.uint8)
        W[i, :len(w)] = np.frombuffer(bytes(w), np.uint8)
    return R, rl, W, wl
