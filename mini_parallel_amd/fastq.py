"""FASTQ(.gz) chunk loader over the C++ reader (include/msw_fastq.h).

Mirrors aligner.rs:107-178 (process_fastq_file_in_chunks) and :535-544
(count_bases_in_fastq): same record rules, same chunking, same error budget;
sequences land in padded SoA numpy slabs (pinned when ``pinned=True``), the
layout Context.align_batch consumes."""
from __future__ import annotations

import ctypes
from typing import Callable, Optional

import numpy as np

from ._lib import DevReadsT, MswError, check, lib


class FastqReader:
    """Streaming reader of one lane file."""

    def __init__(self, path: str):
        self.path = path
        h = ctypes.c_void_p()
        check(lib().msw_fastq_open(path.encode(), ctypes.byref(h)))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            lib().msw_fastq_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def next_chunk(self, max_reads: int, stride: int = 256, with_pos: bool = False):
        """Up to max_reads sequences -> (seqs u8[n, stride], lens u16[n][, pos i64[n]])."""
        seqs = np.zeros((max_reads, stride), np.uint8)
        lens = np.zeros(max_reads, np.uint16)
        pos = np.zeros(max_reads, np.int64) if with_pos else None
        n = ctypes.c_uint64(0)
        check(lib().msw_fastq_next(self._h, seqs.ctypes.data, lens.ctypes.data, stride, max_reads,
                                   ctypes.byref(n), pos.ctypes.data if pos is not None else None))
        k = n.value
        if with_pos:
            return seqs[:k], lens[:k], pos[:k]
        return seqs[:k], lens[:k]

    def next_packed(self, max_reads: int, cap: int):
        """msw_fastq_next_packed: up to max_reads sequences back to back in a
        buffer of cap bytes -> (buf u8[n_bytes], lens u32[n], need): ``need``
        is the length of the next sequence when it did not fit (0 at end of
        file or when max_reads were delivered)."""
        buf = np.zeros(max(cap, 1), np.uint8)
        lens = np.zeros(max(max_reads, 1), np.uint32)
        n, nb, need = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        check(lib().msw_fastq_next_packed(self._h, buf.ctypes.data, cap, lens.ctypes.data, max_reads,
                                          ctypes.byref(n), ctypes.byref(nb), ctypes.byref(need)))
        return buf[:nb.value], lens[:n.value], int(need.value)

    def next_concat(self, n_reads: int):
        """Exactly n_reads sequences (fewer at end of file) of any length,
        concatenated -- the chunk.concat() of aligner.rs:270 -- and their
        lengths; the buffer grows when a sequence does not fit."""
        parts, lens, got, cap = [], [], 0, max(1024, min(n_reads, 65536) * 160)
        while got < n_reads:
            buf, ln, need = self.next_packed(n_reads - got, cap)
            parts.append(buf)
            lens.append(ln)
            got += len(ln)
            if need:
                cap = max(2 * cap, need)
            elif got < n_reads:
                break
        cat = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
        return cat, (np.concatenate(lens) if lens else np.zeros(0, np.uint32))

    def stats(self) -> dict:
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        lib().msw_fastq_stats(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return {"lines": a.value, "reads": b.value, "errors": c.value}


class GpuFastqReader:
    """The GPU-side lane reader (msw_gfastq_*, BGZF files): inflate, CRC,
    line split and record parse run on the context's GPU; next_batch()
    returns the batch's device arrays (valid until the call after next) and,
    for tests, ``host=True`` copies them back.

    Streams: inflate and parse run on the reader's own stream, a blocking
    stream (ordered with the null stream, as a CU-masked HIP stream is).
    Work the caller puts on the null stream -- PyTorch's default stream,
    synchronous hipMemcpy -- therefore serialises with the reader; score on a
    stream of your own (torch.cuda.Stream) to overlap scoring with the next
    span's inflate."""

    def __init__(self, ctx, path: str, stride: int = 256, max_reads: int = 1 << 20, with_pos: bool = False,
                 span_bytes: int = 0):
        self.ctx, self.path, self.stride, self.with_pos = ctx, path, stride, with_pos
        h = ctypes.c_void_p()
        check(lib().msw_gfastq_open(ctx.handle, path.encode(), stride, max_reads, 1 if with_pos else 0,
                                    span_bytes, ctypes.byref(h)))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            lib().msw_gfastq_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, path: str) -> None:
        """msw_gfastq_reset: read another lane file with the same buffers."""
        self.path = path
        check(lib().msw_gfastq_reset(self._h, path.encode()))

    def prefetch(self, path: str) -> None:
        """msw_gfastq_prefetch: open the file the next reset() names ahead of time."""
        check(lib().msw_gfastq_prefetch(self._h, path.encode()))

    def next_batch(self, host: bool = True):
        """-> DevReadsT, or with host=True (seqs u8[n, stride], lens u16[n][, pos i64[n]])."""
        d = DevReadsT()
        check(lib().msw_gfastq_next(self._h, None, ctypes.byref(d)))
        self.last = d  # the batch's descriptor (n, first_read, min_len / max_len bounds)
        if not host:
            return d
        n = int(d.n)
        seqs = np.zeros((n, self.stride), np.uint8)
        lens = np.zeros(n, np.uint16)
        L = lib()
        check(L.msw_synchronize(self.ctx.handle))  # the emit ran on the context's compute stream
        if n:
            check(L.msw_memcpy_d2h(self.ctx.handle, seqs.ctypes.data, d.reads, seqs.nbytes))
            check(L.msw_memcpy_d2h(self.ctx.handle, lens.ctypes.data, d.read_len, lens.nbytes))
        if self.with_pos:
            pos = np.zeros(n, np.int64)
            if n:
                check(L.msw_memcpy_d2h(self.ctx.handle, pos.ctypes.data, d.pos, pos.nbytes))
            return seqs, lens, pos
        return seqs, lens

    def stats(self) -> dict:
        v = [ctypes.c_uint64() for _ in range(6)]
        lib().msw_gfastq_stats(self._h, *[ctypes.byref(x) for x in v])
        keys = ("lines", "reads", "errors", "bases", "bytes_in", "bytes_out")
        return {k: x.value for k, x in zip(keys, v)}


def bgzf_inflate(ctx, data: bytes) -> bytes:
    """msw_bgzf_inflate: a whole BGZF file inflated on the GPU (host to host)."""
    src = np.frombuffer(data, np.uint8)
    cap = 0
    # the trailers give the exact size: sum of ISIZE over the members
    p = 0
    while p + 18 <= len(data):
        bsize = data[p + 16] | (data[p + 17] << 8)
        cap += int.from_bytes(data[p + bsize + 1 - 4:p + bsize + 1], "little")
        p += bsize + 1
    out = np.zeros(max(cap, 1), np.uint8)
    n = ctypes.c_uint64()
    check(lib().msw_bgzf_inflate(ctx.handle, src.ctypes.data if len(src) else None, len(data), out.ctypes.data,
                                 cap, ctypes.byref(n)))
    return out[:n.value].tobytes()


def process_fastq_file_in_chunks(filepath: str, chunk_size_reads: int,
                                 processor: Callable[[list], Optional[object]]) -> None:
    """aligner.rs:107-178: call ``processor`` with lists of sequence strings
    (any length), full chunks of chunk_size_reads then one final partial
    chunk.  (For the GPU path use FastqReader.next_chunk, which fills SoA
    slabs directly, or next_concat for the compat driver's concatenation.)"""
    if chunk_size_reads <= 0:
        raise MswError(-1, "chunk_size_reads must be positive")
    with FastqReader(filepath) as fq:
        while True:
            cat, lens = fq.next_concat(chunk_size_reads)
            if len(lens) == 0:
                break
            ends = np.cumsum(lens.astype(np.int64))
            starts = ends - lens
            raw = cat.tobytes()
            processor([raw[a:b].decode() for a, b in zip(starts, ends)])


def count_bases_in_fastq(filepath: str) -> int:
    """aligner.rs:535-544."""
    bases, reads = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib().msw_fastq_count_bases(filepath.encode(), ctypes.byref(bases), ctypes.byref(reads)))
    return int(bases.value)
