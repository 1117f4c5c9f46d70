"""Seeded synthetic short-read pairs (BASELINE.json configs).

A uniform i.i.d. ACGT genome; each read copies genome[p:p+m] with 1 %
substitutions, 0.1 % indels and 0.05 % 'N'; its window is the length-n
stretch of genome centred on the read; 10 % of reads are unrelated random
sequence (they exercise the zero floor).  Seed 1000 + k for config k.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

ACGT = np.frombuffer(b"ACGT", np.uint8)


@dataclass
class PairBatch:
    reads: np.ndarray      # uint8 [B, read_stride]
    read_len: np.ndarray   # uint16 [B]
    wins: np.ndarray       # uint8 [B, win_stride]
    win_len: np.ndarray    # uint16 [B]
    pos: np.ndarray        # int64 [B] genome offset of the window (-1: unrelated read)

    @property
    def n_pairs(self) -> int:
        return int(self.reads.shape[0])

    @property
    def cells(self) -> int:
        return int(np.sum(self.read_len.astype(np.int64) * self.win_len.astype(np.int64)))

    def slice(self, a: int, b: int) -> "PairBatch":
        return PairBatch(self.reads[a:b], self.read_len[a:b], self.wins[a:b], self.win_len[a:b],
                         self.pos[a:b])


def genome(n_bases: int, rng: np.random.Generator) -> np.ndarray:
    return ACGT[rng.integers(0, 4, n_bases, dtype=np.uint8)]


def _rows(g: np.ndarray, start: np.ndarray, width: int) -> np.ndarray:
    """rows[i] = g[start[i] : start[i] + width], indices past the end clamped
    to the last base (g[min(start + c, len - 1)]), as a u8 copy: a gather
    through a sliding-window view of g padded with its last base, instead of
    an int64 index array of n x width entries."""
    n = int(start.shape[0])
    if n == 0 or width == 0:
        return np.zeros((n, width), np.uint8)
    pad = np.full(width, g[-1], np.uint8)
    view = np.lib.stride_tricks.sliding_window_view(np.concatenate([g, pad]), width)
    return view[np.asarray(start, np.int64)]


def make_pairs(n_pairs: int, read_len, win_factor: float = 2.0, seed: int = 1002,
               genome_bases: int = 1 << 22, unrelated: float = 0.10, read_stride: int = 0,
               win_stride: int = 0, sub: float = 0.01, indel: float = 0.001,
               nrate: float = 0.0005, genome_arr: np.ndarray | None = None) -> PairBatch:
    """``read_len`` is an int (fixed length) or an (lo, hi) range for mixed
    lengths (config 5); window length = round(win_factor * read length).
    Vectorised over pairs; only reads that draw an indel take a Python loop.
    ``genome_arr`` supplies the genome (else one of ``genome_bases`` is drawn);
    ``pos`` is then always the window's genome offset, -1 marking unrelated
    reads only through the returned ``pos`` sign convention below."""
    rng = np.random.default_rng(seed)
    g = genome(genome_bases, rng) if genome_arr is None else genome_arr
    genome_bases = int(g.shape[0])
    if isinstance(read_len, (tuple, list)):
        lens = rng.integers(read_len[0], read_len[1] + 1, n_pairs)
    else:
        lens = np.full(n_pairs, int(read_len), np.int64)
    wlens = np.round(lens * win_factor).astype(np.int64)
    max_m = int(lens.max()) if n_pairs else 0
    max_n = int(wlens.max()) if n_pairs else 0
    rs = read_stride or max(16, (max_m + 15) // 16 * 16)
    ws = win_stride or max(16, (max_n + 15) // 16 * 16)
    assert rs >= max_m and ws >= max_n, "stride smaller than the longest sequence"
    pos = rng.integers(0, genome_bases - max(max_n, 1), n_pairs)
    cols_w = np.arange(ws)
    wins = _rows(g, pos, ws)
    wins[cols_w[None, :] >= wlens[:, None]] = 0
    # read = genome[off : off + m], centred in the window
    off = pos + (wlens - lens) // 2
    cols_r = np.arange(rs)
    reads = _rows(g, off, rs)
    valid = cols_r[None, :] < lens[:, None]
    subs = (rng.random(reads.shape) < sub) & valid
    idx = np.searchsorted(ACGT, reads[subs])
    reads[subs] = ACGT[(idx + rng.integers(1, 4, idx.shape[0])) % 4]
    reads[(rng.random(reads.shape) < nrate) & valid] = ord("N")
    unrel = rng.random(n_pairs) < unrelated
    reads[unrel] = ACGT[rng.integers(0, 4, (int(unrel.sum()), rs), dtype=np.uint8)]
    reads[~valid] = 0
    rl = lens.copy()
    n_indel = rng.binomial(lens, indel)
    for k in np.nonzero((n_indel > 0) & ~unrel)[0]:
        r = reads[k, :rl[k]]
        for _ in range(int(n_indel[k])):
            at = int(rng.integers(0, max(1, r.shape[0])))
            if rng.random() < 0.5 and r.shape[0] > 1:
                r = np.delete(r, at)
            else:
                r = np.insert(r, at, ACGT[int(rng.integers(0, 4))])
        r = r[:rs]
        reads[k, :] = 0
        reads[k, :r.shape[0]] = r
        rl[k] = r.shape[0]
    pos = np.where(unrel, -1, pos)
    return PairBatch(np.ascontiguousarray(reads), rl.astype(np.uint16),
                     np.ascontiguousarray(wins), wlens.astype(np.uint16), pos)


def config_batch(k: int, n_pairs: int = 0, seed_offset: int = 0) -> PairBatch:
    """Batches for BASELINE.json configs (k = 1..5); n_pairs overrides the size."""
    seed = 1000 + k + seed_offset
    if k == 1:
        return make_pairs(n_pairs or 1, 32, win_factor=1.0, seed=seed, unrelated=0.0)
    if k in (2, 3, 4):
        default = {2: 10_000, 3: 1_000_000, 4: 1_000_000}[k]
        return make_pairs(n_pairs or default, 150, 2.0, seed=seed, read_stride=160, win_stride=304)
    if k == 5:
        return make_pairs(n_pairs or 100_000, (75, 250), 2.0, seed=seed, read_stride=256,
                          win_stride=512)
    raise ValueError(f"unknown config {k}")


SHARD_BLOCK = 1024  # pairs per independently seeded block of a global batch


def _config_shape(k: int):
    """(read length spec, win_factor, read_stride, win_stride) of config k."""
    if k in (2, 3, 4):
        return 150, 2.0, 160, 304
    if k == 5:
        return (75, 250), 2.0, 256, 512
    raise ValueError(f"no sharded form for config {k}")


def config_block(k: int, blk: int, genome_arr: np.ndarray | None = None) -> PairBatch:
    """Block ``blk`` (pairs [blk * SHARD_BLOCK, (blk + 1) * SHARD_BLOCK)) of
    config k's global batch.  Its content depends only on (k, blk): the genome
    comes from seed 1000 + k, the pairs from seed [1000 + k, blk]."""
    seed = 1000 + k
    g = config_genome(k) if genome_arr is None else genome_arr
    rl, wf, rs, ws = _config_shape(k)
    return make_pairs(SHARD_BLOCK, rl, wf, seed=[seed, blk], genome_arr=g, read_stride=rs, win_stride=ws)


_GENOMES: dict = {}


def config_genome(k: int, n_bases: int = 1 << 22) -> np.ndarray:
    """The shared genome of config k's global batch (cached per process)."""
    if k not in _GENOMES:
        _GENOMES[k] = genome(n_bases, np.random.default_rng(1000 + k))
    return _GENOMES[k]


def config_shard(k: int, a: int, b: int) -> PairBatch:
    """Pairs [a, b) of config k's GLOBAL seeded batch (bench.py's multi-GPU
    form): pair i is the same whichever rank generates it and however many
    ranks share the batch, so rank r scores ``shard_range(B, r, N)`` of one
    batch and the gathered scores can be checked pair by pair."""
    if b <= a:
        rl, wf, rs, ws = _config_shape(k)
        z = np.zeros((0,), np.uint16)
        return PairBatch(np.zeros((0, rs), np.uint8), z, np.zeros((0, ws), np.uint8), z.copy(),
                         np.zeros((0,), np.int64))
    g = config_genome(k)
    first, last = a // SHARD_BLOCK, (b - 1) // SHARD_BLOCK
    parts = [config_block(k, blk, g) for blk in range(first, last + 1)]
    lo = a - first * SHARD_BLOCK
    hi = lo + (b - a)
    cat = lambda f: np.ascontiguousarray(np.concatenate([f(p) for p in parts])[lo:hi])  # noqa: E731
    return PairBatch(cat(lambda p: p.reads), cat(lambda p: p.read_len), cat(lambda p: p.wins),
                     cat(lambda p: p.win_len), cat(lambda p: p.pos))


BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def bgzf_compress(data: bytes, level: int = 1, strategy: int = 0, block: int = 0xFF00,
                  eof_block: bool = True) -> bytes:
    """BGZF (bgzip's block gzip): a multi-member gzip of <= 64 KiB blocks whose
    'BC' extra field holds the block size, then the empty EOF block.  Any gzip
    reader (zcat, the reference's lane loader) reads it as one stream; the C++
    reader inflates it block by block with libdeflate, the GPU lane reader
    with msw_inflate.hip.  ``strategy`` is zlib's (Z_FIXED, Z_RLE, ...)."""
    import struct
    import zlib
    out = []
    for k in range(0, len(data), block):
        chunk = data[k:k + block]
        c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
        cdata = c.compress(chunk) + c.flush()
        out.append(struct.pack("<4BIBBH2BHH", 0x1F, 0x8B, 8, 4, 0, 0, 0xFF, 6, ord("B"), ord("C"), 2,
                               len(cdata) + 25))
        out.append(cdata)
        out.append(struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
    if eof_block:
        out.append(BGZF_EOF)
    return b"".join(out)


def _lane_reads(g, k, reads_per_file, read_len, win_factor, seed, segment=0):
    """The reads of lane file k of a write_wgs_dataset run and their window
    positions (every read gets a window of the genome: unrelated reads, pos
    -1 in make_pairs, are paired with a random window), plus the rng the
    writer continues with for the quality strings.  ``segment`` > 0: the
    segment-th run of reads of a file written in segments
    (write_lane_file_segmented; segment 0 is the unsegmented file)."""
    genome_bases = int(g.shape[0])
    b = make_pairs(reads_per_file, read_len, win_factor, seed=seed * 1000 + k + 1_000_003 * segment, genome_arr=g,
                   read_stride=(read_len + 16 + 15) // 16 * 16)
    rng = np.random.default_rng([seed, k] if segment == 0 else [seed, k, segment])
    span = genome_bases - int(b.win_len.max())
    pos = np.where(b.pos >= 0, np.minimum(b.pos, span), rng.integers(0, span, b.n_pairs))
    return b, pos, rng


def _with_windows(g, b, pos) -> PairBatch:
    cols = np.arange(b.wins.shape[1])
    wins = _rows(g, pos, b.wins.shape[1])
    wins[cols[None, :] >= b.win_len[:, None].astype(np.int64)] = 0
    return PairBatch(b.reads, b.read_len.copy(), wins, b.win_len.copy(), pos)


def wgs_genome(seed: int = 1004, genome_bases: int = 1 << 20) -> np.ndarray:
    """The genome write_wgs_dataset writes as reference.fa for this seed."""
    return genome(genome_bases, np.random.default_rng(seed))


def lane_file_batch(k: int, reads_per_file: int, read_len: int = 150, win_factor: float = 2.0,
                    seed: int = 1004, genome_bases: int = 1 << 20, genome_arr: np.ndarray | None = None) -> PairBatch:
    """Lane file k (0-based, lane-major: L001_R1, L001_R2, L002_R1, ...) of a
    write_wgs_dataset run with these parameters, regenerated without writing
    it: its reads (file order) paired with their genome windows -- what the
    oracle scores to check the --full-wgs per-file sums."""
    g = wgs_genome(seed, genome_bases) if genome_arr is None else genome_arr
    b, pos, _ = _lane_reads(g, k, reads_per_file, read_len, win_factor, seed)
    return _with_windows(g, b, pos)


def _lane_records(b, pos, rng, tag: bytes, lane: int, qual: str, first: int = 0) -> bytes:
    """FASTQ text of one run of lane reads (read ids from ``first``)."""
    rl = b.read_len.astype(np.int64)
    if qual == "I":
        q = b"I" * int(rl.max() if b.n_pairs else 0)
        quals = [q[:rl[i]] for i in range(b.n_pairs)]
    else:
        # "binned": NovaSeq-style 4-level qualities; "illumina": 2..41 drifting
        # down the read with noise (HiSeq-style, much less compressible)
        tot = int(rl.sum())
        if qual == "binned":
            qb = rng.choice(np.frombuffer(b"F:,#", np.uint8), tot, p=[0.84, 0.11, 0.04, 0.01])
        else:
            cyc = np.concatenate([np.arange(int(m)) for m in rl]) if b.n_pairs else np.zeros(0, np.int64)
            qv = 40 - cyc // 12 + rng.integers(-6, 3, tot)
            qb = (np.clip(qv, 2, 41) + 33).astype(np.uint8)
        ends = np.cumsum(rl)
        raw = qb.tobytes()
        quals = [raw[int(e - m):int(e)] for e, m in zip(ends, rl)]
    return b"".join([b"@%s:%d:%d pos=%d\n%s\n+\n%s\n" % (tag, lane, first + i, int(pos[i]),
                                                          b.reads[i, :rl[i]].tobytes(), quals[i])
                     for i in range(b.n_pairs)])


def _write_lane_file(job):
    """One lane file of write_wgs_dataset (a process-pool job)."""
    import gzip
    (g, name, sample, lane, k, reads_per_file, read_len, win_factor, seed, compresslevel, keep, bgzf, qual) = job
    b, pos, rng = _lane_reads(g, k, reads_per_file, read_len, win_factor, seed)
    text = _lane_records(b, pos, rng, sample.encode(), lane, qual)
    if bgzf:
        with open(name, "wb") as f:
            f.write(bgzf_compress(text, compresslevel))
    else:
        with gzip.open(name, "wb", compresslevel=compresslevel) as f:
            f.write(text)
    if not keep:
        return None
    return _with_windows(g, b, pos)


def write_lane_file_segmented(job) -> int:
    """A BGZF lane file of ``reads_per_file`` reads written in segments of
    ``segment`` reads (bounded memory for full-size lane files: BASELINE
    config 4 is ~50 M reads per lane), each segment its own seeded run of
    reads, appended as whole BGZF members; the EOF block last.  Returns the
    file's size.  (A process-pool job: tools/c4_full.py.)"""
    (g, name, sample, lane, k, reads_per_file, segment, read_len, win_factor, seed, compresslevel, qual) = job
    done = 0
    with open(name, "wb") as f:
        for seg in range((reads_per_file + segment - 1) // segment):
            n = min(segment, reads_per_file - done)
            b, pos, rng = _lane_reads(g, k, n, read_len, win_factor, seed, segment=seg)
            f.write(bgzf_compress(_lane_records(b, pos, rng, sample.encode(), lane, qual, first=done), compresslevel,
                                  eof_block=False))
            done += n
        f.write(BGZF_EOF)
        return f.tell()


def write_wgs_dataset(out_dir: str, sample: str = "SYN", lanes: int = 2, reads_per_lane: int = 2,
                      reads_per_file: int = 1000, read_len: int = 150, win_factor: float = 2.0,
                      seed: int = 1004, genome_bases: int = 1 << 20, keep_batches: bool = True,
                      compresslevel: int = 1, workers: int = 1, bgzf: bool = False, qual: str = "I") -> dict:
    """Config-4-shaped dataset: lane files {sample}_L{lane:03}_R{r}_001.fastq.gz
    (aligner.rs:198-204 naming) whose headers carry "pos=<window start>", and
    the reference genome as reference.fa.  Returns paths and (keep_batches) the
    pair batches (reads, windows) so tests can score them with the oracle.
    Vectorised, and ``workers`` > 1 writes the lane files in parallel processes
    (same files either way).  ``bgzf`` writes block-gzip (bgzip) lane files;
    ``qual`` picks the quality strings: "I" (constant), "binned" (NovaSeq
    4-level) or "illumina" (Q2-Q41 drifting down the read, noisy)."""
    import os
    os.makedirs(out_dir, exist_ok=True)
    g = wgs_genome(seed, genome_bases)
    with open(os.path.join(out_dir, "reference.fa"), "w") as f:
        f.write(">synthetic seed=%d\n" % seed)
        s = g.tobytes().decode()
        f.write("\n".join(s[k:k + 80] for k in range(0, len(s), 80)) + "\n")
    jobs, files = [], []
    k = 0
    for lane in range(1, lanes + 1):
        for r in range(1, reads_per_lane + 1):
            name = os.path.join(out_dir, "%s_L%03d_R%d_001.fastq.gz" % (sample, lane, r))
            jobs.append((g, name, sample, lane, k, reads_per_file, read_len, win_factor, seed, compresslevel,
                         keep_batches, bgzf, qual))
            files.append(name)
            k += 1
    if workers > 1 and len(jobs) > 1:
        from multiprocessing import get_context
        with get_context("fork").Pool(min(workers, len(jobs))) as pool:
            res = pool.map(_write_lane_file, jobs)
    else:
        res = [_write_lane_file(j) for j in jobs]
    batches = [b for b in res if b is not None] if keep_batches else []
    return {"files": files, "reference": os.path.join(out_dir, "reference.fa"), "batches": batches,
            "sample": sample, "lanes": lanes, "reads_per_lane": reads_per_lane}
