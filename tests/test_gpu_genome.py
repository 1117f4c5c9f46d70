"""GPU parity of the host-batch data paths that feed the same kernels:

* reads against an HBM-resident genome (msw_genome_create + msw_align_reads):
  windows cut on the GPU from (position, length), clipped at the genome end;
* pinned caller arrays (msw_host_alloc) DMA'd directly, without staging;
* pageable arrays staged with rows repacked to 16-byte-rounded strides.

Every result is compared bit-exactly with the oracle run on windows cut on
the host with the same semantics.  Run with -m gpu."""
import os

import numpy as np
import pytest

import mini_parallel_amd as mpa
from mini_parallel_amd import Scoring
from mini_parallel_amd.aligner import pinned_empty
from mini_parallel_amd.synthetic import make_pairs

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)
ACGT = np.frombuffer(b"ACGT", np.uint8)
SCHEMES = [Scoring(), Scoring(want_coords=True),
           Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True)]


def oracle_run(oracle, reads, read_len, wins, win_len, sc):
    return oracle.sw_batch(reads, read_len, wins, win_len, match=sc.match, mismatch=sc.mismatch,
                           gap_open=sc.gap_open, gap_extend=sc.gap_extend, affine=sc.affine,
                           threads=THREADS)


def host_windows(genome: np.ndarray, pos: np.ndarray, want: np.ndarray):
    """The documented window semantics (msw.h msw_read_batch_t), on the host."""
    glen = genome.size
    eff = np.where((pos < 0) | (pos >= glen), 0, np.minimum(want.astype(np.int64), glen - pos))
    ws = max(16, (int(eff.max()) + 15) // 16 * 16 if eff.size else 16)
    W = np.zeros((pos.size, ws), np.uint8)
    for k in range(pos.size):
        if eff[k]:
            W[k, :eff[k]] = genome[pos[k]:pos[k] + eff[k]]
    return W, eff.astype(np.uint16)


def assert_same(got, want, coords):
    s, i, j = got
    ws, wi, wj = want
    bad = np.nonzero(s != ws)[0]
    assert bad.size == 0, f"{bad.size} score mismatches at {bad[:5]}: gpu {s[bad[:5]]} oracle {ws[bad[:5]]}"
    if coords:
        bad = np.nonzero((i != wi) | (j != wj))[0]
        assert bad.size == 0, f"{bad.size} coordinate mismatches at {bad[:5]}"


def genome_case(n_pairs, glen, seed, read_stride=160):
    """Reads sampled from a genome (with substitutions), positions around the
    read (window = 2 x read length, centred), plus edge positions: negative,
    past the end, the last base, windows running off the end, zero lengths."""
    rng = np.random.default_rng(seed)
    g = rng.choice(ACGT, glen)
    rl = rng.integers(1, min(256, read_stride) + 1, n_pairs).astype(np.uint16)
    rl[: n_pairs // 2] = np.minimum(150, read_stride)
    want = np.minimum(2 * rl.astype(np.int64), 4096).astype(np.uint16)
    pos = rng.integers(0, glen, n_pairs).astype(np.int64)
    R = np.zeros((n_pairs, read_stride), np.uint8)
    for k in range(n_pairs):
        m = int(rl[k])
        src = int(min(max(pos[k] + (int(want[k]) - m) // 2, 0), max(glen - m, 0)))
        r = g[src:src + m].copy()
        if r.size < m:
            r = np.concatenate([r, rng.choice(ACGT, m - r.size)])
        sub = rng.random(m) < 0.02
        r[sub] = rng.choice(ACGT, int(sub.sum()))
        R[k, :m] = r
    edge = [-5, -1, glen, glen + 100, glen - 1, glen - 7, glen - 150, 0]
    for k, p in enumerate(edge):
        if k < n_pairs:
            pos[k] = p
    if n_pairs > 10:
        want[9] = 0
        want[10] = 1
    return g, R, rl, pos, want


@pytest.mark.parametrize("sc", SCHEMES, ids=["linear", "linear_coords", "affine_coords"])
@pytest.mark.parametrize("chunk", [0, 777])
def test_genome_windows_match_host_cut(gpu_ctx, oracle, sc, chunk):
    g, R, rl, pos, want = genome_case(6000, 1_000_003, seed=5)
    genome = gpu_ctx.load_genome(g)
    assert len(genome) == g.size
    got = gpu_ctx.align_reads(genome, R, rl, pos, want, sc, chunk_pairs=chunk)
    W, wl = host_windows(g, pos, want)
    assert_same(got, oracle_run(oracle, R, rl, W, wl, sc), sc.want_coords)
    assert got[0][0] == 0 and got[0][2] == 0  # negative / past-the-end positions
    genome.close()


def test_genome_tiny_and_unaligned(gpu_ctx, oracle):
    """Genomes of 1..37 bases (lengths not a multiple of 4: the cut kernel's
    dword over-read must stay in the padded allocation), every start position,
    window lengths up to past the end, odd read stride (byte path)."""
    rng = np.random.default_rng(11)
    sc = Scoring(want_coords=True)
    for glen in (1, 2, 3, 5, 16, 17, 37):
        g = rng.choice(ACGT, glen)
        genome = gpu_ctx.load_genome(g.tobytes())
        pos = np.repeat(np.arange(-1, glen + 1, dtype=np.int64), 3)
        want = np.tile(np.array([1, glen, glen + 9], np.uint16), glen + 2)
        n = pos.size
        R = np.zeros((n, 21), np.uint8)
        rl = rng.integers(0, 22, n).astype(np.uint16)
        for k in range(n):
            R[k, :rl[k]] = rng.choice(ACGT, int(rl[k]))
        got = gpu_ctx.align_reads(genome, R, rl, pos, want, sc)
        W, wl = host_windows(g, pos, want)
        assert_same(got, oracle_run(oracle, R, rl, W, wl, sc), True)
        genome.close()


def test_genome_with_other_bytes(gpu_ctx, oracle):
    """A genome holding N and lower-case runs: waves whose windows hold any
    byte outside A/C/G/T stage integer codes (the byte-load path for genome
    windows), the rest take the f16 path; every window start alignment."""
    rng = np.random.default_rng(13)
    g = rng.choice(ACGT, 200_003)
    for a in range(0, g.size, 5000):
        g[a:a + 40] = ord("N")
    g[1000:1100] = np.frombuffer(b"acgt" * 25, np.uint8)
    n = 3000
    pos = np.concatenate([np.arange(980, 980 + 64), rng.integers(0, g.size, n - 64)]).astype(np.int64)
    rl = np.full(n, 150, np.uint16)  # one bucket: the chunk reads its windows from the genome
    want = np.full(n, 300, np.uint16)
    R = np.zeros((n, 160), np.uint8)
    for k in range(n):
        src = int(min(pos[k] + 75, g.size - int(rl[k])))
        R[k, :rl[k]] = g[src:src + int(rl[k])]
    genome = gpu_ctx.load_genome(g)
    W, wl = host_windows(g, pos, want)
    for sc in SCHEMES:
        got = gpu_ctx.align_reads(genome, R, rl, pos, want, sc)
        assert_same(got, oracle_run(oracle, R, rl, W, wl, sc), sc.want_coords)
    genome.close()


@pytest.mark.parametrize("sc", SCHEMES, ids=["linear", "linear_coords", "affine_coords"])
@pytest.mark.parametrize("n,chunk", [(10_000, 0), (9_000, 2_500), (37, 0)])
def test_genome_uniform_chunks(fresh_ctx, oracle, sc, n, chunk, monkeypatch, capfd):
    """Chunks of one length bucket (150 bp reads, 289..300-byte windows: the
    config-2 shape from the genome) -- the chunks the scoring kernels score
    with windows read straight from the genome: every window start residue
    mod 16, windows clipped a few bytes short at the genome end, reads with
    N; async calls as bench.py streams them.  MSW_HOST_TRACE shows the path
    (the library reads it when the context is made: fresh_ctx)."""
    monkeypatch.setenv("MSW_HOST_TRACE", "1")
    rng = np.random.default_rng(n + chunk)
    g = rng.choice(ACGT, 3_000_017)
    pos = rng.integers(0, g.size - 300, n).astype(np.int64)
    pos[:16] = 1000 + np.arange(16)
    pos[16:20] = g.size - np.array([300, 297, 292, 289])
    rl = np.full(n, 150, np.uint16)
    want = np.full(n, 300, np.uint16)
    R = np.zeros((n, 160), np.uint8)
    for k in range(n):
        R[k, :150] = g[pos[k] + 70:pos[k] + 220] if pos[k] + 220 <= g.size else rng.choice(ACGT, 150)
    R[5, 40:44] = ord("N")
    genome = fresh_ctx.load_genome(g)
    W, wl = host_windows(g, pos, want)
    expect = oracle_run(oracle, R, rl, W, wl, sc)
    capfd.readouterr()
    assert_same(fresh_ctx.align_reads(genome, R, rl, pos, want, sc, chunk_pairs=chunk), expect, sc.want_coords)
    trace = [ln for ln in capfd.readouterr().err.splitlines() if ln.startswith("[msw host]")]
    chunks = int(trace[-1].split("chunks=")[1].split()[0])
    genome_chunks = int(trace[-1].split("genome_chunks=")[1].split()[0])
    direct_out = int(trace[-1].split("direct(")[1].split("out=")[1].split(")")[0])
    # one-chunk calls: the kernels store into the slot's mapped block; more
    # chunks copy their results back
    assert direct_out == (0 if chunks > 1 else 1), trace[-1]
    if n == 10_000:  # the config-2 shape: one chunk, pairs layout (smaller chunks may take the split layout)
        assert genome_chunks == chunks == 1, trace[-1]
    pend = [fresh_ctx.align_reads(genome, R, rl, pos, want, sc, chunk_pairs=chunk, asynchronous=True)
            for _ in range(3)]
    for p in pend[::-1]:
        assert_same(p.wait(), expect, sc.want_coords)
    genome.close()


@pytest.mark.parametrize("window", [0, 300, 97])
def test_align_reads_device(gpu_ctx, oracle, window):
    """msw_align_reads_device (the --full-wgs GPU reader's call): reads and
    positions in HBM, windows of `window` bytes (0: twice the read length)
    clipped at the genome end, their lengths written back; scores and best
    cells against the host restatement."""
    import ctypes

    import torch
    from mini_parallel_amd._lib import OutT, check, lib
    g, R, rl, pos, _ = genome_case(7000, 900_007, seed=83)
    want = (np.minimum(2 * rl.astype(np.int64), 4096) if window == 0 else np.full(rl.size, window)).astype(np.uint16)
    genome = gpu_ctx.load_genome(g)
    dev = torch.device("cuda", 0)
    d_reads = torch.from_numpy(R).to(dev)
    d_rl = torch.from_numpy(rl.view(np.int16)).to(dev)
    d_pos = torch.from_numpy(pos).to(dev)
    n = pos.size
    score = torch.full((n,), -7, dtype=torch.int32, device=dev)
    ei = torch.zeros(n, dtype=torch.int16, device=dev)
    ej = torch.zeros(n, dtype=torch.int16, device=dev)
    wlen = torch.full((n,), -1, dtype=torch.int16, device=dev)
    W, wl = host_windows(g, pos, want)
    for sc in SCHEMES:
        out = OutT(score.data_ptr(), ei.data_ptr(), ej.data_ptr())
        check(lib().msw_align_reads_device(gpu_ctx.handle, ctypes.byref(sc.to_c()), genome.handle,
                                           d_reads.data_ptr(), d_rl.data_ptr(), R.shape[1], d_pos.data_ptr(), n,
                                           window, int(rl.max()), ctypes.byref(out), wlen.data_ptr(), None))
        gpu_ctx.synchronize()
        assert np.array_equal(wlen.cpu().numpy().view(np.uint16), wl)
        got = (score.cpu().numpy(), ei.cpu().numpy(), ej.cpu().numpy())
        assert_same(got, oracle_run(oracle, R, rl, W, wl, sc), sc.want_coords)
    genome.close()


def test_genome_mixed_lengths_bucketed(fresh_ctx, oracle, monkeypatch, capfd):
    """Config 5 shape through the genome path (length-bucketed launch): a
    chunk of several buckets cuts its windows into a slab first (no chunk
    reads the genome directly; MSW_HOST_TRACE shows it), and equals the
    oracle."""
    g, R, rl, pos, want = genome_case(8000, 2_000_000, seed=21, read_stride=256)
    rl[:] = np.random.default_rng(3).integers(75, 251, rl.size)
    want[:] = 2 * rl
    monkeypatch.setenv("MSW_HOST_TRACE", "1")
    genome = fresh_ctx.load_genome(g)
    for sc in SCHEMES[1:]:
        capfd.readouterr()
        got = fresh_ctx.align_reads(genome, R, rl, pos, want, sc)
        line = [ln for ln in capfd.readouterr().err.splitlines() if ln.startswith("[msw host]")][-1]
        assert int(line.split("genome_chunks=")[1].split()[0]) == 0, line
        W, wl = host_windows(g, pos, want)
        assert_same(got, oracle_run(oracle, R, rl, W, wl, sc), True)


def test_genome_errors(gpu_ctx):
    g = gpu_ctx.load_genome(b"ACGT" * 10)
    R = np.zeros((2, 16), np.uint8)
    with pytest.raises(mpa.MswError):  # read longer than its stride
        gpu_ctx.align_reads(g, R, np.array([20, 1], np.uint16), np.zeros(2, np.int64),
                            np.array([4, 4], np.uint16))
    other = mpa.Context(0)
    with pytest.raises(mpa.MswError, match="another context"):
        other.align_reads(g, R, np.array([4, 1], np.uint16), np.zeros(2, np.int64),
                          np.array([4, 4], np.uint16))
    other.close()
    s, _, _ = gpu_ctx.align_reads(g, R[:0], np.zeros(0, np.uint16), np.zeros(0, np.int64),
                                  np.zeros(0, np.uint16))
    assert s.size == 0


@pytest.mark.parametrize("sc", SCHEMES[1:], ids=["linear_coords", "affine_coords"])
def test_pinned_direct_and_staged_agree(fresh_ctx, oracle, monkeypatch, capfd, sc):
    """Pinned arrays are DMA'd from the caller's memory, pageable ones are
    staged (MSW_HOST_TRACE shows which); one chunk and several.  All
    bit-exact."""
    b = make_pairs(9000, 150, 2.0, seed=77, read_stride=160, win_stride=304)
    want = oracle_run(oracle, b.reads, b.read_len, b.wins, b.win_len, sc)
    pr = pinned_empty(b.reads.shape, np.uint8)
    pw = pinned_empty(b.wins.shape, np.uint8)
    prl = pinned_empty(b.read_len.shape, np.uint16)
    pwl = pinned_empty(b.win_len.shape, np.uint16)
    pr[:], pw[:], prl[:], pwl[:] = b.reads, b.wins, b.read_len, b.win_len
    monkeypatch.setenv("MSW_HOST_TRACE", "1")
    for arrs, direct in (((pr, prl, pw, pwl), 1), ((b.reads, b.read_len, b.wins, b.win_len), 0)):
        for chunk in (0, 2500):
            capfd.readouterr()
            assert_same(fresh_ctx.align_batch(*arrs, sc, chunk_pairs=chunk), want, True)
            line = [ln for ln in capfd.readouterr().err.splitlines() if ln.startswith("[msw host]")][-1]
            assert f"direct(reads={direct} wins={direct}" in line, line


def test_wide_strides_repacked(gpu_ctx, oracle):
    """Pageable batches with padded strides (256 / 600) are repacked to
    16-byte-rounded rows during staging; odd strides take the byte-load
    staging path in the kernel: same results."""
    base = make_pairs(5000, (60, 150), 2.0, seed=99, read_stride=160, win_stride=304)
    sc = Scoring(want_coords=True)
    want = oracle_run(oracle, base.reads, base.read_len, base.wins, base.win_len, sc)
    rm, wm = int(base.read_len.max()), int(base.win_len.max())
    for rs, ws in ((256, 600), (rm | 1, wm | 1), (rm, wm), (160, 304)):
        R = np.zeros((base.n_pairs, rs), np.uint8)
        W = np.zeros((base.n_pairs, ws), np.uint8)
        R[:, :rm] = base.reads[:, :rm]
        W[:, :wm] = base.wins[:, :wm]
        assert_same(gpu_ctx.align_batch(R, base.read_len, W, base.win_len, sc, chunk_pairs=1999), want, True)


def test_pinned_genome_reads(gpu_ctx, oracle):
    """Genome path with pinned reads / positions (direct DMA)."""
    g, R, rl, pos, want = genome_case(4000, 500_009, seed=41)
    genome = gpu_ctx.load_genome(g)
    pR = pinned_empty(R.shape, np.uint8)
    prl = pinned_empty(rl.shape, np.uint16)
    ppos = pinned_empty(pos.shape, np.int64)
    pwant = pinned_empty(want.shape, np.uint16)
    pR[:], prl[:], ppos[:], pwant[:] = R, rl, pos, want
    sc = Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True)
    got = gpu_ctx.align_reads(genome, pR, prl, ppos, pwant, sc, chunk_pairs=1500)
    W, wl = host_windows(g, pos, want)
    assert_same(got, oracle_run(oracle, R, rl, W, wl, sc), True)


def test_async_calls_in_flight(gpu_ctx, oracle):
    """Several msw_*_async calls in flight on one context (slots alternate
    across calls), waited in and out of order: every result bit-exact."""
    g, R, rl, pos, want = genome_case(3000, 400_000, seed=61)
    genome = gpu_ctx.load_genome(g)
    sc = Scoring(want_coords=True)
    W, wl = host_windows(g, pos, want)
    expect = oracle_run(oracle, R, rl, W, wl, sc)
    parts = [slice(0, 1000), slice(1000, 1700), slice(1700, 3000)]
    pend = [gpu_ctx.align_reads(genome, R[p], rl[p], pos[p], want[p], sc, chunk_pairs=c, asynchronous=True)
            for p, c in zip(parts, (0, 300, 512))]
    pend.append(gpu_ctx.align_batch(R, rl, W, wl, sc, asynchronous=True))
    got = [None] * 4
    for k in (2, 0, 3, 1):  # waiting on a later ticket completes the earlier ones
        got[k] = pend[k].wait()
    for p, r in zip(parts, got[:3]):
        assert_same(r, tuple(e[p] for e in expect), True)
    assert_same(got[3], expect, True)


def test_genome_cut_device_matches_host_cut(gpu_ctx, oracle):
    """msw_genome_cut_device on device arrays: the same windows and clipped
    lengths as the host restatement, then scored through the device API."""
    import torch
    g, R, rl, pos, want = genome_case(5000, 700_001, seed=71)
    want[20] = 400  # clipped at the slab stride (320)
    genome = gpu_ctx.load_genome(g)
    dev = torch.device("cuda", 0)
    ws = 320
    d_pos = torch.from_numpy(pos).to(dev)
    d_want = torch.from_numpy(want.view(np.int16)).to(dev)
    d_wins = torch.full((pos.size, ws), 0xAB, dtype=torch.uint8, device=dev)
    d_len = torch.zeros(pos.size, dtype=torch.int16, device=dev)
    genome.cut_device(d_pos.data_ptr(), d_want.data_ptr(), pos.size, d_wins.data_ptr(), ws, d_len.data_ptr())
    torch.cuda.synchronize()
    W, wl = host_windows(g, pos, np.minimum(want, ws).astype(np.uint16))
    got_len = d_len.cpu().numpy().view(np.uint16)
    assert np.array_equal(got_len, wl)
    got = d_wins.cpu().numpy()
    assert np.array_equal(got[:, :W.shape[1]], W) and not got[:, W.shape[1]:].any()
    sc = Scoring(want_coords=True)
    d_reads = torch.from_numpy(R).to(dev)
    d_rl = torch.from_numpy(rl.view(np.int16)).to(dev)
    score = torch.zeros(pos.size, dtype=torch.int32, device=dev)
    ei = torch.zeros(pos.size, dtype=torch.int16, device=dev)
    ej = torch.zeros(pos.size, dtype=torch.int16, device=dev)
    gpu_ctx.align_batch_device(d_reads.data_ptr(), d_rl.data_ptr(), d_wins.data_ptr(), d_len.data_ptr(),
                               R.shape[1], ws, pos.size, score.data_ptr(), int(rl.max()), ws, sc,
                               ei.data_ptr(), ej.data_ptr())
    gpu_ctx.synchronize()
    assert_same((score.cpu().numpy(), ei.cpu().numpy(), ej.cpu().numpy()),
                oracle_run(oracle, R, rl, W, wl, sc), True)


def test_error_paths(gpu_ctx):
    """Range / argument errors of the new entry points fail loudly, before any
    launch, with a message (the Err(String) analogue)."""
    import ctypes
    from mini_parallel_amd._lib import lib
    g = gpu_ctx.load_genome(b"ACGT" * 100)
    R = np.zeros((2, 16), np.uint8)
    with pytest.raises(mpa.MswError, match="window length"):  # requested window > 32767
        gpu_ctx.align_reads(g, R, np.array([4, 4], np.uint16), np.zeros(2, np.int64),
                            np.array([32768, 4], np.uint16))
    with pytest.raises(mpa.MswError, match="unknown ticket"):
        from mini_parallel_amd._lib import check
        check(lib().msw_wait(gpu_ctx.handle, ctypes.c_uint64(10 ** 12)))
    with pytest.raises(mpa.MswError, match="NULL array"):
        g.cut_device(0, 0, 1, 0, 32)
    with pytest.raises(mpa.MswError, match="multiple of 16"):  # validated before anything is touched
        g.cut_device(16, 16, 1, 16, 30)
    p = gpu_ctx.align_reads(g, R, np.array([4, 4], np.uint16), np.zeros(2, np.int64),
                            np.array([4, 4], np.uint16), asynchronous=True)
    assert list(p.wait()[0]) == [0, 0]  # zero reads vs ACGT: nothing matches byte 0


def test_async_stream_upload_forms(gpu_ctx, oracle):
    """A stream of one-chunk async calls (the host-to-host stream of bench.py,
    three in flight, results waited oldest first and newest first; uploads on
    the copy stream behind an event) between synchronous one-chunk calls
    (uploads on the compute stream); every batch equals the oracle."""
    rng = np.random.default_rng(17)
    g = rng.choice(ACGT, 1_000_003)
    n = 3_000
    pos = rng.integers(0, g.size - 300, n).astype(np.int64)
    rl = np.full(n, 150, np.uint16)
    want = np.full(n, 300, np.uint16)
    R = np.zeros((n, 160), np.uint8)
    for k in range(n):
        R[k, :150] = g[pos[k] + 70:pos[k] + 220]
    genome = gpu_ctx.load_genome(g)
    W, wl = host_windows(g, pos, want)
    sc = SCHEMES[1]
    expect = oracle_run(oracle, R, rl, W, wl, sc)
    pend = []
    for k in range(9):
        pend.append(gpu_ctx.align_reads(genome, R, rl, pos, want, sc, asynchronous=True))
        if len(pend) == 3:
            assert_same(pend.pop(0).wait(), expect, sc.want_coords)
    for p in pend[::-1]:
        assert_same(p.wait(), expect, sc.want_coords)
    pend = []
    for k in range(4):  # synchronous and async calls interleaved
        pend.append(gpu_ctx.align_reads(genome, R, rl, pos, want, sc, asynchronous=True))
        assert_same(gpu_ctx.align_reads(genome, R, rl, pos, want, sc), expect, sc.want_coords)
    for p in pend:
        assert_same(p.wait(), expect, sc.want_coords)
    genome.close()


@pytest.mark.parametrize("form", ["pairs_pinned", "pairs_pageable", "pairs_misaligned", "genome_pinned"])
def test_one_chunk_calls_distinct_batches(gpu_ctx, oracle, form):
    """One-chunk calls pull their rows and metadata from pinned host memory
    with a copy kernel on their compute stream (no DMA, no event): a stream
    of async calls over DIFFERENT batches, three in flight, so every staging
    slot is reused with new data every third call -- pinned arrays read in
    place, pageable ones staged, pinned rows at an odd address (the DMA form
    on the call's stream), and reads against a genome.  Every batch must
    equal the oracle (a stale line of an earlier batch would not)."""
    sc = SCHEMES[1]
    batches = [make_pairs(1500 + 7 * k, (120, 160), 2.0, seed=400 + k, read_stride=160, win_stride=336)
               for k in range(7)]

    def pinned(a, shift=0):
        buf = pinned_empty(a.nbytes + shift, np.uint8)
        v = buf[shift:shift + a.nbytes].view(a.dtype).reshape(a.shape)
        v[...] = a
        return v
    genome = None
    if form == "genome_pinned":
        rng = np.random.default_rng(9)
        g = rng.choice(ACGT, 2_000_000)
        genome = gpu_ctx.load_genome(g)
    calls = []
    for k, b in enumerate(batches):
        if form == "genome_pinned":
            rng = np.random.default_rng(k)
            pos = rng.integers(0, 2_000_000 - 400, b.n_pairs).astype(np.int64)
            want = (2 * b.read_len).astype(np.uint16)
            W, wl = host_windows(g, pos, want)
            expect = oracle_run(oracle, b.reads, b.read_len, W, wl, sc)
            args = (pinned(b.reads), pinned(b.read_len), pinned(pos), pinned(want))
            calls.append((lambda a=args: gpu_ctx.align_reads(genome, *a, scoring=sc, asynchronous=True), expect))
        else:
            expect = oracle_run(oracle, b.reads, b.read_len, b.wins, b.win_len, sc)
            if form == "pairs_pageable":
                args = (b.reads, b.read_len, b.wins, b.win_len)
            else:
                sh = 1 if form == "pairs_misaligned" else 0
                args = (pinned(b.reads, sh), pinned(b.read_len), pinned(b.wins, sh), pinned(b.win_len))
            calls.append((lambda a=args: gpu_ctx.align_batch(*a, sc, asynchronous=True), expect))
    pend = []
    for rnd in range(2):  # the same batches again: slots hold other batches' data by then
        for fn, expect in calls:
            pend.append((fn(), expect))
            if len(pend) == 3:
                p, e = pend.pop(0)
                assert_same(p.wait(), e, True)
    for p, e in pend:
        assert_same(p.wait(), e, True)
    if genome is not None:
        genome.close()
