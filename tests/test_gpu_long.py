"""GPU parity of the long-pair path (msw_long.hip): reads > 256 bases or
windows > 4096, up to 32767 each, scored by sw_long_kernel (i32 cells, strips
of up to 512 rows with boundary rows in global scratch) and mixed with packed
buckets in one call.  Bit-exact against the oracle (oracle/sw_oracle.c, the
textbook recurrence of smith_waterman.cl:112-126 and Gotoh), scores and best
cells.  Run with -m gpu."""
import os

import numpy as np
import pytest

import mini_parallel_amd as mpa
from mini_parallel_amd import Scoring
from mini_parallel_amd.synthetic import make_pairs

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)
ACGT = np.frombuffer(b"ACGT", np.uint8)

KINDS = {
    "linear": dict(),
    "linear_coords": dict(want_coords=True),
    "affine": dict(affine=True, gap_open=3, gap_extend=1),
    "affine_coords": dict(affine=True, gap_open=3, gap_extend=1, want_coords=True),
}
# (match, mismatch, gap_open, gap_extend): the default, a steep affine-style
# scheme, and zero penalties (ties everywhere: the best-cell rule decides)
SCHEMES = [(2, -1, 0, 2), (5, -4, 10, 1), (1, 0, 0, 0)]


def scoring(kind, scheme=None):
    kw = dict(KINDS[kind])
    if scheme is not None:
        m, x, o, e = scheme
        kw.update(match=m, mismatch=x, gap_extend=e)
        if kw.get("affine"):
            kw["gap_open"] = o
    return Scoring(**kw)


def oracle_run(oracle, R, rl, W, wl, sc):
    return oracle.sw_batch(R, rl, W, wl, match=sc.match, mismatch=sc.mismatch, gap_open=sc.gap_open,
                           gap_extend=sc.gap_extend, affine=sc.affine, threads=THREADS)


def assert_same(got, want, coords):
    s, i, j = got
    ws, wi, wj = want
    bad = np.nonzero(s != ws)[0]
    assert bad.size == 0, f"{bad.size} score mismatches, first {bad[:5]}: gpu {s[bad[:5]]} oracle {ws[bad[:5]]}"
    if coords:
        bad = np.nonzero((i != wi) | (j != wj))[0]
        assert bad.size == 0, (f"{bad.size} coordinate mismatches, first {bad[:5]}: gpu "
                               f"{list(zip(i[bad[:5]], j[bad[:5]]))} oracle {list(zip(wi[bad[:5]], wj[bad[:5]]))}")


def related(rng, m, n):
    """A window of n random bases and a read of m bases copied from it (where
    it fits) with ~3 % substitutions and a few indels: nontrivial local
    alignments at any length."""
    w = ACGT[rng.integers(0, 4, n)]
    if n >= m > 0:
        off = int(rng.integers(0, n - m + 1))
        r = w[off:off + m].copy()
    else:
        r = ACGT[rng.integers(0, 4, m)]
        k = min(m, n)
        r[:k] = w[:k]
    sub = rng.random(m) < 0.03
    r[sub] = ACGT[rng.integers(0, 4, int(sub.sum()))]
    for _ in range(int(rng.integers(0, 3))):
        if r.size > 2:
            at = int(rng.integers(0, r.size))
            r = np.delete(r, at) if rng.random() < 0.5 else np.insert(r, at, ACGT[int(rng.integers(0, 4))])
    r = r[:m] if r.size >= m else np.concatenate([r, ACGT[rng.integers(0, 4, m - r.size)]])
    return r.tobytes(), w.tobytes()


# strip and block edges: 64 * R rows per strip (R <= 8: 512), 64-column blocks
EDGE = [(257, 16), (257, 300), (300, 600), (511, 700), (512, 512), (513, 1030), (640, 64), (1024, 65),
        (1025, 127), (1100, 1), (2000, 129), (150, 4097), (64, 5000), (1, 6000), (300, 4096), (777, 2049)]


def edge_batch(seed=11):
    rng = np.random.default_rng(seed)
    pairs = [related(rng, m, n) for m, n in EDGE]
    return mpa.pack_batch([p[0] for p in pairs], [p[1] for p in pairs])


@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("scheme", SCHEMES, ids=["default", "steep", "zero_pen"])
def test_long_edges(gpu_ctx, oracle, kind, scheme):
    sc = scoring(kind, scheme)
    R, rl, W, wl = edge_batch()
    assert_same(gpu_ctx.align_batch(R, rl, W, wl, sc), oracle_run(oracle, R, rl, W, wl, sc), sc.want_coords)


@pytest.mark.parametrize("kind", list(KINDS))
def test_long_random_batch(gpu_ctx, oracle, kind):
    """Synthetic reads of 257..1100 bp against windows of twice their length
    (1 % substitutions, indels, N, 10 % unrelated reads)."""
    sc = scoring(kind)
    b = make_pairs(160, (257, 1100), seed=2024)
    assert_same(gpu_ctx.align_batch(b.reads, b.read_len, b.wins, b.win_len, sc),
                oracle_run(oracle, b.reads, b.read_len, b.wins, b.win_len, sc), sc.want_coords)


@pytest.mark.parametrize("kind", list(KINDS))
def test_wide_buckets_one_launch(gpu_ctx, oracle, kind):
    """Reads of 200..384 bases: the KR <= 16 buckets in one length-bucketed
    launch and the KR 17..24 buckets (257..384) in one launch of its wide
    instance -- host batches (one chunk and several) and a plan."""
    import torch
    sc = scoring(kind)
    b = make_pairs(600, (200, 384), seed=31)
    want = oracle_run(oracle, b.reads, b.read_len, b.wins, b.win_len, sc)
    for chunk in (0, 97):
        assert_same(gpu_ctx.align_batch(b.reads, b.read_len, b.wins, b.win_len, sc, chunk_pairs=chunk), want,
                    sc.want_coords)
    n = b.n_pairs
    dR, dW, drl, dwl = _device([b.reads, b.wins, b.read_len.view(np.int16), b.win_len.view(np.int16)])
    score, ei, ej = _device([np.zeros(n, np.int32), np.zeros(n, np.int16), np.zeros(n, np.int16)])
    launch = gpu_ctx.prepare_planned_launch(dR.data_ptr(), drl.data_ptr(), dW.data_ptr(), dwl.data_ptr(),
                                            b.reads.shape[1], b.wins.shape[1], b.read_len, b.win_len,
                                            score.data_ptr(), sc, ei.data_ptr(), ej.data_ptr())
    try:
        launch()
        gpu_ctx.synchronize()
        torch.cuda.synchronize()
        assert_same((score.cpu().numpy(), ei.cpu().numpy(), ej.cpu().numpy()), want, sc.want_coords)
    finally:
        launch.close()


@pytest.mark.parametrize("blocks", ["1", "7", "0"])
@pytest.mark.parametrize("kind", ["linear", "affine_coords"])
def test_long_work_queue(fresh_ctx, oracle, monkeypatch, kind, blocks):
    """Long pairs of spread lengths (sorted heaviest first by the host) with
    fewer blocks than pairs (MSW_LONG_BLOCKS; "0" = the default grid): the
    blocks take slots from the launch's work queue -- host batches, the device
    API (input order) and a plan."""
    import torch
    monkeypatch.setenv("MSW_LONG_BLOCKS", blocks)
    sc = scoring(kind)
    b = make_pairs(90, (257, 1300), seed=77)
    want = oracle_run(oracle, b.reads, b.read_len, b.wins, b.win_len, sc)
    assert_same(fresh_ctx.align_batch(b.reads, b.read_len, b.wins, b.win_len, sc), want, sc.want_coords)
    n = b.n_pairs
    dR, dW, drl, dwl = _device([b.reads, b.wins, b.read_len.view(np.int16), b.win_len.view(np.int16)])
    score, ei, ej = _device([np.zeros(n, np.int32), np.zeros(n, np.int16), np.zeros(n, np.int16)])
    fresh_ctx.align_batch_device(dR.data_ptr(), drl.data_ptr(), dW.data_ptr(), dwl.data_ptr(), b.reads.shape[1],
                               b.wins.shape[1], n, score.data_ptr(), int(b.read_len.max()), int(b.win_len.max()), sc,
                               ei.data_ptr(), ej.data_ptr())
    torch.cuda.synchronize()
    fresh_ctx.synchronize()
    assert_same((score.cpu().numpy(), ei.cpu().numpy(), ej.cpu().numpy()), want, sc.want_coords)
    score.zero_()
    launch = fresh_ctx.prepare_planned_launch(dR.data_ptr(), drl.data_ptr(), dW.data_ptr(), dwl.data_ptr(),
                                            b.reads.shape[1], b.wins.shape[1], b.read_len, b.win_len,
                                            score.data_ptr(), sc, ei.data_ptr(), ej.data_ptr())
    try:
        launch()
        fresh_ctx.synchronize()
        assert_same((score.cpu().numpy(), ei.cpu().numpy(), ej.cpu().numpy()), want, sc.want_coords)
    finally:
        launch.close()


@pytest.mark.parametrize("chunk", [0, 37, 500])
@pytest.mark.parametrize("kind", ["linear", "affine_coords"])
def test_long_mixed_with_short(gpu_ctx, oracle, kind, chunk):
    """Short and long pairs in one call: the packed buckets (one
    length-bucketed launch) and the long bucket share each chunk."""
    sc = scoring(kind)
    rng = np.random.default_rng(7)
    s = make_pairs(1500, (75, 250), seed=5)
    reads = [bytes(s.reads[k, :s.read_len[k]]) for k in range(s.n_pairs)]
    wins = [bytes(s.wins[k, :s.win_len[k]]) for k in range(s.n_pairs)]
    for m, n in EDGE * 3:
        r, w = related(rng, m, n)
        at = int(rng.integers(0, len(reads) + 1))
        reads.insert(at, r)
        wins.insert(at, w)
    R, rl, W, wl = mpa.pack_batch(reads, wins)
    want = oracle_run(oracle, R, rl, W, wl, sc)
    assert_same(gpu_ctx.align_batch(R, rl, W, wl, sc, chunk_pairs=chunk), want, sc.want_coords)
    p = gpu_ctx.align_batch(R, rl, W, wl, sc, chunk_pairs=chunk, asynchronous=True)
    assert_same(p.wait(), want, sc.want_coords)


def test_long_extremes(gpu_ctx, oracle):
    """The 32767 limits, identical long sequences, empty reads/windows, and
    the range error past the limit."""
    rng = np.random.default_rng(3)
    pairs = [related(rng, 32767, 64), related(rng, 64, 32767), related(rng, 3000, 3000)]
    same = ACGT[rng.integers(0, 4, 4000)].tobytes()
    pairs += [(same, same), (b"", b"ACGT" * 1200), (b"ACGT" * 100, b"")]
    R, rl, W, wl = mpa.pack_batch([p[0] for p in pairs], [p[1] for p in pairs])
    for kind in KINDS:
        sc = scoring(kind)
        got = gpu_ctx.align_batch(R, rl, W, wl, sc)
        assert_same(got, oracle_run(oracle, R, rl, W, wl, sc), sc.want_coords)
        if not sc.affine:
            assert got[0][3] == 8000
            if sc.want_coords:
                assert (got[1][3], got[2][3]) == (3999, 3999)
                assert (got[1][4], got[2][4], got[1][5], got[2][5]) == (-1, -1, -1, -1)
    for m, n in ((32768, 16), (16, 32768)):
        R, rl, W, wl = mpa.pack_batch([b"A" * m], [b"A" * n])
        with pytest.raises(mpa.MswError, match="length"):
            gpu_ctx.align_batch(R, rl, W, wl, Scoring())


def _device(arrs):
    import torch
    dev = torch.device("cuda", 0)
    return [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in arrs]


@pytest.mark.parametrize("kind", ["linear", "affine_coords"])
def test_long_device_api(gpu_ctx, oracle, kind):
    """msw_align_batch_device with bounds past the packed kernels: the whole
    batch on the long kernel (short pairs included)."""
    import torch
    sc = scoring(kind)
    R, rl, W, wl = edge_batch(seed=5)
    dR, dW, drl, dwl = _device([R, W, rl.view(np.int16), wl.view(np.int16)])
    n = R.shape[0]
    score, ei, ej = _device([np.zeros(n, np.int32), np.zeros(n, np.int16), np.zeros(n, np.int16)])
    gpu_ctx.align_batch_device(dR.data_ptr(), drl.data_ptr(), dW.data_ptr(), dwl.data_ptr(), R.shape[1],
                               W.shape[1], n, score.data_ptr(), int(rl.max()), int(wl.max()), sc,
                               ei.data_ptr(), ej.data_ptr())
    torch.cuda.synchronize()
    gpu_ctx.synchronize()
    assert_same((score.cpu().numpy(), ei.cpu().numpy(), ej.cpu().numpy()),
                oracle_run(oracle, R, rl, W, wl, sc), sc.want_coords)


@pytest.mark.parametrize("kind", ["linear_coords", "affine"])
def test_long_planned(gpu_ctx, oracle, kind):
    """A plan over short and long pairs: one length-bucketed launch, the long
    launch, the slot-order gather; twice over the same plan."""
    import torch
    sc = scoring(kind)
    rng = np.random.default_rng(9)
    s = make_pairs(700, (75, 250), seed=8)
    reads = [bytes(s.reads[k, :s.read_len[k]]) for k in range(s.n_pairs)]
    wins = [bytes(s.wins[k, :s.win_len[k]]) for k in range(s.n_pairs)]
    for m, n in EDGE:
        r, w = related(rng, m, n)
        at = int(rng.integers(0, len(reads) + 1))
        reads.insert(at, r)
        wins.insert(at, w)
    R, rl, W, wl = mpa.pack_batch(reads, wins)
    n = R.shape[0]
    dR, dW, drl, dwl = _device([R, W, rl.view(np.int16), wl.view(np.int16)])
    score, ei, ej = _device([np.zeros(n, np.int32), np.zeros(n, np.int16), np.zeros(n, np.int16)])
    launch = gpu_ctx.prepare_planned_launch(dR.data_ptr(), drl.data_ptr(), dW.data_ptr(), dwl.data_ptr(),
                                            R.shape[1], W.shape[1], rl, wl, score.data_ptr(), sc,
                                            ei.data_ptr(), ej.data_ptr())
    want = oracle_run(oracle, R, rl, W, wl, sc)
    try:
        for _ in range(2):
            score.zero_()
            launch()
            gpu_ctx.synchronize()
            assert_same((score.cpu().numpy(), ei.cpu().numpy(), ej.cpu().numpy()), want, sc.want_coords)
    finally:
        launch.close()


@pytest.mark.parametrize("kind", ["linear", "linear_coords", "affine_coords"])
def test_long_genome_reads(gpu_ctx, oracle, kind):
    """Long reads against windows cut from an HBM-resident genome (the
    --full-wgs form), windows up to 6000 bases, positions near the end."""
    sc = scoring(kind)
    rng = np.random.default_rng(12)
    g = ACGT[rng.integers(0, 4, 200_000)]
    gen = gpu_ctx.load_genome(g.tobytes())
    n = 120
    rl = rng.integers(200, 1400, n).astype(np.uint16)
    wl = np.minimum(2 * rl.astype(np.int64) + rng.integers(0, 3000, n), 6000).astype(np.uint16)
    pos = rng.integers(-50, g.size - 100, n).astype(np.int64)
    R = np.zeros((n, 1408), np.uint8)
    for k in range(n):
        src = g[max(0, pos[k]) + 37:max(0, pos[k]) + 37 + rl[k]]
        R[k, :src.size] = src
        R[k, src.size:rl[k]] = ACGT[rng.integers(0, 4, rl[k] - src.size)]
    got = gpu_ctx.align_reads(gen, R, rl, pos, wl, sc, chunk_pairs=50)
    # the same windows cut on the host (clipped at the genome end, empty outside it)
    W = np.zeros((n, 6000), np.uint8)
    eff = np.zeros(n, np.uint16)
    for k in range(n):
        if 0 <= pos[k] < g.size:
            w = g[pos[k]:pos[k] + wl[k]]
            W[k, :w.size] = w
            eff[k] = w.size
    assert_same(got, oracle_run(oracle, R, rl, W, eff, sc), sc.want_coords)


@pytest.mark.parametrize("kind", list(KINDS))
def test_long_kernel_on_short_shapes(fresh_ctx, oracle, monkeypatch, kind):
    """MSW_FORCE_LONG=1: the long-pair kernel over the packed kernels' own
    shapes (config-2 pairs, mixed 75-250 bp reads) -- one strip, R = 1..4."""
    monkeypatch.setenv("MSW_FORCE_LONG", "1")
    sc = scoring(kind)
    for b in (make_pairs(3000, 150, seed=31), make_pairs(2000, (1, 250), seed=32)):
        assert_same(fresh_ctx.align_batch(b.reads, b.read_len, b.wins, b.win_len, sc),
                    oracle_run(oracle, b.reads, b.read_len, b.wins, b.win_len, sc), sc.want_coords)


@pytest.mark.parametrize("kind", list(KINDS))
def test_long_random_sizes(gpu_ctx, oracle, kind):
    """240 pairs of random sizes (reads 1..3000, windows 1..5000; related and
    unrelated), short and long mixed in one call, chunked."""
    sc = scoring(kind)
    rng = np.random.default_rng(77)
    pairs = []
    for _ in range(240):
        m, n = int(rng.integers(1, 3001)), int(rng.integers(1, 5001))
        if rng.random() < 0.2:
            pairs.append((ACGT[rng.integers(0, 4, m)].tobytes(), ACGT[rng.integers(0, 4, n)].tobytes()))
        else:
            pairs.append(related(rng, m, n))
    R, rl, W, wl = mpa.pack_batch([p[0] for p in pairs], [p[1] for p in pairs])
    want = oracle_run(oracle, R, rl, W, wl, sc)
    assert_same(gpu_ctx.align_batch(R, rl, W, wl, sc, chunk_pairs=100), want, sc.want_coords)


@pytest.mark.parametrize("env", [{"MSW_NO_MULTI": "1"}, {"MSW_LAYOUT": "split"}, {"MSW_LAYOUT": "pairs", "MSW_GROUP_LANES": "12"},
                                 {"MSW_NO_F16": "1"}])
def test_long_beside_forced_layouts(fresh_ctx, oracle, monkeypatch, env):
    """The long bucket next to per-bucket launches of the packed kernels
    (forced layouts, no single multi launch) and next to the integer path."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sc = scoring("linear_coords")
    rng = np.random.default_rng(5)
    s = make_pairs(600, (60, 250), seed=9)
    reads = [bytes(s.reads[k, :s.read_len[k]]) for k in range(s.n_pairs)]
    wins = [bytes(s.wins[k, :s.win_len[k]]) for k in range(s.n_pairs)]
    for m, n in EDGE:
        r, w = related(rng, m, n)
        at = int(rng.integers(0, len(reads) + 1))
        reads.insert(at, r)
        wins.insert(at, w)
    R, rl, W, wl = mpa.pack_batch(reads, wins)
    assert_same(fresh_ctx.align_batch(R, rl, W, wl, sc, chunk_pairs=300), oracle_run(oracle, R, rl, W, wl, sc), True)
