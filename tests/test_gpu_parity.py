"""GPU parity: the HIP kernels, called through the C ABI, must be bit-exact
against the oracle (scores and best-cell coordinates).  Run with -m gpu."""
import json
import os

import numpy as np
import pytest

import mini_parallel_amd as mpa
from mini_parallel_amd import Scoring
from mini_parallel_amd.synthetic import config_batch, make_pairs

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
THREADS = min(16, os.cpu_count() or 1)


def oracle_run(oracle, b, sc: Scoring):
    return oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, match=sc.match,
                           mismatch=sc.mismatch, gap_open=sc.gap_open, gap_extend=sc.gap_extend,
                           affine=sc.affine, threads=THREADS)


def gpu_run(ctx, b, sc: Scoring, chunk=0):
    return ctx.align_batch(b.reads, b.read_len, b.wins, b.win_len, sc, chunk_pairs=chunk)


def assert_same(got, want, coords: bool):
    s, i, j = got
    ws, wi, wj = want
    bad = np.nonzero(s != ws)[0]
    assert bad.size == 0, f"{bad.size} score mismatches, first at {bad[:5]}: gpu {s[bad[:5]]} oracle {ws[bad[:5]]}"
    if coords:
        bad = np.nonzero((i != wi) | (j != wj))[0]
        assert bad.size == 0, (f"{bad.size} coordinate mismatches, first {bad[:5]}: gpu "
                               f"{list(zip(i[bad[:5]], j[bad[:5]]))} oracle {list(zip(wi[bad[:5]], wj[bad[:5]]))}")


@pytest.fixture(params=["auto", "pairs", "split", "mixed", "pairs:12", "pairs:9", "pairs:8", "split:11",
                        "split:8"])
def layout(request, monkeypatch):
    """Every lane-group layout of the kernel, with 16-lane groups and with
    narrower ones (G = 12, 11, 9, 8: idle lanes at the wave's end, groups that
    straddle DPP rows).  The runtime normally picks layout and G per launch
    from a makespan model ("auto"; mixed-length batches then run as one
    length-bucketed sw_multi_kernel launch); a forced layout launches each
    length bucket on its own, and a forced G that cannot hold the batch's reads
    (KR > 24, or the LDS budget) falls back to G = 16.  Forced G = 8 / 9 on
    the 150 bp batches runs 19 / 17 packed rows per lane, the narrow groups
    the model picks for batches of >= 16 (G = 9) / 48 (G = 8) waves per SIMD."""
    if request.param == "auto":
        for k in ("MSW_LAYOUT", "MSW_GROUP_LANES", "MSW_NO_MULTI"):
            monkeypatch.delenv(k, raising=False)
        return request.param
    lay, _, g = request.param.partition(":")
    monkeypatch.setenv("MSW_LAYOUT", lay)
    if g:
        monkeypatch.setenv("MSW_GROUP_LANES", g)
    else:
        monkeypatch.delenv("MSW_GROUP_LANES", raising=False)
    return request.param


class B:  # minimal batch holder
    def __init__(self, reads, read_len, wins, win_len):
        self.reads, self.read_len, self.wins, self.win_len = reads, read_len, wins, win_len


def test_device_visible(gpu_ctx):
    devs = mpa.get_gpu_devices()
    assert devs and devs[0].arch.startswith("gfx950"), devs


@pytest.mark.parametrize("section,sc", [
    ("linear_2_-1_2", Scoring(want_coords=True)),
    ("affine_2_-1_o3_e1", Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True)),
])
def test_kat(fresh_ctx, layout, section, sc):
    kats = json.load(open(os.path.join(GOLDEN, "kat.json")))[section]
    R, rl, W, wl = mpa.pack_batch([k["read"].encode() for k in kats], [k["window"].encode() for k in kats])
    s, i, j = fresh_ctx.align_batch(R, rl, W, wl, sc)
    for k, a, b, c in zip(kats, s, i, j):
        assert (int(a), int(b), int(c)) == (k["score"], k["end_i"], k["end_j"]), k


@pytest.mark.parametrize("name", ["linear_150x300.npz", "affine_150x300.npz", "mixed_linear.npz"])
@pytest.mark.parametrize("coords", [False, True])
def test_golden(fresh_ctx, layout, name, coords):
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    sc = Scoring(match=meta["match"], mismatch=meta["mismatch"], gap_open=meta.get("gap_open", 0),
                 gap_extend=meta["gap_extend"], affine=meta["affine"], want_coords=coords)
    got = fresh_ctx.align_batch(z["reads"], z["read_len"], z["wins"], z["win_len"], sc)
    assert_same(got, (z["score"], z["end_i"], z["end_j"]), coords)


def test_config2_linear_score_only(fresh_ctx, layout, oracle):
    """BASELINE config 2 at full size: 10k x (150 bp, 300 bp), linear, score-only."""
    b = config_batch(2)
    sc = Scoring()
    assert_same(gpu_run(fresh_ctx, b, sc), oracle_run(oracle, b, sc), False)


def test_config3_affine_coords_sample(fresh_ctx, layout, oracle):
    """Config 3 shape (affine + best cell), chunked through the pinned pipeline."""
    b = config_batch(3, n_pairs=40_000)
    sc = Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True)
    assert_same(gpu_run(fresh_ctx, b, sc, chunk=9_000), oracle_run(oracle, b, sc), True)


@pytest.mark.parametrize("sc", [Scoring(), Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True)],
                         ids=["linear", "affine_coords"])
def test_narrow_groups_large_batch(fresh_ctx, oracle, monkeypatch, capfd, sc):
    """A batch large enough (>= 48 waves per SIMD of 16-pair waves, sized
    from this GPU's CU count) that the layout model takes narrow lane groups
    of 17..19 rows (150 bp reads: G = 8 or 9) on its own, as one launch --
    the choice read back from MSW_HOST_TRACE -- and every pair against the
    SIMD oracle."""
    for k in ("MSW_LAYOUT", "MSW_GROUP_LANES", "MSW_NO_MULTI"):
        monkeypatch.delenv(k, raising=False)
    n = int(48 * 4 * mpa.get_gpu_devices()[0].cu_count * 16 * 1.02)
    b = config_batch(3, n_pairs=n)
    monkeypatch.setenv("MSW_HOST_TRACE", "1")
    capfd.readouterr()
    got = gpu_run(fresh_ctx, b, sc, chunk=n)
    line = [ln for ln in capfd.readouterr().err.splitlines() if ln.startswith("[msw host]")][-1]
    plan = line.split("last_launch(")[1].split(")")[0]
    g = int(plan.split("G=")[1].split()[0])
    kr = int(plan.split("KR=")[1].split()[0])
    assert "layout=pairs" in plan and g in (8, 9) and 17 <= kr <= 19, line
    s, i, j, _ = oracle.sw_batch_simd(b.reads, b.read_len, b.wins, b.win_len, match=sc.match, mismatch=sc.mismatch,
                                      gap_open=sc.gap_open, gap_extend=sc.gap_extend, affine=sc.affine,
                                      threads=THREADS, coords=sc.want_coords)
    assert_same(got, (s, i, j), sc.want_coords)


def _last_plan(capfd):
    line = [ln for ln in capfd.readouterr().err.splitlines() if ln.startswith("[msw host]")][-1]
    plan = line.split("last_launch(")[1].split(")")[0]
    return line, plan.split("layout=")[1].split()[0], int(plan.split("G=")[1].split()[0]), \
        int(plan.split("KR=")[1].split()[0])


@pytest.mark.parametrize("n", [131_072, 262_144, 524_288])
@pytest.mark.parametrize("sc", [Scoring(), Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True)],
                         ids=["linear", "affine_coords"])
def test_narrow_gate_mid_batches(fresh_ctx, oracle, monkeypatch, capfd, sc, n):
    """Config-3 batches (150 bp reads) either side of the measured narrow-group
    crossover, each at the layout model's own choice: 9-lane groups of 17 rows
    (14 pairs per wave) are taken from 16 waves per SIMD on (229k pairs on 256
    CUs), 8-lane groups of 19 rows only from 48; below that the launch keeps
    rows <= 16 per lane.  Every pair is checked against the SIMD oracle."""
    for k in ("MSW_LAYOUT", "MSW_GROUP_LANES", "MSW_NO_MULTI"):
        monkeypatch.delenv(k, raising=False)
    simds = 4 * mpa.get_gpu_devices()[0].cu_count
    b = config_batch(3, n_pairs=n, seed_offset=n % 977)
    monkeypatch.setenv("MSW_HOST_TRACE", "1")
    capfd.readouterr()
    got = gpu_run(fresh_ctx, b, sc, chunk=n)
    line, lay, g, kr = _last_plan(capfd)
    if kr > 16:  # a narrow launch: only past its family's measured gate
        per = 2 * (64 // g)
        assert lay == "pairs" and -(-n // per) >= (16 if kr <= 17 else 48) * simds, line
    if -(-n // 14) >= 16 * simds:  # past the 9-lane gate: the model takes it
        assert kr > 16 and g in (8, 9), line
    s, i, j, _ = oracle.sw_batch_simd(b.reads, b.read_len, b.wins, b.win_len, match=sc.match, mismatch=sc.mismatch,
                                      gap_open=sc.gap_open, gap_extend=sc.gap_extend, affine=sc.affine,
                                      threads=THREADS, coords=sc.want_coords)
    assert_same(got, (s, i, j), sc.want_coords)


def test_config5_mixed_lengths(fresh_ctx, layout, oracle):
    """Config 5 shape: 75-250 bp reads, window 2m, length-bucketed dispatch."""
    b = config_batch(5, n_pairs=12_000)
    for sc in (Scoring(want_coords=True), Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True)):
        assert_same(gpu_run(fresh_ctx, b, sc), oracle_run(oracle, b, sc), True)


@pytest.mark.parametrize("coords", [False, True])
@pytest.mark.parametrize("affine", [False, True])
def test_integer_domain_on_acgt(fresh_ctx, layout, oracle, monkeypatch, affine, coords):
    """MSW_NO_F16 forces the u16 integer path (xor/min substitution) on
    ACGT windows that would otherwise take the f16 table path."""
    monkeypatch.setenv("MSW_NO_F16", "1")
    b = config_batch(2, n_pairs=3000, seed_offset=91)
    sc = Scoring(gap_open=3 if affine else 0, gap_extend=1 if affine else 2, affine=affine, want_coords=coords)
    assert_same(gpu_run(fresh_ctx, b, sc), oracle_run(oracle, b, sc), coords)


@pytest.mark.parametrize("match,mismatch,go,ge,affine", [
    (1, 0, 0, 1, False), (1, -1, 0, 1, False), (5, -4, 0, 3, False), (3, -2, 0, 0, False),
    (1, -3, 5, 2, True), (2, -1, 3, 1, True), (4, -60, 10, 1, True), (2, 0, 1, 1, True),
    # f16 fast path off: 9 and -9 are not f16 values with a zero low byte; 16 * 200 >= 2048
    (9, -9, 0, 2, False), (16, -8, 0, 4, False), (16, -8, 20, 3, True),
    # gap penalties of 2048 and more (capped in the f16 domain)
    (2, -1, 0, 1024, False), (2, -1, 5000, 1024, True),
])
def test_scoring_schemes(fresh_ctx, layout, oracle, match, mismatch, go, ge, affine):
    b = make_pairs(3000, (1, 200), 1.7, seed=match * 100 + ge, read_stride=208, win_stride=352)
    sc = Scoring(match=match, mismatch=mismatch, gap_open=go, gap_extend=ge, affine=affine, want_coords=True)
    assert_same(gpu_run(fresh_ctx, b, sc), oracle_run(oracle, b, sc), True)


def test_edge_lengths(fresh_ctx, layout, oracle):
    """Empty, 1-base, 16k+/-1 boundaries, max read 256, long windows, byte zoo."""
    rng = np.random.default_rng(17)
    lens_r = [0, 1, 2, 15, 16, 17, 31, 32, 33, 150, 255, 256, 256, 7, 0, 100]
    lens_w = [5, 0, 1, 16, 15, 17, 300, 4096, 1, 512, 256, 4096, 1000, 3000, 0, 2]
    reads, wins = [], []
    for m, n in zip(lens_r, lens_w):
        alpha = np.frombuffer(bytes(range(256)), np.uint8) if m % 2 else np.frombuffer(b"ACGTN", np.uint8)
        reads.append(bytes(rng.choice(alpha, m)))
        wins.append(bytes(rng.choice(alpha, n)))
    # plant exact copies so long alignments exist
    wins[11] = wins[11][:100] + reads[11] + wins[11][356:]
    wins[12] = reads[12] + wins[12][256:]
    R, rl, W, wl = mpa.pack_batch(reads * 3, wins * 3)
    b = B(R, rl, W, wl)
    for sc in (Scoring(want_coords=True), Scoring(gap_open=2, gap_extend=1, affine=True, want_coords=True)):
        assert_same(gpu_run(fresh_ctx, b, sc), oracle_run(oracle, b, sc), True)


def test_identical_and_all_mismatch(fresh_ctx, layout, oracle):
    rng = np.random.default_rng(23)
    seqs = [bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), 150)) for _ in range(64)]
    reads = seqs + [b"A" * 150] * 8 + [b"N" * 150] * 8
    wins = seqs + [b"C" * 300] * 8 + [b"N" * 300] * 8
    R, rl, W, wl = mpa.pack_batch(reads, wins)
    b = B(R, rl, W, wl)
    sc = Scoring(want_coords=True)
    got = gpu_run(fresh_ctx, b, sc)
    assert_same(got, oracle_run(oracle, b, sc), True)
    assert all(got[0][:64] == 300) and all(got[0][64:72] == 0) and all(got[1][64:72] == -1)
    assert all(got[0][72:] == 300)


def test_acgt_fast_path_and_fallback(fresh_ctx, layout, oracle):
    """Waves whose windows are pure A/C/G/T take the v_perm table path (reads
    may hold any byte: N, lower case, bytes whose class formula collides with
    A/C/G/T such as 'E', high-bit bytes); a window with any other byte sends its
    wave down the xor/min path.  Both must agree with the oracle."""
    rng = np.random.default_rng(31)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    zoo = np.frombuffer(b"ACGTACGTACGTNacgtEBDHS\x00\xc1\xc3\x41", np.uint8)
    reads, wins = [], []
    for k in range(1024):
        m = int(rng.integers(1, 257))
        n = int(rng.integers(1, 520))
        r = bytes(rng.choice(zoo if k % 3 else acgt, m))
        w = bytearray(rng.choice(acgt, n))
        if k % 5 == 0:
            w[int(rng.integers(0, n))] = int(rng.choice(np.frombuffer(b"NaEx\x00", np.uint8)))
        if k % 7 == 0 and n > m:  # plant the read so long alignments exist
            w[: m] = r
        reads.append(r)
        wins.append(bytes(w))
    R, rl, W, wl = mpa.pack_batch(reads, wins)
    b = B(R, rl, W, wl)
    for sc in (Scoring(want_coords=True), Scoring(),
               Scoring(gap_open=2, gap_extend=1, affine=True, want_coords=True),
               Scoring(match=3, mismatch=-61, gap_open=7, gap_extend=1024, affine=True)):
        assert_same(gpu_run(fresh_ctx, b, sc), oracle_run(oracle, b, sc), sc.want_coords)


def test_async_and_chunking_agree(gpu_ctx, oracle):
    b = config_batch(2, n_pairs=5000, seed_offset=40)
    sc = Scoring(want_coords=True)
    want = oracle_run(oracle, b, sc)
    for chunk in (0, 1, 7, 999, 5000):
        if chunk == 1:
            sub = B(b.reads[:50], b.read_len[:50], b.wins[:50], b.win_len[:50])
            assert_same(gpu_run(gpu_ctx, sub, sc, chunk), tuple(w[:50] for w in want), True)
        else:
            assert_same(gpu_run(gpu_ctx, b, sc, chunk), want, True)


def test_dropped_pending_then_more_calls(gpu_ctx, oracle):
    """an async call dropped without wait() must not leave chunks
    that later drain into its freed output arrays (Pending.__del__ waits)."""
    import gc
    b = config_batch(2, n_pairs=3000, seed_offset=41)
    sc = Scoring(want_coords=True)
    want = oracle_run(oracle, b, sc)
    for _ in range(3):
        p = gpu_ctx.align_batch(b.reads, b.read_len, b.wins, b.win_len, sc, chunk_pairs=700, asynchronous=True)
        del p
        gc.collect()
        junk = [np.full(3000, 7, np.int32) for _ in range(8)]  # reuse the freed memory
        assert_same(gpu_run(gpu_ctx, b, sc, 1000), want, True)
        assert all((j == 7).all() for j in junk)


def test_ctx_stats_count_kernel_time(gpu_ctx):
    """msw_ctx_stats: kernel time and algorithmic bytes of host-batch calls."""
    b = config_batch(2, n_pairs=4000, seed_offset=42)
    gpu_ctx.stats(reset=True)
    gpu_run(gpu_ctx, b, Scoring(), 1000)
    st = gpu_ctx.stats(reset=True)
    assert st["launches"] == 4 and st["pairs"] == 4000
    assert st["cells"] == int((b.read_len.astype(np.int64) * b.win_len).sum())
    assert st["alg_bytes"] == int(b.read_len.astype(np.int64).sum() + b.win_len.astype(np.int64).sum()) + 4 * 4000
    assert 0 < st["kernel_ms"] < 1000
    assert gpu_ctx.stats()["launches"] == 0


def test_ctx_stats_kernel_time_is_a_union(gpu_ctx):
    """kernel_ms counts GPU time covered by scoring launches once: the chunks
    of a multi-chunk call alternate two compute streams and overlap, so the
    sum of their durations can exceed the call's wall time; the union cannot."""
    import time
    b = config_batch(2, n_pairs=40_000, seed_offset=43)
    gpu_run(gpu_ctx, b, Scoring(), 4000)  # warm
    gpu_ctx.stats(reset=True)
    t0 = time.perf_counter()
    gpu_run(gpu_ctx, b, Scoring(), 4000)
    wall_ms = (time.perf_counter() - t0) * 1e3
    st = gpu_ctx.stats(reset=True)
    assert st["launches"] >= 10 and st["pairs"] == 40_000
    assert 0 < st["kernel_ms"] <= wall_ms, (st["kernel_ms"], wall_ms)


def test_ctx_stats_kernel_time_lower_bound(gpu_ctx):
    """the union must not lose intervals either.  Async calls in
    pairs, each pair waited on its second ticket, drain their slots oldest
    chunk first whatever slots they landed in (slots rotate in threes, so
    pairs of calls put the newer chunk in the lower slot every third pair);
    with large one-chunk launches the two calls of a pair barely overlap, so
    their union is within a few percent of the same launches run one by one."""
    b = config_batch(2, n_pairs=200_000, seed_offset=44)
    sc = Scoring()

    def run(k):
        return gpu_ctx.align_batch(b.reads, b.read_len, b.wins, b.win_len, sc, chunk_pairs=200_000,
                                   asynchronous=k is not None)
    run(None)  # warm
    gpu_ctx.stats(reset=True)
    for _ in range(6):
        run(None)
    serial = gpu_ctx.stats(reset=True)["kernel_ms"]
    for _ in range(3):
        pend = [run(k) for k in range(2)]
        pend[1].wait()
        pend[0].wait()
    paired = gpu_ctx.stats(reset=True)
    assert paired["launches"] == 6
    assert 0.9 * serial <= paired["kernel_ms"] <= 1.1 * serial, (paired["kernel_ms"], serial)


def test_empty_batch(gpu_ctx):
    R = np.zeros((0, 16), np.uint8)
    s, i, j = gpu_ctx.align_batch(R, np.zeros(0, np.uint16), R, np.zeros(0, np.uint16), Scoring(want_coords=True))
    assert s.shape == (0,)


@pytest.mark.parametrize("bad", ["long_read", "long_window", "match", "mismatch", "delta"])
def test_range_errors(gpu_ctx, bad):
    # lengths past the long-pair kernel's 32767 (i16 coordinates)
    R, rl, W, wl = mpa.pack_batch([b"A" * 32768 if bad == "long_read" else b"ACGT"],
                                  [b"A" * 32768 if bad == "long_window" else b"ACGT"])
    sc = {"match": Scoring(match=65), "mismatch": Scoring(mismatch=1),
          "delta": Scoring(match=10, mismatch=-55)}.get(bad, Scoring())
    with pytest.raises(mpa.MswError):
        gpu_ctx.align_batch(R, rl, W, wl, sc)


def test_device_resident_api(fresh_ctx, layout, oracle):
    """msw_align_batch_device over HBM-resident arrays (the bench path)."""
    import torch
    b = config_batch(2, n_pairs=4000, seed_offset=77)
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(b, k))).to(dev)
         for k in ("reads", "wins")}
    rl = torch.from_numpy(b.read_len.view(np.int16)).to(dev)
    wl = torch.from_numpy(b.win_len.view(np.int16)).to(dev)
    score = torch.zeros(b.n_pairs, dtype=torch.int32, device=dev)
    ei = torch.zeros(b.n_pairs, dtype=torch.int16, device=dev)
    ej = torch.zeros(b.n_pairs, dtype=torch.int16, device=dev)
    sc = Scoring(want_coords=True)
    fresh_ctx.align_batch_device(t["reads"].data_ptr(), rl.data_ptr(), t["wins"].data_ptr(), wl.data_ptr(),
                               b.reads.shape[1], b.wins.shape[1], b.n_pairs, score.data_ptr(),
                               int(b.read_len.max()), int(b.win_len.max()), sc, ei.data_ptr(),
                               ej.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = (score.cpu().numpy(), ei.cpu().numpy(), ej.cpu().numpy())
    assert_same(got, oracle_run(oracle, b, sc), True)


def _device_batch(b):
    import torch
    dev = torch.device("cuda", 0)
    d = {k: torch.from_numpy(np.ascontiguousarray(getattr(b, k))).to(dev) for k in ("reads", "wins")}
    d["rl"] = torch.from_numpy(np.ascontiguousarray(b.read_len).view(np.int16)).to(dev)
    d["wl"] = torch.from_numpy(np.ascontiguousarray(b.win_len).view(np.int16)).to(dev)
    d["score"] = torch.full((b.n_pairs,), -7, dtype=torch.int32, device=dev)
    d["ei"] = torch.zeros(b.n_pairs, dtype=torch.int16, device=dev)
    d["ej"] = torch.zeros(b.n_pairs, dtype=torch.int16, device=dev)
    return d


def _planned(gpu_ctx, b, sc, passes=1):
    import torch
    d = _device_batch(b)
    step = gpu_ctx.prepare_planned_launch(d["reads"].data_ptr(), d["rl"].data_ptr(), d["wins"].data_ptr(),
                                          d["wl"].data_ptr(), b.reads.shape[1], b.wins.shape[1],
                                          b.read_len, b.win_len, d["score"].data_ptr(), sc,
                                          d["ei"].data_ptr(), d["ej"].data_ptr(),
                                          torch.cuda.current_stream().cuda_stream)
    for _ in range(passes):
        step()
    torch.cuda.synchronize()
    step.close()
    return d["score"].cpu().numpy(), d["ei"].cpu().numpy(), d["ej"].cpu().numpy()


@pytest.mark.parametrize("multi", [True, False])
@pytest.mark.parametrize("sc", [Scoring(), Scoring(want_coords=True), Scoring(gap_open=3, gap_extend=1, affine=True),
                                Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True)],
                         ids=["linear", "linear+coords", "affine", "affine+coords"])
def test_planned_mixed_lengths(fresh_ctx, oracle, monkeypatch, sc, multi):
    """msw_plan_create + msw_align_batch_planned (config 5 shape, unsorted,
    device-resident): one length-bucketed launch (multi) or the single-bucket
    path over the plan's order (MSW_NO_MULTI), twice over the same plan."""
    for k in ("MSW_LAYOUT", "MSW_GROUP_LANES", "MSW_NO_MULTI"):
        monkeypatch.delenv(k, raising=False)
    if not multi:
        monkeypatch.setenv("MSW_NO_MULTI", "1")
    b = config_batch(5, n_pairs=9_000, seed_offset=31)
    assert_same(_planned(fresh_ctx, b, sc, passes=2), oracle_run(oracle, b, sc), sc.want_coords)


def test_planned_edge_cases(gpu_ctx, oracle, monkeypatch):
    """Plans over every read-length bucket at once (1..256 bp, windows 0..600,
    non-ACGT bytes in some windows so some waves take the integer path),
    a one-pair plan and an empty plan."""
    for k in ("MSW_LAYOUT", "MSW_GROUP_LANES", "MSW_NO_MULTI"):
        monkeypatch.delenv(k, raising=False)
    rng = np.random.default_rng(5)
    n = 3000
    rlen = rng.integers(0, 257, n).astype(np.uint16)
    wlen = rng.integers(0, 601, n).astype(np.uint16)
    reads = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=(n, 256)).astype(np.uint8)
    wins = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=(n, 608)).astype(np.uint8)
    wins[::7, 5] = ord("N")
    b = B(reads, rlen, wins, wlen)
    b.n_pairs = n
    for sc in (Scoring(want_coords=True), Scoring(gap_open=2, gap_extend=1, affine=True, want_coords=True)):
        assert_same(_planned(gpu_ctx, b, sc), oracle_run(oracle, b, sc), True)
    one = B(reads[:1], rlen[:1], wins[:1], wlen[:1])
    one.n_pairs = 1
    assert_same(_planned(gpu_ctx, one, Scoring(want_coords=True)), oracle_run(oracle, one, Scoring()), True)
    step = gpu_ctx.prepare_planned_launch(0, 0, 0, 0, 16, 16, np.zeros(0, np.uint16), np.zeros(0, np.uint16),
                                          0, Scoring())
    step()
    step.close()


def test_compat_kats(gpu_ctx):
    for k in json.load(open(os.path.join(GOLDEN, "kat.json")))["compat"]:
        assert gpu_ctx.compat(k["s1"].encode(), k["s2"].encode(), k["wg"], k["max_groups"]) == k["expected"], k


def test_compat_random_vs_oracle(gpu_ctx, oracle):
    rng = np.random.default_rng(31)
    for L, wg, mg in [(1, 1024, 0), (1000, 64, 3), (5000, 256, 7), (1 << 20, 1024, 0), (3_000_001, 1024, 0),
                      (100_000, 64, 5)]:
        a = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), L))
        b = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), L + 3))
        assert gpu_ctx.compat(a, b, wg, mg) == oracle.compat_align(a, b, wg, mg)


def test_gpu_align_reference_semantics(gpu_ctx):
    dev = mpa.get_gpu_devices()[0]
    assert mpa.gpu_align("ACGTACGT", "ACGTACGT", dev) == 2
    assert mpa.gpu_align("AAAA", "CCCC", dev) == 0
    assert mpa.gpu_align("", "ACGT", dev) == 0
    assert mpa.gpu_align_chunk_self("ACGT" * 200, dev) == 0          # < 1000 bases
    assert mpa.gpu_align_chunk_self("ACGT" * 300, dev) == 2


def test_full_size_properties(gpu_ctx, oracle):
    """1M pairs (config 3 size): size-independent invariants on all pairs and
    bit-exact parity on a random sample."""
    b = config_batch(3)
    sc = Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True)
    s, i, j = gpu_run(gpu_ctx, b, sc)
    assert (s >= 0).all()
    zero = s == 0
    assert ((i == -1) == zero).all() and ((j == -1) == zero).all()
    assert (i[~zero] < b.read_len[~zero]).all() and (j[~zero] < b.win_len[~zero]).all()
    assert (s <= 2 * b.read_len.astype(np.int32)).all()
    rng = np.random.default_rng(0)
    idx = np.sort(rng.choice(b.n_pairs, 3000, replace=False))
    sub = B(b.reads[idx], b.read_len[idx], b.wins[idx], b.win_len[idx])
    assert_same((s[idx], i[idx], j[idx]), oracle_run(oracle, sub, sc), True)
    # linear score-only on the same million: the best-cell kernel gives the same scores
    s_lin = gpu_run(gpu_ctx, b, Scoring())[0]
    s_lin_c = gpu_run(gpu_ctx, b, Scoring(want_coords=True))[0]
    assert np.array_equal(s_lin, s_lin_c)


def test_config1_plumbing(gpu_ctx, oracle):
    """BASELINE config 1: two 32 bp synthetic sequences (seed 1001) through the
    batched path and through the CLI's pair mode (`-1 -2 --gpu --score-mode sw`),
    against the oracle; the legacy pair mode against the compat restatement."""
    import subprocess
    b = config_batch(1)
    sc = Scoring(want_coords=True)
    want = oracle_run(oracle, b, sc)
    assert_same(gpu_run(gpu_ctx, b, sc), want, True)
    s1 = bytes(b.reads[0, :b.read_len[0]]).decode()
    s2 = bytes(b.wins[0, :b.win_len[0]]).decode()
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini_parallel_amd",
                       "rustseq_mini")
    out = subprocess.run([cli, "-1", s1, "-2", s2, "--gpu", "--score-mode", "sw"], capture_output=True, text=True,
                         check=True).stdout
    assert f"GPU Alignment score: {int(want[0][0])}" in out
    assert f"Best cell: read {int(want[1][0])}, window {int(want[2][0])}" in out
    out = subprocess.run([cli, "-1", s1, "-2", s2, "--gpu"], capture_output=True, text=True, check=True).stdout
    assert f"GPU Alignment score: {oracle.compat_align(s1.encode(), s2.encode(), 1024, 1_000_000)}" in out


def test_ctx_prepare_then_score(gpu_ctx, oracle):
    """msw_ctx_prepare loads the scoring modules (no launch) for every scheme;
    scoring right after is unchanged."""
    b = config_batch(2, n_pairs=2000, seed_offset=45)
    for sc in (Scoring(), Scoring(want_coords=True), Scoring(gap_open=3, gap_extend=1, affine=True),
               Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True)):
        gpu_ctx.prepare(sc)
        assert_same(gpu_run(gpu_ctx, b, sc), oracle_run(oracle, b, sc), sc.want_coords)


@pytest.mark.parametrize("nbytes,src_off,dst_off", [(1, 0, 0), (15, 0, 0), (4096 * 3 + 7, 0, 0), (1 << 20, 0, 0),
                                                    (100_003, 4, 4), (65_536, 3, 7), (262_144 * 2, 16, 0)])
@pytest.mark.parametrize("pinned", [True, False])
def test_memcpy_d2h_async(gpu_ctx, nbytes, src_off, dst_off, pinned):
    """msw_memcpy_d2h_async: into pinned memory a copy kernel on the stream
    when source and destination share their alignment mod 16, a DMA when they
    do not (no byte-by-byte stores over PCIe); into pageable
    memory a DMA; all followed by a fence."""
    import ctypes
    from mini_parallel_amd._lib import check, lib
    from mini_parallel_amd.aligner import pinned_empty
    L = lib()
    rng = np.random.default_rng(nbytes)
    data = rng.integers(0, 256, nbytes + src_off, dtype=np.uint8)
    d = L.msw_dev_alloc(gpu_ctx.handle, nbytes + src_off + 16)
    assert d
    try:
        check(L.msw_memcpy_h2d(gpu_ctx.handle, d, data.ctypes.data, data.nbytes))
        out = pinned_empty(nbytes + dst_off + 16, np.uint8) if pinned else np.zeros(nbytes + dst_off + 16, np.uint8)
        out[:] = 0xA5
        fence = ctypes.c_uint64()
        check(L.msw_memcpy_d2h_async(gpu_ctx.handle, out.ctypes.data + dst_off, d + src_off, nbytes, None))
        check(L.msw_fence_record(gpu_ctx.handle, None, ctypes.byref(fence)))
        check(L.msw_fence_wait(gpu_ctx.handle, fence.value))
        assert np.array_equal(out[dst_off:dst_off + nbytes], data[src_off:])
        assert (out[:dst_off] == 0xA5).all() and (out[dst_off + nbytes:] == 0xA5).all()
    finally:
        L.msw_dev_free(gpu_ctx.handle, d)


@pytest.mark.parametrize("chunk", [20_000, 65_536, 70_000, 131_072])
def test_chunk_ramp(gpu_ctx, oracle, chunk):
    """A multi-chunk call: a short first chunk, then (chunk_pairs > 64k)
    chunks doubling up to chunk_pairs, or (smaller chunks) the rest full size
    -- 100k config-3 pairs, affine + best cell, pairs arrays and genome form,
    every pair against the SIMD oracle."""
    b = config_batch(3, n_pairs=100_000, seed_offset=77)
    sc = Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True)
    want = oracle_run(oracle, b, sc)
    assert_same(gpu_run(gpu_ctx, b, sc, chunk=chunk), want, True)
    ws = b.wins.shape[1]
    g = gpu_ctx.load_genome(np.ascontiguousarray(b.wins).reshape(-1))
    try:
        got = gpu_ctx.align_reads(g, b.reads, b.read_len, np.arange(b.n_pairs, dtype=np.int64) * ws, b.win_len,
                                  scoring=sc, chunk_pairs=chunk)
    finally:
        g.close()
    assert_same(got, want, True)


def _trace_line(capfd):
    return [ln for ln in capfd.readouterr().err.splitlines() if ln.startswith("[msw host]")][-1]


def _cache_counts(line):
    c = line.split("pinned_cache(")[1].split(")")[0]
    return int(c.split("hits=")[1].split()[0]), int(c.split("misses=")[1].split()[0])


def test_pinned_cache_lru_and_invalidation(fresh_ctx, oracle, monkeypatch, capfd):
    """the pinned-range cache is LRU over 16 ranges, so six pinned
    batches used in rotation (twelve ranges: reads and windows) all hit after
    the first round -- the 8-entry FIFO it replaces missed every one -- and
    msw_host_free empties it (a freed block's address may come back as
    pageable memory).  Results stay bit-exact throughout."""
    from mini_parallel_amd.aligner import pinned_empty
    monkeypatch.setenv("MSW_HOST_TRACE", "1")
    sc = Scoring()
    batches = []
    for k in range(6):
        b = config_batch(2, n_pairs=500, seed_offset=300 + k)
        pr, pw = pinned_empty(b.reads.shape, np.uint8), pinned_empty(b.wins.shape, np.uint8)
        pr[...] = b.reads
        pw[...] = b.wins
        batches.append((B(pr, b.read_len, pw, b.win_len), oracle_run(oracle, b, sc)))
    import gc
    gc.collect()  # no other test's pinned array freed (cache emptied) mid-test
    capfd.readouterr()
    for b, want in batches:  # first round: every range is new
        assert_same(gpu_run(fresh_ctx, b, sc), want, False)
    h0, m0 = _cache_counts(_trace_line(capfd))
    for b, want in batches * 2:  # later rounds: all hits
        assert_same(gpu_run(fresh_ctx, b, sc), want, False)
        assert "direct(reads=1 wins=1" in _trace_line(capfd)
    gpu_run(fresh_ctx, batches[0][0], sc)
    h1, m1 = _cache_counts(_trace_line(capfd))
    assert m1 == m0 and h1 - h0 == 2 * 12 + 2, (h0, m0, h1, m1)
    # any msw_host_free: the next lookups miss, and re-learn the ranges
    junk = pinned_empty(4096, np.uint8)
    del junk
    gc.collect()
    assert_same(gpu_run(fresh_ctx, batches[1][0], sc), batches[1][1], False)
    h2, m2 = _cache_counts(_trace_line(capfd))
    assert m2 == m1 + 2 and h2 == h1, (h1, m1, h2, m2)
