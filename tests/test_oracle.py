"""The oracle pinned against the golden vectors (CPU only).

The reference ships no tests or fixtures for this path, so the
pins are the SURVEY.md 8(c) known-answer table plus two independent
restatements (C and numpy) that must agree with each other.
"""
import json
import os

import numpy as np
import pytest

from mini_parallel_amd.synthetic import make_pairs
from oracle.sw_oracle_np import oracle_compat_np, sw_batch_np, sw_pair_np

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load_kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def load_npz(name):
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    return {k: z[k] for k in z.files}, json.loads(str(z["meta"]))


@pytest.mark.parametrize("kat", load_kat()["linear_2_-1_2"], ids=lambda k: f"{k['read']}/{k['window']}")
def test_linear_kat(oracle, kat):
    r, w = kat["read"].encode(), kat["window"].encode()
    want = (kat["score"], kat["end_i"], kat["end_j"])
    assert sw_pair_np(r, w) == want
    R = np.zeros((1, 16), np.uint8)
    W = np.zeros((1, 16), np.uint8)
    R[0, :len(r)] = np.frombuffer(r, np.uint8) if r else []
    W[0, :len(w)] = np.frombuffer(w, np.uint8) if w else []
    s, i, j = oracle.sw_batch(R, [len(r)], W, [len(w)])
    assert (int(s[0]), int(i[0]), int(j[0])) == want
    # symmetric score under swapping read and window (SURVEY 8c property)
    assert sw_pair_np(w, r)[0] == want[0]


@pytest.mark.parametrize("kat", load_kat()["affine_2_-1_o3_e1"], ids=lambda k: f"{k['read']}/{k['window']}")
def test_affine_kat(oracle, kat):
    r, w = kat["read"].encode(), kat["window"].encode()
    want = (kat["score"], kat["end_i"], kat["end_j"])
    assert sw_pair_np(r, w, gap_open=3, gap_extend=1, affine=True) == want
    R = np.zeros((1, 16), np.uint8)
    W = np.zeros((1, 16), np.uint8)
    R[0, :len(r)] = np.frombuffer(r, np.uint8) if r else []
    W[0, :len(w)] = np.frombuffer(w, np.uint8) if w else []
    s, i, j = oracle.sw_batch(R, [len(r)], W, [len(w)], gap_open=3, gap_extend=1, affine=True)
    assert (int(s[0]), int(i[0]), int(j[0])) == want


@pytest.mark.parametrize("kat", load_kat()["compat"], ids=lambda k: f"{len(k['s1'])}-{k['wg']}-{k['max_groups']}")
def test_compat_kat(oracle, kat):
    s1, s2 = kat["s1"].encode(), kat["s2"].encode()
    assert oracle_compat_np(s1, s2, kat["wg"], kat["max_groups"]) == kat["expected"]
    assert oracle.compat_align(s1, s2, kat["wg"], kat["max_groups"]) == kat["expected"]


def test_compat_is_diagonal_indicator(oracle):
    """With the reference geometry (W=1024, G=ceil(L/W)) the launched kernel
    returns 2 iff some position matches."""
    rng = np.random.default_rng(3)
    for L in (1, 7, 1000, 4097):
        a = bytes(rng.choice(np.frombuffer(b"AC", np.uint8), L))
        b = bytes(np.where(np.frombuffer(a, np.uint8) == ord("A"), ord("C"), ord("A")).astype(np.uint8))
        assert oracle.compat_align(a, b, 1024) == 0
        assert oracle.compat_align(a, a, 1024) == 2


@pytest.mark.parametrize("name", ["linear_150x300.npz", "affine_150x300.npz", "mixed_linear.npz"])
def test_golden_batches(oracle, name):
    d, meta = load_npz(name)
    kw = dict(match=meta["match"], mismatch=meta["mismatch"], gap_open=meta.get("gap_open", 0),
              gap_extend=meta["gap_extend"], affine=meta["affine"])
    s, i, j = oracle.sw_batch(d["reads"], d["read_len"], d["wins"], d["win_len"], threads=4, **kw)
    assert np.array_equal(s, d["score"])
    assert np.array_equal(i, d["end_i"]) and np.array_equal(j, d["end_j"])


@pytest.mark.parametrize("affine", [False, True])
def test_c_vs_numpy_random(oracle, affine):
    """Edge-heavy random batch: tiny alphabets, empty and ragged lengths."""
    rng = np.random.default_rng(5 + affine)
    B = 200
    R = rng.choice(np.frombuffer(b"ACN", np.uint8), (B, 40)).astype(np.uint8)
    W = rng.choice(np.frombuffer(b"ACNa", np.uint8), (B, 70)).astype(np.uint8)
    rl = rng.integers(0, 41, B).astype(np.uint16)
    wl = rng.integers(0, 71, B).astype(np.uint16)
    kw = dict(gap_open=2 if affine else 0, gap_extend=1 if affine else 2, affine=affine)
    a = oracle.sw_batch(R, rl, W, wl, **kw)
    b = sw_batch_np(R, rl, W, wl, **kw)
    for x, y in zip(a, b):
        assert np.array_equal(x.astype(np.int32), y)


def test_linear_equals_affine_open0(oracle):
    b = make_pairs(64, 60, 2.0, seed=9)
    lin = oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len)
    aff = oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, gap_open=0, gap_extend=2, affine=True)
    for x, y in zip(lin, aff):
        assert np.array_equal(x, y)


def test_threads_do_not_change_results(oracle):
    b = make_pairs(97, 50, 2.0, seed=10)
    one = oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, threads=1)
    many = oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, threads=7)
    for x, y in zip(one, many):
        assert np.array_equal(x, y)


@pytest.mark.skipif(not os.path.exists("/root/reference/smith_waterman/src/smith_waterman.cl"),
                    reason="reference sources absent (the GPU box uses the prebuilt oracle/_ref)")
def test_reference_kernel_object_built():
    """`make -C oracle ref` compiles the reference's own OpenCL kernels for
    gfx950 (the checker tests/test_gpu_reference_kernel.py runs on the box)."""
    import subprocess
    from oracle import ref_cl
    subprocess.run(["make", "-C", os.path.dirname(ref_cl.__file__), "-s", "ref"], check=True)
    assert ref_cl.available()
    data = open(ref_cl.CO, "rb").read()
    assert data[:4] == b"\x7fELF" and b"smith_waterman_align" in data and b"smith_waterman_detailed" in data


@pytest.mark.parametrize("affine", [False, True])
@pytest.mark.parametrize("coords", [False, True])
def test_simd_baseline_bit_exact(oracle, affine, coords):
    """The SIMD CPU baseline (bench.py cpu_baseline) equals the scalar oracle:
    mixed lengths incl. empty pairs, a ragged last group, several schemes."""
    from mini_parallel_amd.synthetic import make_pairs
    b = make_pairs(1000 + 13, (0, 200), 1.7, seed=404 + affine, read_stride=208, win_stride=352)
    for match, mis, go, ge in ((2, -1, 3 if affine else 0, 1 if affine else 2), (5, -4, 10, 3), (1, 0, 0, 1),
                               (64, 0, 30000, 1024), (3, -61, 7, 0)):
        want = oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, match=match, mismatch=mis, gap_open=go,
                               gap_extend=ge, affine=affine, threads=4)
        s, i, j, isa = oracle.sw_batch_simd(b.reads, b.read_len, b.wins, b.win_len, match=match, mismatch=mis,
                                            gap_open=go, gap_extend=ge, affine=affine, threads=3, coords=coords)
        assert np.array_equal(s, want[0]), (match, mis, go, ge, isa)
        if coords:
            assert np.array_equal(i, want[1]) and np.array_equal(j, want[2])
