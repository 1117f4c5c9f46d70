"""Regenerate the committed golden fixtures (run from the repo root):

    python tests/golden/make_golden.py

Inputs are seeded synthetic pairs (mini_parallel_amd.synthetic) plus the
hand-written known-answer table of SURVEY.md 8(c).  Expected outputs come from
the C oracle (oracle/sw_oracle.c) and are cross-checked here against the
independent numpy restatement (oracle/sw_oracle_np.py); the script refuses to
write a fixture on any disagreement.  The reference itself cannot be run here
(Rust host, no toolchain; its SW kernel is dead code), so these fixtures are
the parity anchor ("parity unpinned" against the reference).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from mini_parallel_amd.synthetic import make_pairs  # noqa: E402
from oracle import oracle_lib  # noqa: E402
from oracle.sw_oracle_np import oracle_compat_np, sw_batch_np, sw_pair_np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

# SURVEY.md 8(c) known-answer table, linear +2/-1/-2: (read, window, (score, i, j)).
KAT_LINEAR = [
    ("ACGT", "ACGT", (8, 3, 3)),
    ("ACGT", "TTACGTTT", (8, 3, 5)),
    ("AAAA", "CCCC", (0, -1, -1)),
    ("ACGTACGT", "ACGACGT", (12, 7, 6)),
    ("GATTACA", "GCATGCU", (4, 2, 3)),
    ("TTTACGTAAA", "ACGT", (8, 6, 3)),
    ("ACCA", "ACA", (4, 1, 1)),
    ("N", "N", (2, 0, 0)),
    ("acgt", "ACGT", (0, -1, -1)),
    ("", "ACGT", (0, -1, -1)),
]


def cross_checked(batch, **kw):
    s, i, j = oracle_lib.sw_batch(batch.reads, batch.read_len, batch.wins, batch.win_len, **kw)
    s2, i2, j2 = sw_batch_np(batch.reads, batch.read_len, batch.wins, batch.win_len, **kw)
    assert np.array_equal(s, s2), "C oracle and numpy restatement disagree on scores"
    assert np.array_equal(i.astype(np.int32), i2) and np.array_equal(j.astype(np.int32), j2), \
        "C oracle and numpy restatement disagree on coordinates"
    return s, i, j


def save_npz(name, batch, s, i, j, **meta):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, reads=batch.reads, read_len=batch.read_len, wins=batch.wins,
                        win_len=batch.win_len, score=s, end_i=i, end_j=j,
                        meta=np.array(json.dumps(meta)))
    print("wrote", path, os.path.getsize(path), "bytes")


def main():
    oracle_lib.build()
    # 1. KATs: check both restatements against the survey table, store it.
    kats = []
    for r, w, want in KAT_LINEAR:
        got = sw_pair_np(r.encode(), w.encode())
        assert got == want, (r, w, got, want)
        kats.append({"read": r, "window": w, "score": want[0], "end_i": want[1], "end_j": want[2]})
    # affine KATs (go=3, ge=1) from the two restatements
    aff = []
    for r, w in [("ACGTTTACGT", "ACGTACGT"), ("ACGTACGTAC", "ACGTTTTTACGTAC"), ("GGGG", "GGAGG"),
                 ("ACGT", "ACGT"), ("A", "C"), ("", "")]:
        a = sw_pair_np(r.encode(), w.encode(), gap_open=3, gap_extend=1, affine=True)
        aff.append({"read": r, "window": w, "score": a[0], "end_i": a[1], "end_j": a[2]})
    # compat KATs: smith_waterman_align semantics
    rng = np.random.default_rng(7)
    rnd = lambda n: bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), n))  # noqa: E731
    x1000, y1000 = rnd(1000), rnd(1000)
    compat = [
        {"s1": "ACGTACGT", "s2": "ACGTACGT", "wg": 1024, "max_groups": 0},
        {"s1": "AAAA", "s2": "CCCC", "wg": 1024, "max_groups": 0},
        {"s1": "", "s2": "ACGT", "wg": 1024, "max_groups": 0},
        {"s1": x1000.decode(), "s2": y1000.decode(), "wg": 64, "max_groups": 3},
        {"s1": x1000.decode(), "s2": x1000.decode(), "wg": 64, "max_groups": 3},
        {"s1": x1000.decode(), "s2": y1000.decode(), "wg": 1024, "max_groups": 0},
    ]
    for c in compat:
        c["expected"] = oracle_compat_np(c["s1"].encode(), c["s2"].encode(), c["wg"], c["max_groups"])
        assert c["expected"] == oracle_lib.compat_align(c["s1"].encode(), c["s2"].encode(), c["wg"],
                                                        c["max_groups"])
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump({"linear_2_-1_2": kats, "affine_2_-1_o3_e1": aff, "compat": compat}, f, indent=1)
    print("wrote kat.json")

    # 2. Seeded batches (config-2 shape, affine config-3 shape, mixed config-5 shape).
    b = make_pairs(384, 150, 2.0, seed=11002, read_stride=160, win_stride=304)
    save_npz("linear_150x300.npz", b, *cross_checked(b), match=2, mismatch=-1, gap_extend=2,
             affine=False, seed=11002)
    b = make_pairs(256, 150, 2.0, seed=11003, read_stride=160, win_stride=304)
    save_npz("affine_150x300.npz", b, *cross_checked(b, gap_open=3, gap_extend=1, affine=True),
             match=2, mismatch=-1, gap_open=3, gap_extend=1, affine=True, seed=11003)
    b = make_pairs(256, (0, 250), 2.0, seed=11005, read_stride=256, win_stride=512)
    save_npz("mixed_linear.npz", b, *cross_checked(b), match=2, mismatch=-1, gap_extend=2,
             affine=False, seed=11005)


if __name__ == "__main__":
    main()
