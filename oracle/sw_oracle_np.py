"""Independent numpy restatement of the scoring path (TEST INFRASTRUCTURE ONLY).

Written separately from ``oracle/sw_oracle.c`` so the two restatements check
each other.  Vectorised across pairs (the batch dimension), scalar over the DP
cells, so it finishes in seconds for a few thousand 150x300 pairs.

Follows:
  * smith_waterman.cl:5-7      scoring constants (+2 / -1 / gap 2)
  * smith_waterman.cl:112-126  intended linear recurrence (global max)
  * smith_waterman.cl:43,114   byte equality (case-sensitive, 'N' == 'N')
  * smith_waterman.cl:11-71 + aligner.rs:413-424   compat kernel (oracle_compat_np)

Parity status: "parity unpinned" against the reference itself (it has no
tests and no runnable SW implementation); pinned by the SURVEY.md 8(c)
known-answer table.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module.
"""
from __future__ import annotations

import numpy as np

NEG = -(1 << 28)


def sw_batch_np(reads, read_len, wins, win_len, match=2, mismatch=-1,
                gap_open=0, gap_extend=2, affine=False):
    """Score a padded SoA batch.

    reads: uint8 [B, Ms], wins: uint8 [B, Ns]; lengths int arrays [B].
    Returns (score int32[B], end_i int32[B], end_j int32[B]); coordinates are
    the first best cell in row-major order, (-1, -1) when the score is 0.
    ``affine=False`` is linear gap with penalty ``gap_extend``.
    """
    reads = np.asarray(reads, dtype=np.uint8)
    wins = np.asarray(wins, dtype=np.uint8)
    read_len = np.asarray(read_len, dtype=np.int64)
    win_len = np.asarray(win_len, dtype=np.int64)
    B = reads.shape[0]
    M = int(read_len.max()) if B else 0
    N = int(win_len.max()) if B else 0
    go = gap_open if affine else 0
    ge = gap_extend
    goe = go + ge
    best = np.zeros(B, np.int64)
    bi = np.full(B, -1, np.int64)
    bj = np.full(B, -1, np.int64)
    if B == 0 or M == 0 or N == 0:
        return best.astype(np.int32), bi.astype(np.int32), bj.astype(np.int32)
    Hprev = np.zeros((B, N + 1), np.int64)   # H[i-1][j-1] at index j
    Fprev = np.full((B, N + 1), NEG, np.int64)
    for i in range(M):
        row_ok = read_len > i
        Hcur = np.zeros((B, N + 1), np.int64)
        Fcur = np.full((B, N + 1), NEG, np.int64)
        E = np.full(B, NEG, np.int64)
        ri = reads[:, i] if i < reads.shape[1] else np.zeros(B, np.uint8)
        for j in range(N):
            col_ok = row_ok & (win_len > j)
            s = np.where(ri == wins[:, j], match, mismatch)
            E = np.maximum(E - ge, Hcur[:, j] - goe)
            F = np.maximum(Fprev[:, j + 1] - ge, Hprev[:, j + 1] - goe)
            h = np.maximum.reduce([Hprev[:, j] + s, E, F, np.zeros(B, np.int64)])
            h = np.where(col_ok, h, 0)
            E = np.where(col_ok, E, NEG)
            F = np.where(col_ok, F, NEG)
            Hcur[:, j + 1] = h
            Fcur[:, j + 1] = F
            upd = h > best
            best = np.where(upd, h, best)
            bi = np.where(upd, i, bi)
            bj = np.where(upd, j, bj)
        Hprev, Fprev = Hcur, Fcur
    return best.astype(np.int32), bi.astype(np.int32), bj.astype(np.int32)


def sw_pair_np(read: bytes, win: bytes, **kw):
    """Single pair convenience wrapper -> (score, end_i, end_j)."""
    m, n = len(read), len(win)
    r = np.zeros((1, max(m, 1)), np.uint8)
    w = np.zeros((1, max(n, 1)), np.uint8)
    r[0, :m] = np.frombuffer(read, np.uint8) if m else r[0, :0]
    w[0, :n] = np.frombuffer(win, np.uint8) if n else w[0, :0]
    s, i, j = sw_batch_np(r, [m], w, [n], **kw)
    return int(s[0]), int(i[0]), int(j[0])


def oracle_compat_np(s1: bytes, s2: bytes, wg: int = 1024, max_groups: int = 0) -> int:
    """smith_waterman_align (smith_waterman.cl:11-71) with gpu_align's geometry
    (aligner.rs:413-424), as a pure-Python loop for small inputs.
    ``max_groups`` replaces GPU_MAX_WORK_GROUPS (gpu.rs:10) when non-zero."""
    L = min(len(s1), len(s2))
    if L == 0:
        return 0
    W = wg
    G = min((L + W - 1) // W, max_groups or 1_000_000)
    C = (L + G - 1) // G
    res = 0
    for g in range(G):
        start = g * C
        if start >= L:
            continue
        end = min(start + C, L)
        for t in range(W):
            cur = best = 0
            for p in range(start + t, end, W):
                cur = max(cur + (2 if s1[p] == s2[p] else -1), 0)
                best = max(best, cur)
            res = max(res, best)
    return res
