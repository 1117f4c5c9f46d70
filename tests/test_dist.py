"""World-size-2 gloo test of the multi-GPU control flow (CPU only): batch
sharding, max-over-ranks timing and the final result gather."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mini_parallel_amd import dist as mdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", init_method="env://")
    a, b = mdist.shard_range(n_total, rank, world)
    # stand-in for the per-rank scores: a deterministic function of the pair index
    scores = torch.arange(a, b, dtype=torch.int32) * 3 + 1
    ei = torch.arange(a, b, dtype=torch.int16) % 7
    t = mdist.max_over_ranks([1.0 + rank, 5.0 - rank])
    cells = mdist.sum_over_ranks([b - a, 10 ** 12 + rank])
    g_scores, g_ei = mdist.gather_results(scores, ei)
    if rank == 0:
        np.save(os.path.join(out_dir, "scores.npy"), g_scores.numpy())
        np.save(os.path.join(out_dir, "ei.npy"), g_ei.numpy())
        np.save(os.path.join(out_dir, "t.npy"), np.array(t))
        np.save(os.path.join(out_dir, "cells.npy"), np.array(cells, dtype=np.int64))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [10, 10_001])
def test_gloo_world2_shard_and_gather(tmp_path, n_total):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), n_total, str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    scores = np.load(tmp_path / "scores.npy")
    ei = np.load(tmp_path / "ei.npy")
    assert np.array_equal(scores, np.arange(n_total, dtype=np.int32) * 3 + 1)
    assert np.array_equal(ei, (np.arange(n_total) % 7).astype(np.int16))
    assert list(np.load(tmp_path / "t.npy")) == [2.0, 5.0]
    assert list(np.load(tmp_path / "cells.npy")) == [n_total, 2 * 10 ** 12 + 1]


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 7, 10_000, 1_000_003):
        for w in (1, 2, 3, 8):
            rs = [mdist.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1
