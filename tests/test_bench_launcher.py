"""bench.py's multi-rank path on the CPU (gloo, world size 2).

The driver runs ``python -m torch.distributed.run --nproc-per-node N bench.py
--gpus N`` (and a plain ``python bench.py --gpus N`` must start N ranks
itself).  With ``--cpu-standin`` the ranks use gloo and a stand-in scorer, so
these tests check the launcher, the sharding of ONE global batch, the
max-over-ranks / sum-over-ranks bookkeeping and the ordered gather without a
GPU.  Without a GPU, asking for 2 GPUs must fail loudly (exit status 3).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import standin_scores  # noqa: E402
from mini_parallel_amd.synthetic import config_shard  # noqa: E402

ARGS = ["--cpu-standin", "--steps", "2", "--warmup", "1", "--pairs", "3000", "--cpu-seconds", "0",
        "--no-pcie", "--extra-configs", ""]


def _env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _json_line(out):
    """The full record (the detail file the one-line record names), with the
    line itself under "_line"; the line's own summary is checked here."""
    lines = [l for l in out.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    line = json.loads(lines[0])
    path = line["detail"]
    with open(path if os.path.isabs(path) else os.path.join(ROOT, path)) as f:
        full = json.load(f)
    for k in ("metric", "value", "n_gpus", "steps", "warmup", "config", "roofline", "collectives"):
        assert k in line, k
    assert line["summary"]["c2"]["gcups"] == full["value"]
    full["_line"] = line
    return full


def _check(d, world, per_gpu=3000):
    assert d["n_gpus"] == world
    assert d["config"]["global_pairs"] == per_gpu * world
    assert d["gathered_scores"]["pairs"] == per_gpu * world
    want = standin_scores(config_shard(2, 0, per_gpu * world))
    got = np.array(d["standin_scores"], dtype=np.int32)
    assert np.array_equal(got, want), "gather out of order or shards overlap"
    assert d["config"]["cells_per_job_step"] == config_shard(2, 0, per_gpu * world).cells


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_self_launch_two_ranks(tmp_path):
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"] + ARGS + ["--detail", str(tmp_path / "d.json")],
                       cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    _check(_json_line(r.stdout), 2)


def test_torchrun_two_ranks(tmp_path):
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2"]
                       + ARGS + ["--detail", str(tmp_path / "d.json")],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    _check(_json_line(r.stdout), 2)


def test_single_rank_standin(tmp_path):
    r = subprocess.run([sys.executable, "bench.py"] + ARGS + ["--detail", str(tmp_path / "d.json")],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    _check(_json_line(r.stdout), 1)


EXTRA = ["--cpu-standin", "--steps", "1", "--warmup", "0", "--pairs", "1000", "--cpu-seconds", "0", "--no-pcie",
         "--extra-configs", "3,4,5", "--c3-pairs", "1500", "--c5-pairs", "1300", "--c4-reads-per-file", "120",
         "--c4-segment-reads", "40", "--c4-pool", "5", "--c3-fastq-reads", "320"]


def _check_extras(d, world):
    """configs_extra at N = world: configs 3 / 5 sharded over the ranks and
    gathered in order, config 4's lane files sharded by file (each exactly
    once) with the per-file rows gathered and file 0 recomputed."""
    ex = d["configs_extra"]
    for c, per in (("config3", 1500), ("config5", 1300)):
        e = ex[c]
        assert e["n_ranks"] == world and e["global_pairs"] == per * world and e["gathered_pairs"] == per * world
        assert e["parity"]["gather_in_order"] is True, c
        assert e["valu"]["frac_i32_ceiling"] >= 0 and e["valu"]["frac_lone_wave"] >= 0
    c4 = ex["config4"]
    assert c4["n_ranks"] == world and c4["files_per_rank"] == 16 // world and c4["scaling"] == "strong"
    p = c4["parity"]
    assert p["files_once"] and p["files_done"] == 16 and p["reads"] == p["reads_expected"] == 16 * 120
    assert p["file0_ok"] is True and p["rows_ok"] is True and p["files_checked"] == 16
    assert p["files_by_rank"] == [list(range(r, 16, world)) for r in range(world)] and p["files_sharded_as_cli"]
    assert c4["reads_per_s"] > 0 and c4["gcups"] > 0
    assert c4["segments"] == {**c4["segments"], "pool": 5, "segment_reads": 40, "segments_per_file": 3}
    f3 = ex["config3"]["fastq"]  # per-read records of 2N lane files, gathered in file order
    assert f3["n_ranks"] == world and f3["reads"] == 320 * world and f3["scaling"] == "weak"
    assert f3["parity"]["bit_exact"] is True and f3["parity"]["records_checked"] == 320 * world
    assert f3["parity"]["files_by_rank"] == [[r, r + world] for r in range(world)]
    # one rank's two lane files generated and scored, byte-identical copies for the rest
    ds = f3["dataset"]
    assert ds["files_generated"] == 2 and ds["files_copied"] == 2 * world - 2, ds
    assert ds["distinct_reads"] == 320 and ds["cells"] > 0
    # config 4's lane set does not depend on N: 16 files of 3 pooled segments
    assert c4["dataset"]["segments_total"] == 5 and c4["parity"]["reads_expected"] == 16 * 120
    col = d["collectives"]
    assert col["backend"] == "gloo" and col["world"] == world and col["calls_rank0"]["all_gather:int16->int32"] >= 1


@pytest.mark.parametrize("launch", ["self", "torchrun"])
def test_two_ranks_run_every_config(tmp_path, launch):
    args = EXTRA + ["--c4-dir", str(tmp_path / "c4"), "--detail", str(tmp_path / "d.json")]
    if launch == "self":
        cmd = [sys.executable, "bench.py", "--gpus", "2"] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2"] + args
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    _check(d, 2, per_gpu=1000)
    _check_extras(d, 2)


def test_eight_ranks_run_every_config(tmp_path):
    """The driver's largest N: 8 ranks (gloo stand-in), every leg sharded and
    gathered -- config 4's 16 lane files two per rank, config 3's FASTQ lane
    per rank, configs 3 / 5 in order."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8"] + EXTRA + ["--c4-dir", str(tmp_path / "c4"),
                                                                     "--detail", str(tmp_path / "d.json")],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    _check(d, 8, per_gpu=1000)
    _check_extras(d, 8)


def test_one_rank_runs_every_config(tmp_path):
    r = subprocess.run([sys.executable, "bench.py"] + EXTRA + ["--c4-dir", str(tmp_path / "c4"),
                                                               "--detail", str(tmp_path / "d.json")], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    _check_extras(d, 1)
    v = d["valu"]
    for k in ("frac", "frac_i32_ceiling", "frac_lone_wave"):  # a CPU stand-in rate: tiny, present
        assert v[k] >= 0, k
    assert v["ceiling_gcups"] > v["lone_wave_ceiling_gcups"] > 0 and v["i32_ceiling_gcups"] > 0
    assert v["i32_ceiling_gcups"] == pytest.approx(13107.2, abs=0.1)  # 13.1 TCUPS linear


def test_shards_of_one_global_batch():
    """Pair i of the global batch is the same whichever range generates it."""
    whole = config_shard(5, 0, 2500)
    for a, b in ((0, 1), (1000, 1100), (1023, 1025), (2048, 2500)):
        s = config_shard(5, a, b)
        assert np.array_equal(s.reads, whole.reads[a:b]) and np.array_equal(s.wins, whole.wins[a:b])
        assert np.array_equal(s.read_len, whole.read_len[a:b])
    assert config_shard(2, 7, 7).n_pairs == 0


def test_too_few_gpus_fails_loudly():
    """--gpus larger than the visible GPU count: non-zero exit and a message,
    never a quiet n_gpus = 1 line (here: no GPU at all; on a 1-GPU box the
    GPU variant in test_bench_contract.py asks for 2)."""
    import torch
    n = torch.cuda.device_count()
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(max(n + 1, 2)), "--steps", "1", "--warmup", "0"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) are visible" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("cfg,world", [(2, 2), (5, 3)])
def test_parity_sample_covers_every_shard(cfg, world):
    """bench.parity_sample (rank 0, N > 1, GPU runs): the sample it checks
    comes from every rank's shard of the global batch, and it flags a wrong
    score in any of them -- checked here with the oracle's own scores standing
    in for the gathered GPU results."""
    import bench
    from oracle import oracle_lib
    from mini_parallel_amd import dist as mdist
    n_total = 700 * world
    sc = bench.scoring_of(cfg)
    b = config_shard(cfg, 0, n_total)
    s, i, j, _ = oracle_lib.sw_batch_simd(b.reads, b.read_len, b.wins, b.win_len, threads=4,
                                          coords=sc.want_coords, **bench._oracle_kw(sc))
    par = bench.parity_sample(cfg, sc, n_total, world, s, i, j, per_shard=64)
    assert par["bit_exact"] and par["checked_pairs"] == 64 * world
    for (lo, hi), r in zip(par["checked_ranges"], range(world)):
        a, bb = mdist.shard_range(n_total, r, world)
        assert a <= lo < hi <= bb
    lo, _ = par["checked_ranges"][-1]
    bad = s.copy()
    bad[lo] += 1  # one wrong score in the last shard's sample
    assert bench.parity_sample(cfg, sc, n_total, world, bad, i, j, per_shard=64)["mismatches"] == 1
