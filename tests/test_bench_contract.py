"""bench.py's one-line JSON contract, checked on a short GPU run.

The driver parses the last stdout line of `python bench.py`; this test runs a
reduced instance (fewer pairs, short CPU sample, no PCIe variants) and checks
the fields the contract and DESIGN.md section 5 promise: the BASELINE.json
metric, whole-job value consistent with ms_per_step, the roofline object
(frac = achieved / peak), the cpu_baseline object and bit-exact parity.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import LINE_LIMIT, compact_line  # noqa: E402


def test_compact_line_fits_the_driver_tail():
    """The one-line record of a full default run (round 4's, committed under
    profiles/) stays under LINE_LIMIT and keeps every leg's rate, parity,
    CPU baseline, VALU fraction and traffic ratio in its summary."""
    with open(os.path.join(ROOT, "profiles", "r04", "final5", "bench_default.json")) as f:
        full = json.load(f)
    line = compact_line(full, "gpurun_out/bench_detail_n1.json")
    assert len(json.dumps(line).encode()) <= LINE_LIMIT
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert line[k] == full[k] if k not in ("config", "roofline", "cpu_baseline") else line[k], k
    assert line["roofline"]["frac"] == full["roofline"]["frac"] and line["roofline"]["traffic"] > 0
    assert line["cpu_baseline"]["value"] == full["cpu_baseline"]["value"] and line["cpu_baseline"]["sample"]
    s = line["summary"]
    assert s["c2"]["bit_exact"] is True and s["c2"]["checked"] == 10000
    assert s["c3_hbm"]["valu_frac"] == full["configs_extra"]["config3"]["valu"]["frac"]
    assert s["c3_hbm"]["traffic_over_alg"] == 1.11 and s["c5_hbm"]["traffic_over_alg"] == 1.328
    assert s["c3_fastq"]["checked"] == 1_000_000 and s["c3_fastq"]["bit_exact"] is True
    assert s["c4"]["checked"] == 16 and s["c4"]["reads_per_s"] == full["configs_extra"]["config4"]["reads_per_s"]
    assert s["c3_h2h"]["bit_exact"] is True and s["pcie"]["submit_us"] == 57.6
    for leg in ("c2", "c3_hbm", "c5_hbm", "c4"):
        assert s[leg]["cpu_gcups"] > 0, leg


def test_fit_line_enforces_the_limit_at_run_time():
    """bench.fit_line: a line pushed over LINE_LIMIT by long
    error prose and phase splits is cut back under it, keeping every contract
    key and each leg's parity."""
    from bench import fit_line
    with open(os.path.join(ROOT, "profiles", "r04", "final5", "bench_default.json")) as f:
        full = json.load(f)
    line = compact_line(full, "gpurun_out/bench_detail_n1.json")
    for leg in line["summary"].values():
        if isinstance(leg, dict):
            leg["error"] = "x" * 900
            leg["setup_phases"] = {f"phase{k}": k for k in range(12)}
    assert len(json.dumps(line).encode()) > LINE_LIMIT
    out = fit_line(line)
    assert len(json.dumps(out).encode()) <= LINE_LIMIT
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "config", "roofline", "cpu_baseline"):
        assert k in out, k
    assert out["summary"]["c2"]["bit_exact"] is True and out["summary"]["c4"]["checked"] == 16


@pytest.mark.gpu
def test_bench_json_line(tmp_path):
    cmd = [sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--pairs", "2000",
           "--cpu-seconds", "1", "--no-pcie", "--c3-pairs", "20000", "--c5-pairs", "10000",
           "--c4-reads-per-file", "20000", "--c4-segment-reads", "10000", "--c4-pool", "3",
           "--c3-fastq-reads", "16000", "--c4-dir", str(tmp_path / "c4"),
           "--detail", str(tmp_path / "detail.json")]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    # the line fits the driver's output tail; every leg is in its summary
    assert len(lines[0].encode()) <= LINE_LIMIT, len(lines[0])
    summ = line["summary"]
    for leg in ("c2", "c3_hbm", "c3_h2h", "c3_fastq", "c4", "c5_hbm"):
        assert summ[leg]["bit_exact"] is True and summ[leg]["checked"] > 0, (leg, summ[leg])
    for leg in ("c2", "c3_hbm", "c5_hbm"):
        assert summ[leg]["cpu_gcups"] > 0 and 0 < summ[leg]["valu_frac"] < 1.5, (leg, summ[leg])
    assert summ["c3_fastq"]["checked"] == 16000 and summ["c4"]["checked"] == 16
    for k in ("roofline", "cpu_baseline", "parity", "valu"):
        assert line[k], k
    with open(tmp_path / "detail.json") as f:
        d = json.load(f)
    assert line["value"] == d["value"] and line["roofline"]["frac"] == d["roofline"]["frac"]
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert d["metric"] == base["metric"]
    assert d["unit"] == "GCUPS" and d["higher_is_better"] is True
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["scaling"] == "weak" and d["vs_baseline"] is None
    assert d["value"] > 0 and d["ms_per_step"] > 0
    cells = d["config"]["cells_per_gpu_step"]
    # value is cells per second over the timed steps (GCUPS); ms_per_step is rounded
    assert abs(d["value"] - cells / (d["ms_per_step"] * 1e-3) / 1e9) <= 0.05 * d["value"]
    roof = d["roofline"]
    assert roof["bound"] in ("hbm", "mfma") and roof["unit"] in ("GB/s", "TFLOP/s")
    assert roof["peak"] > 0 and roof["achieved"] > 0
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
    cpu = d["cpu_baseline"]
    assert cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["kind"] in ("port", "reference")
    assert cpu["sample"]
    assert d["parity"]["bit_exact"] is True and d["parity"]["mismatches"] == 0
    # VALU ceilings beside the instruction-mix one: SURVEY 8d's i32 ceiling
    # and the lone-wave bound, for the headline and configs 3 / 5
    for v in (d["valu"], d["configs_extra"]["config3"]["valu"], d["configs_extra"]["config5"]["valu"]):
        for k in ("frac", "frac_i32_ceiling", "frac_lone_wave"):
            assert 0 < v[k] < 1.5, (k, v[k])
        assert abs(v["frac_i32_ceiling"] - v["kernel_gcups"] / v["i32_ceiling_gcups"]) < 1e-3
    assert d["valu"]["i32_ceiling_gcups"] == pytest.approx(13107.2, abs=0.1)
    assert d["configs_extra"]["config3"]["valu"]["i32_ceiling_gcups"] == pytest.approx(6049.5, abs=0.1)
    ex = d["configs_extra"]
    for c in ("config3", "config5"):
        assert ex[c]["parity"]["bit_exact"] is True, c
    h = ex["config3"]["host_to_host"]
    assert h["equal_to_hbm_resident_run"] is True and h["value"] > 0 and h["chunk_pairs"] > 0
    c4 = ex["config4"]
    assert c4["parity"]["bit_exact"] is True and c4["reads"] == 16 * 20000
    assert c4["parity"]["files_checked"] == 16 and c4["parity"]["files_mismatched"] == []
    assert c4["reads_per_s"] >= c4["reads_per_s_incl_setup"] > 0 and c4["setup_ms"] > 0
    assert c4["setup_phases_ms"]["context_ms"] > 0 and c4["setup_phases_ms"]["hip_init_ms"] > 0
    sb = c4["setup_bound_by"]
    assert sb["phase"] in c4["setup_phases_ms"] and sb["ms"] == max(
        c4["setup_phases_ms"][k] for k in ("context_ms", "genome_ms", "result_sets_ms", "lane_reader_ms")) and sb["why"]
    assert c4["segments"]["segments_per_file"] == 2 and c4["segments"]["pool"] == 3
    # BASELINE config 3 from lane files: every per-read record against the oracle
    f3 = ex["config3"]["fastq"]
    assert f3["parity"]["bit_exact"] is True and f3["parity"]["records_checked"] == 16000
    assert f3["reads"] == 16000 and f3["reads_per_s"] > 0 and f3["setup_ms"] > 0
    # the CLI child's process wall, split
    for leg in (f3, c4):
        pp = leg["process_phases_ms"]
        assert pp["start_ms"] > 0 and pp["main_to_record_ms"] > 0 and pp["exit_ms"] >= 0, pp
        assert sum(pp.values()) <= leg["process_wall_ms"] + 2.0, (pp, leg["process_wall_ms"])
        assert leg["teardown_ms"] >= 0
    for leg in ("c3_fastq", "c4"):
        assert summ[leg]["setup_phases"]["context"] > 0 and "exit" in summ[leg]["process_phases"], summ[leg]
        assert summ[leg]["process_wall_ms"] > 0 and "teardown_ms" in summ[leg]
    assert summ["c3_fastq"]["distinct_reads"] == 16000
    # CPU baselines of the other configs' own work (BASELINE.md's plan)
    for leg in (ex["config3"], ex["config4"], ex["config5"]):
        cb = leg["cpu_baseline"]
        assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port" and cb["sample"], cb
    assert ex["config3"]["parity"]["rank0_cpu_sample"]["bit_exact"] is True
    # every max / sum / gather of the run went through RCCL, at N = 1 too
    col = d["collectives"]
    assert col["backend"] == "nccl" and col["world"] == 1
    for k in ("all_reduce_max:float64", "all_reduce_sum:int64", "all_gather:int64", "all_gather:int32",
              "all_gather:int16->int32"):
        assert col["calls_rank0"].get(k, 0) >= 1, (k, col)


@pytest.mark.gpu
def test_bench_more_gpus_than_visible_fails():
    """On the 1-GPU box `bench.py --gpus 2` must exit non-zero with a message
    (never a quiet n_gpus = 1 line)."""
    import torch
    n = torch.cuda.device_count()
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(max(n + 1, 2)), "--steps", "1", "--warmup", "0"],
                       cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) are visible" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


@pytest.mark.gpu
def test_bench_share_gpu_two_ranks(tmp_path):
    """The world > 1 GPU branches of bench.py on the one-GPU box (VERDICT r05,
    next 1): `--gpus 2 --share-gpu` starts two ranks that both run the real
    GPU path on device 0 -- set_device, Context, the HBM-resident legs, the
    host-to-host leg, each rank's own --full-wgs CLI child (MSW_DEVICES=0) on
    its own lane files, parity_sample over the real gathered shards -- with
    the collectives over gloo on host tensors (RCCL refuses two ranks on one
    device).  Every leg must be bit-exact with results gathered in shard
    order, and the line must say it is oversubscribed (never a scaling point).
    Anchor: gpu.rs:117,125 (the reference uses devices[0] only)."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--share-gpu", "--steps", "3", "--warmup", "1",
           "--pairs", "2000", "--cpu-seconds", "1", "--no-pcie", "--c3-pairs", "20000", "--c5-pairs", "10000",
           "--c4-reads-per-file", "20000", "--c4-segment-reads", "10000", "--c4-pool", "3",
           "--c3-fastq-reads", "16000", "--c4-dir", str(tmp_path / "c4"), "--detail", str(tmp_path / "detail.json")]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["oversubscribed"] is True
    assert line["collectives"]["backend"] == "gloo" and line["collectives"]["world"] == 2
    summ = line["summary"]
    for leg in ("c2", "c3_hbm", "c3_h2h", "c3_fastq", "c4", "c5_hbm"):
        assert summ[leg]["bit_exact"] is True and summ[leg]["checked"] > 0, (leg, summ[leg])
    with open(tmp_path / "detail.json") as f:
        d = json.load(f)
    assert d["oversubscribed"] is True and d["config"]["global_pairs"] == 4000
    assert d["gathered_scores"]["pairs"] == d["gathered_scores"]["pairs_expected"] == 4000
    # config 2: the gathered scores of BOTH shards against the oracle
    par = d["parity"]
    assert par["bit_exact"] is True and par["all_shards"]["bit_exact"] is True
    (lo0, hi0), (lo1, hi1) = par["all_shards"]["checked_ranges"]
    assert 0 <= lo0 < hi0 <= 2000 <= lo1 < hi1 <= 4000
    ex = d["configs_extra"]
    for c, per in (("config3", 20000), ("config5", 10000)):
        e = ex[c]
        assert e["n_ranks"] == 2 and e["gathered_pairs"] == 2 * per and e["parity"]["bit_exact"] is True, c
        (a0, b0), (a1, b1) = e["parity"]["checked_ranges"]
        assert 0 <= a0 < b0 <= per <= a1 < b1 <= 2 * per, c
    assert ex["config3"]["host_to_host"]["equal_to_hbm_resident_run"] is True
    # each rank's CLI child ran on GPU 0 over its own lane files (WGS_FILE_SHARD r/2)
    f3 = ex["config3"]["fastq"]["parity"]
    assert f3["bit_exact"] is True and f3["records_checked"] == 2 * 16000
    assert f3["files_by_rank"] == [[0, 2], [1, 3]] and f3["child_device_by_rank"] == [0, 0]
    c4 = ex["config4"]["parity"]
    assert c4["bit_exact"] is True and c4["files_once"] and c4["files_mismatched"] == []
    assert c4["files_by_rank"] == [list(range(0, 16, 2)), list(range(1, 16, 2))]
    assert c4["child_device_by_rank"] == [0, 0]
