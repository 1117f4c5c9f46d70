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


@pytest.mark.gpu
def test_bench_json_line():
    cmd = [sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--pairs", "2000",
           "--cpu-seconds", "1", "--no-pcie"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
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
