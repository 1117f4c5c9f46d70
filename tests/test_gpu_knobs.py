"""Every environment knob the product still reads, exercised on the GPU (the
other knobs are covered where their paths are tested: MSW_LAYOUT /
MSW_GROUP_LANES / MSW_NO_MULTI / MSW_NO_F16 in test_gpu_parity.py,
MSW_FORCE_LONG / MSW_LONG_BLOCKS in test_gpu_long.py, MSW_HOST_TRACE in
test_gpu_genome.py, the MSW_GZ_* reader knobs in test_gpu_gz.py, MSW_DEVICES /
MSW_GPU_INFLATE / MSW_GFASTQ_BATCH / MSW_GFASTQ_SPAN_MB / MSW_MAX_READ_LEN in
test_cli.py; INTEGRATION.md lists them all).  Tracing knobs must not change
results; tuning knobs must not change results either.  The library reads
its knobs once, when a context (or a GPU lane reader) is made: tests that
set one use a context of their own."""
import json
import os
import re
import subprocess
import sys
import textwrap

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "mini_parallel_amd", "rustseq_mini")


def _wgs(tmp_path, oracle, lanes=2, reads=1200):
    from mini_parallel_amd.synthetic import write_wgs_dataset
    ds = write_wgs_dataset(str(tmp_path / "wgs"), lanes=lanes, reads_per_lane=2, reads_per_file=reads, bgzf=True)
    want = sum(int(oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, threads=8)[0].astype(np.int64).sum())
               for b in ds["batches"])
    return ds, want


def _run_cli(tmp_path, ds, extra_env, tag):
    env = dict(os.environ, WGS_DATA_DIR=str(tmp_path / "wgs"), WGS_SAMPLE_ID="SYN", WGS_LANES="2",
               WGS_READS_PER_LANE="2", GPU_CHUNK_SIZE_READS="500", WGS_RUN_ID=f"knob_{tag}", **extra_env)
    rec = tmp_path / f"rec_{tag}.json"
    r = subprocess.run([CLI, "--full-wgs", "--gpu", "--score-mode", "sw", "--reference", ds["reference"], "--window",
                        "300", "--checkpoint-dir", str(tmp_path), "--json", str(rec)], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return json.load(open(rec)), r.stderr


@pytest.mark.gpu
def test_gpu_reader_traces(tmp_path, oracle):
    """MSW_GFASTQ_TRACE (per-span phase times), MSW_GZ_TIMING (inflate /
    CRC kernel times) and MSW_CLI_TRACE (the CLI's per-batch arrival, submit
    and settle times) print their lines; the sums stay the oracle's."""
    ds, want = _wgs(tmp_path, oracle)
    rec, err = _run_cli(tmp_path, ds, {"MSW_GPU_INFLATE": "1", "MSW_GFASTQ_TRACE": "1", "MSW_GZ_TIMING": "1",
                                       "MSW_CLI_TRACE": "1"}, "tr")
    assert rec["gpu_inflate"] is True and rec["total_score"] == want
    assert "[gfastq]" in err and "span:" in err
    assert "[gz]" in err and "inflate" in err and "crc" in err
    assert "[cli trace] worker" in err and "submitted" in err and "settled" in err


@pytest.mark.gpu
def test_host_reader_threads(tmp_path, oracle):
    """MSW_HOST_THREADS (the CLI's CPU share: reader threads and, with fewer
    files than threads, the BGZF inflate threads per file): 1 and 3 give the
    oracle's sums through the host reader."""
    ds, want = _wgs(tmp_path, oracle)
    for n in ("1", "3"):
        rec, _ = _run_cli(tmp_path, ds, {"MSW_GPU_INFLATE": "0", "MSW_HOST_THREADS": n}, f"ht{n}")
        assert rec["gpu_inflate"] is False and rec["total_score"] == want
        assert rec["host_threads"] == int(n)


CHILD = textwrap.dedent(r"""
    import json, os, sys
    import numpy as np
    sys.path.insert(0, sys.argv[1])
    import torch
    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd.synthetic import config_batch
    b = config_batch(2, n_pairs=3000, seed_offset=9)
    ctx = Context(0)
    s, i, j = ctx.align_batch(b.reads, b.read_len, b.wins, b.win_len, Scoring(want_coords=True), chunk_pairs=1000)
    dev = torch.device("cuda", 0)
    t = lambda a, dt=None: torch.from_numpy(np.ascontiguousarray(a if dt is None else a.view(dt))).to(dev)
    r, w, rl, wl = t(b.reads), t(b.wins), t(b.read_len, np.int16), t(b.win_len, np.int16)
    out = torch.zeros(b.n_pairs, dtype=torch.int32, device=dev)
    ctx.align_batch_device(r.data_ptr(), rl.data_ptr(), w.data_ptr(), wl.data_ptr(), b.reads.shape[1],
                           b.wins.shape[1], b.n_pairs, out.data_ptr(), int(b.read_len.max()), int(b.win_len.max()),
                           Scoring())
    torch.cuda.synchronize()
    np.savez(sys.argv[2], s=s, i=i, j=j, d=out.cpu().numpy())
    ctx.close()
""")


@pytest.mark.gpu
def test_library_traces(tmp_path, oracle):
    """MSW_HOST_TRACE (per-call host phase times) and MSW_WAVE_TRACE
    (per-wave records of a device launch, tools/wave_trace.py) leave the
    scores as the oracle's; the trace lands where it should."""
    trace = tmp_path / "waves.bin"
    env = dict(os.environ, MSW_HOST_TRACE="1", MSW_WAVE_TRACE=str(trace))
    out = tmp_path / "res.npz"
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(out)], env=env, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    assert re.search(r"\[msw host\] pairs=3000 chunks=[2-9] ", r.stderr), r.stderr[-2000:]
    from mini_parallel_amd.synthetic import config_batch
    b = config_batch(2, n_pairs=3000, seed_offset=9)
    ws, wi, wj = oracle.sw_batch(b.reads, b.read_len, b.wins, b.win_len, threads=8)
    z = np.load(out)
    assert np.array_equal(z["s"], ws) and np.array_equal(z["i"], wi) and np.array_equal(z["j"], wj)
    assert np.array_equal(z["d"], ws)
    raw = np.fromfile(trace, dtype=np.uint64)
    assert raw.size >= 2
    n_blocks = int(raw[0])
    assert n_blocks >= 1 and raw.size >= 2 + 4 * n_blocks
    blk = raw[2:2 + 4 * n_blocks].reshape(n_blocks, 4)
    assert (blk[:, 1] >= blk[:, 0]).all() and (blk[:, 1] != 0).any()  # end >= start, blocks recorded
