"""RCCL on the MI355X: the collectives bench.py relies on,
run through mini_parallel_amd/dist.py on an `nccl` process group before the
driver's multi-GPU run depends on them.

One GPU box has one GPU, so the group has one rank: RCCL still builds a
communicator and runs every call (float64 MAX and int64 SUM all_reduce, the
int64 length exchange and the int32 / int64 / int16 -> int32 all_gathers of
gather_results, barriers).  The child process owns the group so that the
pytest process's own HIP state is untouched.  bench.py itself (which creates
an nccl group at N = 1 and runs every leg through it) is covered by
tests/test_bench_contract.py.
"""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent(r"""
    import datetime, json, socket, sys
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, sys.argv[1])
    from mini_parallel_amd import dist as mdist

    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            timeout=datetime.timedelta(minutes=2))
    out = {"backend": mdist.backend(), "active": mdist.active()}
    out["max"] = mdist.max_over_ranks([1.5, -2.25, 3e12], device=dev)
    out["sum"] = mdist.sum_over_ranks([7, -3, 2 ** 40], device=dev)
    rng = np.random.default_rng(5)
    s32 = torch.from_numpy(rng.integers(-2 ** 31, 2 ** 31 - 1, 4099, dtype=np.int64).astype(np.int32)).to(dev)
    s16 = torch.from_numpy(rng.integers(-2 ** 15, 2 ** 15 - 1, 4099).astype(np.int16)).to(dev)
    s64 = torch.from_numpy(rng.integers(-2 ** 62, 2 ** 62, 4099)).to(dev)
    g32, g16, g64 = mdist.gather_results(s32, s16, s64)
    out["gather_equal"] = [bool(torch.equal(a, b)) for a, b in ((g32, s32), (g16, s16), (g64, s64))]
    out["gather_dtypes"] = [str(t.dtype) for t in (g32, g16, g64)]
    (e,) = mdist.gather_results(torch.zeros(0, dtype=torch.int64, device=dev))
    out["empty"] = int(e.numel())
    dist.barrier()
    torch.cuda.synchronize()
    out["calls"] = dict(mdist.CALLS)
    dist.destroy_process_group()
    print(json.dumps(out))
""")


@pytest.mark.gpu
def test_rccl_collectives_world1():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["backend"] == "nccl" and d["active"] is True
    assert d["max"] == [1.5, -2.25, 3e12]
    assert d["sum"] == [7, -3, 2 ** 40]
    assert d["gather_equal"] == [True, True, True]
    assert d["gather_dtypes"] == ["torch.int32", "torch.int16", "torch.int64"]
    assert d["empty"] == 0
    # every collective bench.py uses went through RCCL
    for k in ("all_reduce_max:float64", "all_reduce_sum:int64", "all_gather:int64", "all_gather:int32",
              "all_gather:int16->int32"):
        assert d["calls"].get(k, 0) >= 1, (k, d["calls"])
