"""Multi-GPU helpers: one process per GPU, batch shards with no data-path
collective, and the final score/coordinate gather (north_star: RCCL over xGMI
"only for the final score/coord gather").  The same code runs on the `nccl`
(RCCL) backend on GPUs and on `gloo` for the CPU tests.

Every helper runs its collective whenever a process group is initialised,
whatever its size: bench.py creates an `nccl` group at N = 1 too, so the
driver's single-GPU run already executes the same RCCL calls (float64 MAX,
int64 SUM, all_gather of int32 / int64 and int16 cast to int32 on the wire)
that N = 8 does.  Without a group (library use in one process) they return
their inputs."""
from __future__ import annotations

import os
from collections import Counter

# Collectives this process has issued, by "op:dtype" (bench.py reports them
# beside the backend, so a record shows which RCCL calls actually ran).
CALLS: Counter = Counter()


def world() -> tuple:
    """(rank, world_size, local_rank) from the torch.distributed.run env."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def active() -> bool:
    """True when a process group exists: the helpers below then run their
    collective (at world size 1 too)."""
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def backend() -> str:
    """The process group's backend ("nccl" = RCCL on ROCm, "gloo"), or "none"."""
    import torch.distributed as dist
    return str(dist.get_backend()) if active() else "none"


def shard_range(n_total: int, rank: int, world_size: int) -> tuple:
    """Contiguous shard [a, b) of a global batch of n_total pairs."""
    a = n_total * rank // world_size
    b = n_total * (rank + 1) // world_size
    return a, b


def max_over_ranks(values, device=None):
    """Element-wise max of a list of floats over all ranks (timing)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if active():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        CALLS["all_reduce_max:float64"] += 1
    return [float(x) for x in t.tolist()]


def sum_over_ranks(values, device=None):
    """Element-wise sum of a list of integers over all ranks (work counts)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.int64, device=device)
    if active():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        CALLS["all_reduce_sum:int64"] += 1
    return [int(x) for x in t.tolist()]


def gather_results(*tensors):
    """Gather per-rank result tensors to every rank, concatenated in rank
    order.  The tensors of one call share one length on a rank; ranks may
    differ: shards are padded to the longest and trimmed after the
    all_gather (one collective per tensor)."""
    import torch
    import torch.distributed as dist
    if not active():
        return [t for t in tensors]
    ws = dist.get_world_size()
    dev = tensors[0].device
    n = torch.tensor([tensors[0].numel()], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(ws)]
    dist.all_gather(ns, n)
    CALLS["all_gather:int64"] += 1
    ns = [int(x.item()) for x in ns]
    mx = max(ns)
    if mx == 0:  # nothing on any rank
        return [t.reshape(-1)[:0].clone() for t in tensors]
    out = []
    for t in tensors:
        # neither RCCL nor gloo moves int16: ship 16-bit results as int32
        wire = torch.int32 if t.dtype in (torch.int16, torch.uint16) else t.dtype
        pad = torch.zeros(mx, dtype=wire, device=dev)
        pad[: t.numel()] = t.reshape(-1).to(wire)
        parts = [torch.zeros_like(pad) for _ in range(ws)]
        dist.all_gather(parts, pad)
        CALLS[f"all_gather:{str(t.dtype).replace('torch.', '')}" + ("->int32" if wire != t.dtype else "")] += 1
        out.append(torch.cat([p[:k] for p, k in zip(parts, ns)]).to(t.dtype))
    return out
