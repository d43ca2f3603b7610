"""Control plane for one-reader-process-per-GPU runs.

[new] The reference is a single process.  Here each rank owns
one GPU (``LOCAL_RANK``) and its own node-local endpoint/objects; ranks only
exchange tiny control messages over RCCL (torch.distributed backend "nccl" is
RCCL on ROCm, riding xGMI within a node):

  R1/R2  start/stop barrier: all_reduce of one int32 on the rank's device,
         followed by torch.cuda.synchronize()  
  R3     stats reduce: one packed float64 vector, SUM/MAX/MIN all_reduces
  R4     per-rank table: all_gather of [p50, p99, MiB/s]

The data plane never crosses xGMI, so these are latency-bound (<1 KiB).
Without a GPU (CPU tests) the same calls run over gloo.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: object = None       # where control-plane tensors live (cuda:<gpu> for RCCL, cpu for gloo)
    gpu: int = -1               # this rank's HIP device, -1 without a GPU
    backend: str = "none"
    initialized_here: bool = False


def env_rank() -> tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def local_device(local_rank: int) -> int:
    """HIP device of a local rank: LOCAL_RANK on a full node (one rank per
    GPU).  More ranks than visible GPUs only happens in rehearsals
    (GCSB_DIST_BACKEND=gloo on a 1-GPU box) and wraps around."""
    import torch

    n = torch.cuda.device_count()
    return local_rank % n if n > 0 else -1


def init(local_rank: int | None = None, world: int | None = None, rank: int | None = None,
         backend: str | None = None, timeout_s: float = 600.0) -> DistContext:
    """backend None: "nccl" (RCCL) with a GPU, "gloo" without.  The
    GCSB_DIST_BACKEND env var overrides it (gloo rehearsals of N ranks on a
    box with fewer GPUs: RCCL rejects two ranks on one GPU)."""
    import torch
    import torch.distributed as dist

    r, w, lr = env_rank()
    rank = r if rank is None else rank
    world = w if world is None else world
    local_rank = lr if local_rank is None else local_rank
    ctx = DistContext(rank=rank, world=world, local_rank=local_rank)
    use_cuda = torch.cuda.is_available()
    backend = backend or os.environ.get("GCSB_DIST_BACKEND") or None
    if use_cuda:
        ctx.gpu = local_device(local_rank)
        torch.cuda.set_device(ctx.gpu)
        ctx.device = torch.device("cuda", ctx.gpu) if backend in (None, "nccl") else torch.device("cpu")
    else:
        ctx.device = torch.device("cpu")
    if world > 1:
        if backend is None:
            backend = "nccl" if use_cuda else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        if not dist.is_initialized():
            kw = {}
            if backend == "nccl" and use_cuda:
                kw["device_id"] = ctx.device
            dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
            ctx.initialized_here = True
        ctx.backend = backend
    return ctx


def barrier(ctx: DistContext) -> None:
    """R1/R2: RCCL all_reduce of one int32 + device sync (gloo on CPU)."""
    if ctx.world <= 1:
        return
    import torch
    import torch.distributed as dist

    t = torch.ones(1, dtype=torch.int32, device=ctx.device)
    dist.all_reduce(t)
    if ctx.gpu >= 0:
        torch.cuda.synchronize(ctx.gpu)
    if int(t.item()) != ctx.world:
        raise RuntimeError(f"barrier mismatch: {int(t.item())} != {ctx.world}")


def reduce_stats(ctx: DistContext, **vals: float) -> dict:
    """R3: returns {k_sum, k_max, k_min} for every value (+ per-rank list)."""
    import torch

    keys = sorted(vals)
    out: dict = {}
    if ctx.world <= 1:
        for k in keys:
            v = float(vals[k])
            out[k + "_sum"] = out[k + "_max"] = out[k + "_min"] = v
            out[k + "_per_rank"] = [v]
        return out
    import torch.distributed as dist

    base = torch.tensor([float(vals[k]) for k in keys], dtype=torch.float64, device=ctx.device)
    s, mx, mn = base.clone(), base.clone(), base.clone()
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(mn, op=dist.ReduceOp.MIN)
    gathered = [torch.zeros_like(base) for _ in range(ctx.world)]
    dist.all_gather(gathered, base)
    for i, k in enumerate(keys):
        out[k + "_sum"] = float(s[i])
        out[k + "_max"] = float(mx[i])
        out[k + "_min"] = float(mn[i])
        out[k + "_per_rank"] = [float(g[i]) for g in gathered]
    return out


def reduce_histogram(ctx: DistContext, buckets: list[int]) -> list[int]:
    """Sum the OpenCensus latency buckets over ranks (node-level view)."""
    if ctx.world <= 1:
        return list(buckets)
    import torch
    import torch.distributed as dist

    t = torch.tensor(buckets, dtype=torch.int64, device=ctx.device)
    dist.all_reduce(t)
    return [int(x) for x in t.tolist()]


def shutdown(ctx: DistContext) -> None:
    if ctx.world > 1 and ctx.initialized_here:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()
