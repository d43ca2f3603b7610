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
import sys
import threading
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
    pg: bool = False            # a process group exists (collectives run even at world 1)
    fallback: bool = False      # RCCL failed to initialise; the control plane runs on gloo
    guard_groups: dict = None   # gloo subgroups with a collective timeout of their own, by timeout


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


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def init(local_rank: int | None = None, world: int | None = None, rank: int | None = None,
         backend: str | None = None, timeout_s: float = 600.0, always_pg: bool = False) -> DistContext:
    """backend None: "nccl" (RCCL) with a GPU, "gloo" without.  The
    GCSB_DIST_BACKEND env var overrides it (gloo rehearsals of N ranks on a
    box with fewer GPUs: RCCL rejects two ranks on one GPU).

    always_pg: create the process group at world 1 too, so a 1-GPU run still
    initialises an RCCL communicator and every barrier / reduction below goes
    through it (the bench does this: the R0-R4 path then runs on MI355X in
    every 1-GPU run, not only on an 8-GPU node)."""
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
    if world > 1 or always_pg:
        if backend is None:
            backend = "nccl" if use_cuda else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()) if world == 1 else "29512")
        if not dist.is_initialized():
            kw = {}
            if backend == "nccl" and use_cuda:
                kw["device_id"] = ctx.device
            if os.environ.get("GCSB_INIT_METHOD"):
                # e.g. file:///tmp/x: a rendezvous with no TCP port to race
                # for (tests that run beside others under pytest-xdist)
                kw["init_method"] = os.environ["GCSB_INIT_METHOD"]
            explicit = os.environ.get("GCSB_DIST_BACKEND")
            try:
                dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                        timeout=datetime.timedelta(seconds=timeout_s), **kw)
            except Exception as e:  # noqa: BLE001
                if backend != "nccl" or explicit:
                    raise
                # RCCL refused to initialise (same on every rank, e.g. no
                # peer-memory IPC on the host): keep the run alive on a gloo
                # control plane (CPU tensors) at the next port, and say so
                sys.stderr.write(f"[rank {rank}] RCCL init failed ({type(e).__name__}: {e}); "
                                 f"falling back to a gloo control plane\n")
                if dist.is_initialized():
                    dist.destroy_process_group()
                os.environ["MASTER_PORT"] = str(int(os.environ["MASTER_PORT"]) + 1)
                backend = "gloo"
                ctx.device = torch.device("cpu")
                ctx.fallback = True
                dist.init_process_group(backend="gloo", rank=rank, world_size=world,
                                        timeout=datetime.timedelta(seconds=timeout_s))
            ctx.initialized_here = True
        ctx.backend = backend
        ctx.pg = True
        if backend == "gloo" and world > 1:
            # while every rank is alive: new_group itself is a collective
            _timed_group(ctx, collective_timeout_s())
    return ctx


def collective_timeout_s() -> float:
    """Guarded collectives (the fan-out all-gather) give up after this
    (GCSB_COLLECTIVE_TIMEOUT_S, default 120 s)."""
    return float(os.environ.get("GCSB_COLLECTIVE_TIMEOUT_S", "120"))


_fatal_hooks: list = []


def on_fatal(fn) -> None:
    """Run fn() before a barrier watchdog ends the process (the bench prints
    the headline line it has measured so far)."""
    _fatal_hooks.append(fn)


def _run_fatal_hooks() -> None:
    for fn in list(_fatal_hooks):
        try:
            fn()
        except Exception as e:  # noqa: BLE001 - never stop the exit path
            sys.stderr.write(f"fatal hook failed: {e}\n")


class BarrierTimeout(RuntimeError):
    """A peer rank did not reach a barrier in time (dead or stuck)."""


def _watchdog(ctx: DistContext, what: str, timeout_s: float, done: threading.Event, hard_exit: bool = True) -> None:
    """SURVEY.md §5 failure detection: a rank whose peer died would otherwise
    sit in the collective until the process-group timeout (10 min).  After
    `timeout_s` the watchdog names the barrier, aborts the communicator
    (ncclCommAbort through torch's _abort_process_group) so the blocked
    collective raises, and if it still has not returned shortly after,
    ends the process with exit status 3."""
    if done.wait(timeout_s):
        return
    sys.stderr.write(f"[rank {ctx.rank}] {what}: peer ranks did not arrive within {timeout_s:.0f} s "
                     f"(dead or stuck rank); aborting the {ctx.backend} communicator\n")
    sys.stderr.flush()
    try:
        from torch.distributed import distributed_c10d as c10d

        c10d._abort_process_group()
    except Exception as e:  # gloo has no abort; fall through to the hard exit
        sys.stderr.write(f"[rank {ctx.rank}] communicator abort unavailable: {e}\n")
    if hard_exit and not done.wait(5.0):
        _run_fatal_hooks()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(3)


def barrier_timeout_s() -> float:
    """Control-plane collectives (barriers, stat reductions) give up after
    this (GCSB_BARRIER_TIMEOUT_S, default 300 s)."""
    return float(os.environ.get("GCSB_BARRIER_TIMEOUT_S", "300"))


class _Watched:
    """A control-plane collective under the hard-exit watchdog (_watchdog):
    a peer that never arrives ends this rank with status 3 instead of
    leaving it in the collective until the process-group timeout."""

    def __init__(self, ctx: DistContext, what: str, timeout_s: float | None = None):
        self.done = threading.Event()
        self.t = threading.Thread(target=_watchdog,
                                  args=(ctx, what, barrier_timeout_s() if timeout_s is None else timeout_s,
                                        self.done),
                                  name="gcsb-barrier-watchdog", daemon=True)

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *exc):
        self.done.set()
        return False


def barrier(ctx: DistContext, what: str = "barrier", timeout_s: float | None = None) -> None:
    """R1/R2: RCCL all_reduce of one int32 + device sync (gloo on CPU), under a
    watchdog (GCSB_BARRIER_TIMEOUT_S, default 300 s)."""
    if not ctx.pg:
        return
    import torch
    import torch.distributed as dist

    try:
        with _Watched(ctx, what, timeout_s):
            t = torch.ones(1, dtype=torch.int32, device=ctx.device)
            dist.all_reduce(t)
            if ctx.gpu >= 0:
                torch.cuda.synchronize(ctx.gpu)
    except Exception as e:
        raise BarrierTimeout(f"{what} failed on rank {ctx.rank}: {e}") from e
    if int(t.item()) != ctx.world:
        raise RuntimeError(f"barrier mismatch: {int(t.item())} != {ctx.world}")


def _timed_group(ctx: DistContext, timeout_s: float):
    """A gloo subgroup over every rank whose collectives give up after
    timeout_s.  gloo has no communicator abort, so the guard's watchdog
    cannot unblock a collective stuck on a dead peer: without this it would
    sit until the process group's own timeout (600 s).  Created on first use;
    every rank reaches the same guarded collective, so every rank creates it
    (new_group is itself collective)."""
    import torch.distributed as dist

    if ctx.guard_groups is None:
        ctx.guard_groups = {}
    key = int(timeout_s)
    if key not in ctx.guard_groups:
        ctx.guard_groups[key] = dist.new_group(ranks=list(range(ctx.world)), backend="gloo",
                                               timeout=datetime.timedelta(seconds=timeout_s))
    return ctx.guard_groups[key]


class _Guard:
    """Watchdog around one collective (see _watchdog)."""

    def __init__(self, ctx: DistContext, what: str, timeout_s: float):
        self.done = threading.Event()
        # abort the communicator but keep the process: the caller reports the
        # failed block and prints the rest of its results
        self.t = threading.Thread(target=_watchdog, args=(ctx, what, timeout_s, self.done, False),
                                  name="gcsb-collective-watchdog", daemon=True)

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *exc):
        self.done.set()
        return False


def all_gather_bytes(ctx: DistContext, out, part, what: str = "all-gather", timeout_s: float | None = None) -> None:
    """Every rank's `part` (uint8, equal sizes) into `out` in rank order.
    RCCL: all_gather_into_tensor on the GPUs (peer-to-peer over xGMI within a
    node).  gloo: the parts go through host memory."""
    if not ctx.pg or ctx.world == 1:
        out.copy_(part)
        return
    import torch
    import torch.distributed as dist

    if timeout_s is None:
        timeout_s = collective_timeout_s()
    if ctx.device.type == "cuda":
        with _Guard(ctx, what, timeout_s):
            dist.all_gather_into_tensor(out, part)
    else:
        # gloo: the collective carries its own timeout (no abort to call)
        group = _timed_group(ctx, timeout_s)
        host = part.cpu()
        parts = [torch.empty_like(host) for _ in range(ctx.world)]
        dist.all_gather(parts, host, group=group)
        out.copy_(torch.cat(parts).to(out.device))


def reduce_stats(ctx: DistContext, **vals: float) -> dict:
    """R3: returns {k_sum, k_max, k_min} for every value (+ per-rank list)."""
    import torch

    keys = sorted(vals)
    out: dict = {}
    if not ctx.pg:
        for k in keys:
            v = float(vals[k])
            out[k + "_sum"] = out[k + "_max"] = out[k + "_min"] = v
            out[k + "_per_rank"] = [v]
        return out
    import torch.distributed as dist

    base = torch.tensor([float(vals[k]) for k in keys], dtype=torch.float64, device=ctx.device)
    s, mx, mn = base.clone(), base.clone(), base.clone()
    gathered = [torch.zeros_like(base) for _ in range(ctx.world)]
    with _Watched(ctx, "R3 stats reduce"):
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
        dist.all_gather(gathered, base)
        # RCCL collectives return once enqueued: the wait for a peer is the
        # host read-out, so it must happen under the watchdog too
        s_, mx_, mn_ = s.tolist(), mx.tolist(), mn.tolist()
        g_ = [g.tolist() for g in gathered]
    for i, k in enumerate(keys):
        out[k + "_sum"] = float(s_[i])
        out[k + "_max"] = float(mx_[i])
        out[k + "_min"] = float(mn_[i])
        out[k + "_per_rank"] = [float(g[i]) for g in g_]
    return out


def reduce_histogram(ctx: DistContext, buckets: list[int]) -> list[int]:
    """Sum the OpenCensus latency buckets over ranks (node-level view)."""
    if not ctx.pg:
        return list(buckets)
    import torch
    import torch.distributed as dist

    t = torch.tensor(buckets, dtype=torch.int64, device=ctx.device)
    with _Watched(ctx, "R3 histogram reduce"):
        dist.all_reduce(t)
        vals = t.tolist()  # the blocking read-out, under the watchdog
    return [int(x) for x in vals]


def gather_floats(ctx: DistContext, vals: list[float]) -> list[list[float]]:
    """R4: every rank's small float vector, in rank order (all_gather)."""
    if not ctx.pg:
        return [list(map(float, vals))]
    import torch
    import torch.distributed as dist

    base = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=ctx.device)
    out = [torch.zeros_like(base) for _ in range(ctx.world)]
    with _Watched(ctx, "R4 gather"):
        dist.all_gather(out, base)
        vals = [t.tolist() for t in out]  # the blocking read-out, under the watchdog
    return [[float(x) for x in v] for v in vals]


def shutdown(ctx: DistContext) -> None:
    if ctx.initialized_here:
        import torch.distributed as dist

        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception as e:  # noqa: BLE001 - an aborted communicator
                sys.stderr.write(f"[rank {ctx.rank}] process group teardown: {e}\n")
