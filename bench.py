#!/usr/bin/env python3
"""Headline benchmark: whole-object reads from a (synthetic, loopback) GCS
endpoint into MI355X HBM, one reader process per GPU.

Metric (BASELINE.json): p50/p99 read latency (ms) + MB/s per GPU, HTTP vs gRPC
at 1/2/4/8 MI355X.  Config: 256 MiB objects, gRPC ReadObject stream (HTTP with
--protocol http), bytes land in HBM through the pinned ring + hipMemcpyAsync
and every ChecksummedData CRC32C is verified by the CDNA4 kernels.

One step = every rank's reader reads its own 256 MiB object (file_<rank>) once,
so per-GPU work is fixed as N grows (weak scaling).  Each read is a sliced read
by default (--slices 8: stat, then 8 concurrent ranged streams on their own
connections landing at their offsets in HBM, object CRC32C = combine of the
slice CRCs, checked against the stored CRC32C); a single-stream read (the
reference's one NewReader per object) is measured right after on the same
endpoint and reported as `single_stream_*`, and the other transport (HTTP
when the headline is gRPC) on the same sliced config as `compare`; both run
after the timed region.  W untimed warmup reads,
then K timed reads bracketed by an RCCL barrier + torch.cuda.synchronize();
the elapsed time is the MAX over ranks and `value` is total bytes / that time.

    python bench.py --gpus 1 --steps 20 --warmup 3
    torchrun --nproc-per-node 8 bench.py --gpus 8 ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "p50/p99 read latency (ms) + MB/s per GPU; HTTP vs gRPC at 1/2/4/8 MI355X"


def parse_size(s: str) -> int:
    s = s.strip()
    mult = {"k": 1 << 10, "kib": 1 << 10, "m": 1 << 20, "mib": 1 << 20, "g": 1 << 30, "gib": 1 << 30}
    for suf in sorted(mult, key=len, reverse=True):
        if s.lower().endswith(suf):
            return int(float(s[: -len(suf)]) * mult[suf])
    return int(s)


def cpu_snapshot() -> dict:
    """Process CPU time (client + node-local endpoint share this process) and
    the cgroup's CFS throttling counters: on the GPU boxes the container runs
    under a CPU quota (profiles/r1_gpu_box_env.txt), and loopback TCP costs CPU
    at both ends, so these explain throughput and the p99 tail."""
    import resource

    ru = resource.getrusage(resource.RUSAGE_SELF)
    snap = {"user_s": ru.ru_utime, "sys_s": ru.ru_stime}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, _, v = line.partition(" ")
                if k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec"):
                    snap[k] = int(v)
    except OSError:
        pass
    return snap


def cpu_delta(a: dict, b: dict, nbytes: float) -> dict:
    gib = max(nbytes, 1.0) / (1 << 30)
    out = {"process_cpu_s_per_gib": round((b["user_s"] + b["sys_s"] - a["user_s"] - a["sys_s"]) / gib, 4),
           "process_sys_fraction": round((b["sys_s"] - a["sys_s"]) /
                                         max(1e-9, b["user_s"] + b["sys_s"] - a["user_s"] - a["sys_s"]), 3)}
    for k in ("nr_periods", "nr_throttled", "throttled_usec"):
        if k in a and k in b:
            out["cgroup_" + k] = b[k] - a[k]
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--protocol", default="auto", help="grpc | http | auto (grpc when built)")
    ap.add_argument("--object-size", default="256MiB")
    ap.add_argument("--workers", type=int, default=1, help="readers per GPU (config: 1)")
    ap.add_argument("--sink", default="gpu", help="gpu (HBM landing + GPU CRC) | discard (CPU baseline)")
    ap.add_argument("--slot-bytes", default="4MiB")
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--grpc-pool", type=int, default=1)
    ap.add_argument("--slices", type=int, default=8,
                    help="concurrent ranged streams per object read, each on its own connection (1 = one stream)")
    ap.add_argument("--piece-bytes", default="8MiB",
                    help="sliced reads: streams pull pieces of this size from a shared cursor (0 = fixed shares; "
                         "8 MiB measured best: profiles/r1_pieces)")
    ap.add_argument("--piece-min-bytes", default="0",
                    help="sliced reads: taper the piece size toward the end of the object down to this "
                         "(guided self-scheduling, storage/sliced.h; 0 = fixed-size pieces)")
    ap.add_argument("--affinity", default="share",
                    help="CPU placement of client/endpoint threads: share|same|split|numa|none (see parallel/affinity.py)")
    ap.add_argument("--single-stream-steps", type=int, default=-1,
                    help="timed single-stream reads measured after the main run for comparison (-1: = --steps, 0: skip)")
    ap.add_argument("--event-wait", default="block", choices=["spin", "block"],
                    help="how GPU sinks wait on slot events: block (interrupt, the library default) or spin. "
                         "Spin won 5 of 6 interleaved pairs but not on the mean, with one bad p99 "
                         "(profiles/r1_session12, r1_session13)")
    ap.add_argument("--compare-steps", type=int, default=-1,
                    help="timed reads over the other transport (HTTP vs gRPC) on the same config, reported "
                         "as `compare` (-1: = --steps, 0: skip)")
    ap.add_argument("--json-out", default="")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import custom_go_client_benchmark_amd as pkg
    from custom_go_client_benchmark_amd.ops import hbm
    from custom_go_client_benchmark_amd.parallel import dist as gdist
    from custom_go_client_benchmark_amd.utils import cpuacct

    n = pkg._native
    rank, world, local_rank = gdist.env_rank()
    ctx = gdist.init(local_rank=local_rank, world=world, rank=rank)
    use_gpu = args.sink == "gpu"
    if use_gpu:
        hbm.gpu_required()
    protocol = args.protocol
    if protocol == "auto":
        protocol = "grpc" if "grpc" in hbm.available_protocols() else "http"
    size = parse_size(args.object_size)

    # Node-local synthetic GCS endpoint for this rank (no network on the box).
    from custom_go_client_benchmark_amd.parallel import affinity

    gpu = ctx.gpu if ctx.gpu >= 0 else 0
    placement = affinity.plan(gpu, args.affinity) if use_gpu else {"client": [], "server": []}
    srv = n.Server({"port": 0, "md5": False, "cpus": placement["server"]})
    srv.start()
    bucket = "princer-working-dirs"
    prefix = "princer_100M_files/file_"
    first = rank * args.workers
    srv.add_synthetic(bucket, prefix, "", first, args.workers, size)

    cfg = {
        "protocol": protocol,
        "endpoint": srv.url,
        "bucket": bucket,
        "object_prefix": prefix,
        "workers": args.workers,
        "reads_per_worker": args.warmup,
        "worker_id_offset": first,
        "sink": args.sink,
        "device": gpu if use_gpu else 0,
        "ring_slot_bytes": parse_size(args.slot_bytes),
        "ring_slots": args.slots,
        "landing": "object",
        "grpc_conn_pool_size": args.grpc_pool,
        "keep_records": False,
        "cpus": placement["client"],
        "retry_initial_s": 0.05,
        "slices": args.slices,
        "slice_piece_bytes": parse_size(args.piece_bytes),
        "slice_piece_min_bytes": parse_size(args.piece_min_bytes),
        "blocking_sync": args.event_wait == "block",
    }
    run = n.Runner(cfg)
    if args.warmup > 0:
        run.start()
        run.wait()
        s = run.summary()
        if s["errors"]:
            print(f"[rank {rank}] warmup failed: {s['first_error']}", file=sys.stderr)
            return 1
    run.reset_stats()
    run.set_reads_per_worker(args.steps)

    gdist.barrier(ctx, "R1/R2 bench barrier")
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    c0 = cpu_snapshot()
    th0 = cpuacct.thread_cpu()
    t0 = time.perf_counter()
    run.start()
    run.wait()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    gdist.barrier(ctx, "R1/R2 bench barrier")
    elapsed = time.perf_counter() - t0
    s = run.summary()
    cpu = cpu_delta(c0, cpu_snapshot(), float(s["bytes"]))
    cpu["cpu_s_per_gib_by_thread"] = cpuacct.per_gib(cpuacct.delta_by_group(th0, cpuacct.thread_cpu()),
                                                     float(s["bytes"]))

    def side_run(overrides: dict, steps: int, what: str):
        """One untimed read, then `steps` timed reads of a variant config;
        every rank joins (the reductions below are collective)."""
        r1 = n.Runner({**cfg, **overrides, "reads_per_worker": 1})
        r1.start()
        r1.wait()
        r1.reset_stats()
        r1.set_reads_per_worker(steps)
        gdist.barrier(ctx, f"R1/R2 {what} barrier")
        t1 = time.perf_counter()
        r1.start()
        r1.wait()
        gdist.barrier(ctx, f"R1/R2 {what} barrier")
        e1 = time.perf_counter() - t1
        s1 = r1.summary()
        del r1
        return gdist.reduce_stats(ctx, elapsed=e1, nbytes=float(s1["bytes"]), p50=s1["p50_ms"], p99=s1["p99_ms"],
                                  ok=1.0 if s1["errors"] == 0 else 0.0)

    # single-stream comparison (slices=1: the reference's one stream per read)
    ss_steps = args.steps if args.single_stream_steps < 0 else args.single_stream_steps
    ss_stats = side_run({"slices": 1}, ss_steps, "single-stream") if args.slices > 1 and ss_steps > 0 else None
    # the other transport on the same config (the metric is HTTP vs gRPC)
    other = {"grpc": "http", "http": "grpc"}.get(protocol)
    cmp_steps = args.steps if args.compare_steps < 0 else args.compare_steps
    cmp_stats = None
    if other and cmp_steps > 0 and other in hbm.available_protocols():
        cmp_stats = side_run({"protocol": other}, cmp_steps, f"{other} comparison")
    srv.stop()

    ok = 1.0 if s["errors"] == 0 and s["reads"] == args.steps * args.workers else 0.0
    stats = gdist.reduce_stats(ctx, elapsed=elapsed, nbytes=float(s["bytes"]), ok=ok, p50=s["p50_ms"],
                               p99=s["p99_ms"], host_p50=s["host_p50_ms"])
    if rank == 0:
        if stats["ok_min"] < 1.0:
            print(f"benchmark failed: {s['first_error'] or 'incomplete reads'}", file=sys.stderr)
            return 1
        total = stats["nbytes_sum"]
        tmax = stats["elapsed_max"]
        value = total / tmax / (1 << 20)
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "MiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(tmax / args.steps * 1000.0, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8",
            "data": "synthetic",
            "config": {
                "model": f"{protocol} ReadObject {args.object_size} object -> HBM (CRC32C on GPU)"
                if use_gpu else f"{protocol} read {args.object_size} -> discard (CPU baseline)",
                "global_batch": world * args.workers,
                "seq_len": size,
                "parallelism": f"dp{world}",
                "protocol": protocol,
                "object_bytes": size,
                "readers_per_gpu": args.workers,
                "sink": args.sink,
                "ring": f"{args.slots}x{args.slot_bytes}",
                "streams_per_read": args.slices,
                "piece_bytes": parse_size(args.piece_bytes),
                "piece_min_bytes": parse_size(args.piece_min_bytes),
                "event_wait": args.event_wait,
            },
            "per_gpu_mib_s": round(value / world, 2),
            "p50_ms": round(stats["p50_max"], 3),
            "p99_ms": round(stats["p99_max"], 3),
            "host_landed_p50_ms": round(stats["host_p50_max"], 3),
            "slice_skew_ms": round(s.get("slice_skew_ms", 0.0), 3),
            "endpoint": "loopback synthetic GCS (one per rank)",
            "affinity": args.affinity,
            "rank0_cpu": cpu,
        }
        if ss_stats is not None:
            out["single_stream_mib_s"] = round(ss_stats["nbytes_sum"] / ss_stats["elapsed_max"] / (1 << 20), 2)
            out["single_stream_p50_ms"] = round(ss_stats["p50_max"], 3)
            out["single_stream_p99_ms"] = round(ss_stats["p99_max"], 3)
        if cmp_stats is not None:
            out["compare"] = {"protocol": other, "ok": cmp_stats["ok_min"] >= 1.0,
                              "mib_s": round(cmp_stats["nbytes_sum"] / cmp_stats["elapsed_max"] / (1 << 20), 2),
                              "p50_ms": round(cmp_stats["p50_max"], 3), "p99_ms": round(cmp_stats["p99_max"], 3)}
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    gdist.shutdown(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
