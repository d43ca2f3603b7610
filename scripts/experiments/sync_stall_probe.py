"""First slot hand-off after torch.cuda.synchronize(): which HIP call blocks,
on which pool stream, and what removes it.

Reads a 256 MiB object over one gRPC stream into HBM (the bench headline's
sink: 8 x 2 MiB ring, async submitter), `--reps` times per gap variant:
  none       back to back;
  sync       torch.cuda.synchronize() before each read (the bench's bracket);
  sync_warm  the same, then one tiny copy on every pool stream (warm_device_streams);
  sleep      time.sleep(0.05) (an idle gap without a device sync).
Per read: latency, host-landed latency, and the slot hand-off HIP calls that
blocked >= 1 ms (engine.hip note_hip_call).  One JSON line per variant.
Environment variants (GPU_MAX_HW_QUEUES, GCSB_STREAMS) are set by the caller.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402

import custom_go_client_benchmark_amd as pkg  # noqa: E402
from custom_go_client_benchmark_amd.parallel import affinity  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=8)
ap.add_argument("--size", type=int, default=256 << 20)
ap.add_argument("--variants", default="none,sync,sync_warm,sleep,sync")
ap.add_argument("--protocol", default="grpc")
args = ap.parse_args()

n = pkg._native
pl = affinity.plan(0, "pair", 0)
if pl.get("aux"):
    n.set_submitter_cpus(pl["aux"])
srv = n.Server({"port": 0, "md5": False, "cpus": pl["server"], "retain_uploads": False})
srv.start()
srv.add_synthetic("b", "f_", "", 0, 1, args.size)
os.sched_setaffinity(0, pl["client"])
cli = n.Client({"protocol": args.protocol, "endpoint": srv.url, "rcvbuf": 64 << 20, "retry_initial_s": 0.05})
dst = torch.empty(args.size, dtype=torch.uint8, device="cuda:0")
sink = n.GpuSink({"device": 0, "ring_slot_bytes": 2 << 20, "ring_slots": 8, "async_submit": True})
sink.set_external_destination(dst.data_ptr(), args.size)


def one():
    n.reset_slow_hip_calls()
    t0 = time.perf_counter_ns()
    r = cli.read_gpu("b", "f_0", sink)
    ms = (time.perf_counter_ns() - t0) / 1e6
    assert r["bytes"] == args.size and r["verified"] and not r["crc_mismatch"], r
    s = n.slow_hip_calls()
    return {"ms": round(ms, 3), "host_ms": round((r["host_done_ns"] - t0) / 1e6, 3) if r["host_done_ns"] else None,
            "slow": s["slow"], "slow_ms": round(s["slow_ms_total"], 3), "max": s["max_call"], "max_ms": round(s["max_ms"], 3)}


gaps = {
    "none": lambda: None,
    "sync": torch.cuda.synchronize,
    "sync_warm": lambda: (torch.cuda.synchronize(), n.warm_device_streams(0)),
    "sleep": lambda: time.sleep(0.05),
}
for _ in range(3):
    one()
env = {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES", "GCSB_STREAMS", "GCSB_SINK_STREAMS", "GCSB_WARM_STREAMS")}
for v in args.variants.split(","):
    rows = []
    for _ in range(args.reps):
        gaps[v]()
        rows.append(one())
    ms = sorted(r["ms"] for r in rows)
    print(json.dumps({"variant": v, "env": env, "p50": ms[len(ms) // 2], "max": ms[-1],
                      "slow_reads": sum(1 for r in rows if r["slow"]), "reads": rows}), flush=True)
srv.stop()
