"""What does one gRPC stream's receiving thread pay per byte, and for what?

Same endpoint, object (256 MiB), placement (pair) and ring as the bench
headline; variants interleaved `--reps` times:
  tcp        core/ceiling.cc: one loopback TCP stream, no framing, THP ring
  grpc_null  gRPC ReadObject into a discard sink, no CRC (framing only)
  grpc_gpu   the headline: pinned THP ring -> H2D -> HBM, CRC kernels
  grpc_copy  same, CRC kernels off (gpu_verify false): H2D copies only
Per variant: MiB/s, receiving thread CPU-s/GiB (gcsb-h2-reader), recv() size.
One JSON line per variant and rep."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402,F401

import custom_go_client_benchmark_amd as pkg  # noqa: E402
from custom_go_client_benchmark_amd.parallel import affinity  # noqa: E402
from custom_go_client_benchmark_amd.utils import cpuacct  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--reads", type=int, default=20)
ap.add_argument("--size", type=int, default=256 << 20)
args = ap.parse_args()

n = pkg._native
pl = affinity.plan(0, "pair", 0)
if pl.get("aux"):
    n.set_submitter_cpus(pl["aux"])
srv = n.Server({"port": 0, "md5": False, "cpus": pl["server"], "retain_uploads": False})
srv.start()
srv.add_synthetic("b", "f_", "", 0, 1, args.size)
base = {"protocol": "grpc", "endpoint": srv.url, "bucket": "b", "object_prefix": "f_", "workers": 1,
        "reads_per_worker": 3, "device": 0, "ring_slot_bytes": 2 << 20, "ring_slots": 8, "landing": "object",
        "keep_records": False, "cpus": pl["client"], "rcvbuf": 64 << 20, "async_submit": True,
        "blocking_sync": True}
variants = {
    "grpc_null": {"sink": "discard", "host_crc": False},
    "grpc_gpu": {"sink": "gpu"},
    "grpc_copy": {"sink": "gpu", "gpu_verify": False},
}
runners = {k: n.Runner({**base, **v}) for k, v in variants.items()}
for r in runners.values():  # warm: connections, rings, sinks
    r.start()
    r.wait()


def run(name):
    if name == "tcp":
        c = n.loopback_ceiling({"mode": "tcp", "object_bytes": args.size, "reads": args.reads, "ring_bytes": 16 << 20,
                                "rcvbuf": 64 << 20, "recv_cpus": pl["client"], "send_cpus": pl["server"]})
        return {"mib_s": round(c["gbps"] * 1e9 / (1 << 20), 1), "recv_cpu_s_per_gib": round(c["recv_cpu_s_per_gib"], 4)}
    r = runners[name]
    r.reset_stats()
    r.set_reads_per_worker(args.reads)
    t0 = cpuacct.thread_cpu()
    rv0 = n.recv_stats()
    w0 = time.perf_counter()
    r.start()
    r.wait()
    el = time.perf_counter() - w0
    s = r.summary()
    gib = max(s["bytes"], 1) / (1 << 30)
    d = cpuacct.delta_by_name(t0, cpuacct.thread_cpu())
    rv1 = n.recv_stats()
    return {"mib_s": round(s["bytes"] / el / (1 << 20), 1), "p50_ms": round(s["p50_ms"], 3),
            "recv_cpu_s_per_gib": round(d.get("gcsb-h2-reader", 0.0) / gib, 4),
            "endpoint_cpu_s_per_gib": round(sum(v for k, v in d.items() if k.startswith("gcsb-srv")) / gib, 4),
            "recv_avg_kib": round((rv1[1] - rv0[1]) / max(1, rv1[0] - rv0[0]) / 1024, 1),
            "verified": s["verified"], "errors": s["errors"], "gpu": s["gpu"]}


for rep in range(args.reps):
    for name in ["tcp", "grpc_null", "grpc_gpu", "grpc_copy"]:
        print(json.dumps({"rep": rep, "variant": name, **run(name)}), flush=True)
srv.stop()
