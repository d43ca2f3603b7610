"""Why does the one-stream headline (gRPC -> pinned ring -> H2D -> HBM) read
slower than the same-run reference-semantics read (discard + host CRC32C)?

VERDICT r3 "What's missing" #1.  Same endpoint, 256 MiB object, pair
placement and 8 x 2 MiB THP ring as bench.py's headline; variants
interleaved `--reps` times in one process:

  head      the headline: ring -> hipMemcpyAsync -> HBM, CRC32C kernels
  head_wc   the same, ring in write-combined pinned memory
  head_4m   the same, 4 x 4 MiB slots
  head_4x2  the same, 4 x 2 MiB slots (the discard sink's 8 MiB footprint)
  head_refill  the same, recv_refill (one recvmsg per DATA frame tail + next header)
  head_spin the same, the device submitter polls 200 us before it sleeps
  nodma     the same ring, filled by the same receive path, handed straight
            back: nothing reads it (gpu_stage none)
  hostread  the submitter thread reads each slot (host CRC32C) instead of
            the copy engine (gpu_stage host_read)
  base      reference semantics: discard sink + host CRC32C on the worker,
            client + aux cores (bench.py's cpu_baseline)

Per variant and rep: MiB/s, p50, the h2 reader's CPU and where its wall time
went (frame-header wait vs DATA), the endpoint's TCP busy fraction, and the
host view (utils/sysdiag): per-thread run-queue delay and involuntary
switches, interrupts and softirqs on the placement's CPUs.  One JSON line
each.  Run it once as is and once with HSA_ENABLE_INTERRUPT=0 (no GPU
completion interrupts) to see what those cost the two busy cores."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402,F401

import custom_go_client_benchmark_amd as pkg  # noqa: E402
from custom_go_client_benchmark_amd.parallel import affinity  # noqa: E402
from custom_go_client_benchmark_amd.utils import cpuacct, sysdiag  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--reads", type=int, default=20)
ap.add_argument("--size", type=int, default=256 << 20)
ap.add_argument("--variants", default="head,nodma,hostread,base")
ap.add_argument("--tag", default="")
args = ap.parse_args()

n = pkg._native
pl = affinity.plan(0, "pair", 0)
if pl.get("aux"):
    n.set_submitter_cpus(pl["aux"])
srv = n.Server({"port": 0, "md5": False, "cpus": pl["server"], "retain_uploads": False})
srv.start()
srv.add_synthetic("b", "f_", "", 0, 1, args.size)
cpus_all = sorted(set(pl["client"]) | set(pl["server"]) | set(pl.get("aux") or []))
base = {"protocol": "grpc", "endpoint": srv.url, "bucket": "b", "object_prefix": "f_", "workers": 1,
        "reads_per_worker": 3, "device": 0, "ring_slot_bytes": 2 << 20, "ring_slots": 8, "landing": "object",
        "keep_records": False, "cpus": pl["client"], "rcvbuf": 64 << 20, "async_submit": True,
        "blocking_sync": True, "retry_initial_s": 0.05, "tcp_congestion": "cubic"}
two_core = sorted(set(pl["client"]) | set(pl.get("aux") or []))
variants = {
    "head": {"sink": "gpu"},
    "nodma": {"sink": "gpu", "gpu_stage": "none"},
    "hostread": {"sink": "gpu", "gpu_stage": "host_read"},
    "base": {"sink": "discard", "host_crc": True, "cpus": two_core},
    # the headline's ring in write-combined pinned memory (no RFO, no dirty
    # lines for the copy engine to read), and with 4 MiB slots (half the
    # hand-offs per read)
    "head_wc": {"sink": "gpu", "ring_wc": True},
    "head_4m": {"sink": "gpu", "ring_slot_bytes": 4 << 20, "ring_slots": 4},
    # half the ring (8 MiB, the discard sink's 4 recycled 2 MiB blocks)
    "head_4x2": {"sink": "gpu", "ring_slots": 4},
    # ring footprint sweep (main5: 4 x 2 MiB read 8-10% faster than 8 x 2 MiB
    # in all five reps, with 12% less reader CPU per GiB)
    "head_2x2": {"sink": "gpu", "ring_slots": 2},
    "head_3x2": {"sink": "gpu", "ring_slots": 3},
    "head_4x1m": {"sink": "gpu", "ring_slot_bytes": 1 << 20, "ring_slots": 4},
    "head_8x512k": {"sink": "gpu", "ring_slot_bytes": 512 << 10, "ring_slots": 8},
    "head_4x2_wc": {"sink": "gpu", "ring_slots": 4, "ring_wc": True},
    "head_2x1m": {"sink": "gpu", "ring_slot_bytes": 1 << 20, "ring_slots": 2},
    "head_3x1m": {"sink": "gpu", "ring_slot_bytes": 1 << 20, "ring_slots": 3},
    "head_6x1m": {"sink": "gpu", "ring_slot_bytes": 1 << 20, "ring_slots": 6},
    "head_4x512k": {"sink": "gpu", "ring_slot_bytes": 512 << 10, "ring_slots": 4},
    "head_8x256k": {"sink": "gpu", "ring_slot_bytes": 256 << 10, "ring_slots": 8},
    # the headline with the next frame header read in the payload's recvmsg
    "head_refill": {"sink": "gpu", "recv_refill": True},
    # the headline with the device submitter polling 200 us for the next
    # hand-off before it sleeps (no futex wake per slot on the receiver)
    "head_spin": {"sink": "gpu"},
    "head_4x1m_spin": {"sink": "gpu", "ring_slot_bytes": 1 << 20, "ring_slots": 4},
    # windows stop at each slot's end (before: a recv ran on into the next free slot)
    # the headline's receiving thread free to run on both of the baseline's
    # cores (the submitter stays pinned to the aux core)
    "head_4x1m_2core": {"sink": "gpu", "ring_slot_bytes": 1 << 20, "ring_slots": 4, "cpus": "TWO_CORE"},
    "head_4x1m_nospan": {"sink": "gpu", "ring_slot_bytes": 1 << 20, "ring_slots": 4, "ring_span": False},
    "head_8x512k_nospan": {"sink": "gpu", "ring_slot_bytes": 512 << 10, "ring_slots": 8, "ring_span": False},
    # the multiplexed reader's destination footprint on one stream: 48 MiB /
    # 96 MiB rings (48 workers x 1-2 MiB), with and without the DMA
    "head_24x2": {"sink": "gpu", "ring_slots": 24},
    "head_48x2": {"sink": "gpu", "ring_slots": 48},
    "nodma_48x2": {"sink": "gpu", "gpu_stage": "none", "ring_slots": 48},
    # round 5: the one stream through a connection ring in arena mode (recv
    # straight into the ring, a slot's worth per recv).  The staged-copy and
    # cross-CCD recv-helper variants measured in profiles/r5_arena were
    # removed after that measurement (git history has them).
    "nodma_4x1m": {"sink": "gpu", "gpu_stage": "none", "ring_slot_bytes": 1 << 20, "ring_slots": 4},
    "arena_4x1m": {"sink": "gpu", "conn_ring_single": True, "conn_ring_inplace": True, "conn_ring_slots": 4,
                   "conn_ring_slot_bytes": 1 << 20},
}
SPIN_US = {"head_spin": 200, "head_4x1m_spin": 200}
names = [v for v in args.variants.split(",") if v]
for v in variants.values():
    if v.get("cpus") == "TWO_CORE":
        v["cpus"] = two_core
runners = {k: n.Runner({**base, **variants[k]}) for k in names}
for r in runners.values():  # warm: connections, rings, sinks
    r.start()
    r.wait()
print(json.dumps({"tag": args.tag, "placement": pl, "hsa_enable_interrupt": os.environ.get("HSA_ENABLE_INTERRUPT")}),
      flush=True)


def run(name):
    n.set_submitter_spin_us(SPIN_US.get(name, 0))
    r = runners[name]
    r.reset_stats()
    r.set_reads_per_worker(args.reads)
    t0 = cpuacct.thread_cpu()
    h0 = n.h2_reader_stats()
    sv0 = srv.stats()
    win = sysdiag.Window()
    w0 = time.perf_counter()
    r.start()
    r.wait()
    el = time.perf_counter() - w0
    diag = win.report(cpus_all, args.reads)
    sv1 = srv.stats()
    h1 = n.h2_reader_stats()
    s = r.summary()
    gib = max(s["bytes"], 1) / (1 << 30)
    d = cpuacct.delta_by_name(t0, cpuacct.thread_cpu())
    hd = {k: h1[k] - h0[k] for k in h1}
    wall = max(1, sv1["body_wall_us"] - sv0["body_wall_us"])
    return {"mib_s": round(s["bytes"] / el / (1 << 20), 1), "p50_ms": round(s["p50_ms"], 3),
            "p99_ms": round(s["p99_ms"], 3), "host_p50_ms": round(s["host_p50_ms"], 3),
            "reader_cpu_s_per_gib": round(d.get("gcsb-h2-reader", 0.0) / gib, 4),
            "reader_wait_s_per_gib": round(hd["header_wait_ns"] / 1e9 / gib, 4),
            "reader_data_s_per_gib": round(hd["data_ns"] / 1e9 / gib, 4),
            "endpoint_cpu_s_per_gib": round(sum(v for k, v in d.items() if k.startswith("gcsb-srv")) / gib, 4),
            "submit_cpu_s_per_gib": round(d.get("gcsb-submit", 0.0) / gib, 4),
            "handoff_s_per_gib": round((s.get("gpu") or {}).get("handoff_s", 0.0) / gib, 5),
            "worker_cpu_s_per_gib": round(s.get("worker_cpu_s", 0.0) / gib, 4),
            "conn_ring": r.conn_ring_stats(),
            "endpoint_busy_frac": round((sv1["tcp_busy_us"] - sv0["tcp_busy_us"]) / wall, 3),
            "errors": s["errors"], "sched": diag}


for rep in range(args.reps):
    for name in names:
        print(json.dumps({"tag": args.tag, "rep": rep, "variant": name, **run(name)}), flush=True)
srv.stop()
