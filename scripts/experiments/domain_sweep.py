"""Does the L3 domain (CCD) the one-stream headline receives on matter?

For each L3 domain of the GPU's NUMA node: a pair placement inside that
domain (receiving core, endpoint core, submitter core), then the headline
(4 x 1 MiB ring -> H2D -> HBM) and the same ring never DMA-read (nodma),
interleaved, `--reps` times.  If the copy engine's read costs the receiving
core less on some CCDs (closer to the GPU's PCIe root in the IO die), the
headline's placement should pick them."""
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
ap.add_argument("--reads", type=int, default=10)
ap.add_argument("--size", type=int, default=256 << 20)
args = ap.parse_args()
n = pkg._native
cpus = affinity.gpu_local_cpus(0)
groups = affinity.l3_groups(cpus)
busy = affinity.cpu_busy(0.1)
print(json.dumps({"domains": len(groups), "first_cpus": [g[0] for g in groups]}), flush=True)
for di, dom in enumerate(groups):
    q = affinity.quiet_cores(dom, busy)
    if len(q) < 3:
        continue
    pl = {"client": q[0], "server": q[1], "aux": q[2]}
    n.set_submitter_cpus(pl["aux"])
    srv = n.Server({"port": 0, "md5": False, "cpus": pl["server"], "retain_uploads": False})
    srv.start()
    srv.add_synthetic("b", "f_", "", 0, 1, args.size)
    base = {"protocol": "grpc", "endpoint": srv.url, "bucket": "b", "object_prefix": "f_", "workers": 1,
            "reads_per_worker": 3, "device": 0, "ring_slot_bytes": 1 << 20, "ring_slots": 4, "landing": "object",
            "keep_records": False, "cpus": pl["client"], "rcvbuf": 64 << 20, "async_submit": True,
            "blocking_sync": True, "retry_initial_s": 0.05, "tcp_congestion": "cubic", "sink": "gpu"}
    runners = {"head": n.Runner(base), "nodma": n.Runner({**base, "gpu_stage": "none"})}
    for r in runners.values():
        r.start()
        r.wait()
    for rep in range(args.reps):
        for name, r in runners.items():
            r.reset_stats()
            r.set_reads_per_worker(args.reads)
            t0 = cpuacct.thread_cpu()
            w0 = time.perf_counter()
            r.start()
            r.wait()
            el = time.perf_counter() - w0
            d = cpuacct.delta_by_name(t0, cpuacct.thread_cpu())
            s = r.summary()
            gib = max(s["bytes"], 1) / (1 << 30)
            print(json.dumps({"domain": di, "cpus": pl, "rep": rep, "variant": name,
                              "mib_s": round(s["bytes"] / el / (1 << 20), 1), "p50_ms": round(s["p50_ms"], 3),
                              "reader_cpu_s_per_gib": round(d.get("gcsb-h2-reader", 0.0) / gib, 4),
                              "errors": s["errors"]}), flush=True)
    del runners
    srv.stop()
