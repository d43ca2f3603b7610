"""The reference's default experiment on gRPC (48 workers, 1 MiB objects, ONE
connection: /root/reference/main.go:30,36,111) against endpoints whose HTTP/2
frame writes are FIFO-granted with a DATA frame quantum of `--quanta` KiB
(0 = whole messages; ServerConfig::h2_quantum), interleaved `--reps` times.
Placement as bench.py's ref_default_grpc ("same": one L3 domain).  Per run:
MiB/s, p50/p99, the endpoint's per-frame queue wait and request -> HEADERS
time (avg / max), and the slowest reads [index, ms, host ms, TTFB ms]."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402,F401

import custom_go_client_benchmark_amd as pkg  # noqa: E402
from custom_go_client_benchmark_amd.parallel import affinity  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--reads", type=int, default=50)
ap.add_argument("--workers", type=int, default=48)
ap.add_argument("--size", type=int, default=1 << 20)
ap.add_argument("--quanta", default="0,256,1024")
ap.add_argument("--leads", default="0",
                help="KiB: a new read's first DATA frame ahead of the queue (h2_lead_bytes, removed after "
                     "profiles/r4_main7: only 0 runs on today's endpoint)")
ap.add_argument("--protocol", default="grpc")
ap.add_argument("--bufs", default="0:0",
                help="comma list of SNDBUF_KIB:RCVBUF_KIB (endpoint send buffer, client receive buffer; 0 = "
                     "autotuned): the bytes in flight ahead of a new stream's first byte")
args = ap.parse_args()
n = pkg._native
pl = affinity.plan(0, "same", 0) if torch.cuda.is_available() else {"client": [], "server": []}
for rep in range(args.reps):
    for q, lead, bufs in [(int(x), int(y), z) for x in args.quanta.split(",") for y in args.leads.split(",")
                          for z in args.bufs.split(",")]:
        sndk, rcvk = (int(v) for v in bufs.split(":"))
        srv = n.Server({"port": 0, "md5": False, "retain_uploads": False, "h2_quantum": q << 10,
                        "h2_lead_bytes": lead << 10, "cpus": pl["server"], "sndbuf": sndk << 10})
        srv.start()
        srv.add_synthetic("b", "f_", "", 0, args.workers, args.size)
        r = n.Runner({"protocol": args.protocol, "endpoint": srv.url, "bucket": "b", "object_prefix": "f_",
                      "workers": args.workers, "reads_per_worker": 2, "sink": "discard", "host_crc": True,
                      "keep_records": False, "grpc_conn_pool_size": 1, "cpus": pl["client"],
                      "rcvbuf": rcvk << 10})
        r.start()
        r.wait()
        r.reset_stats()
        r.set_reads_per_worker(args.reads)
        s0 = srv.stats()
        t = time.perf_counter()
        r.start()
        r.wait()
        el = time.perf_counter() - t
        s = r.summary()
        s1 = srv.stats()
        fr = max(1, s1["h2_data_frames"] - s0["h2_data_frames"])
        rs = max(1, s1["h2_responses"] - s0["h2_responses"])
        print(json.dumps({"rep": rep, "quantum_kib": q, "lead_kib": lead, "bufs_kib": bufs, "mib_s": round(s["bytes"] / el / 2**20, 1),
                          "p50_ms": round(s["p50_ms"], 3), "p99_ms": round(s["p99_ms"], 3),
                          "ttfb_p50_ms": round(s["ttfb_p50_ms"], 3), "ttfb_p99_ms": round(s["ttfb_p99_ms"], 3),
                          "errors": s["errors"],
                          "queue_wait_avg_us": round((s1["h2_queue_wait_us"] - s0["h2_queue_wait_us"]) / fr, 1),
                          "queue_wait_max_us": s1["h2_queue_wait_max_us"],
                          "srv_ttfb_avg_us": round((s1["h2_ttfb_us"] - s0["h2_ttfb_us"]) / rs, 1),
                          "srv_ttfb_max_us": s1["h2_ttfb_max_us"],
                          "slowest": [[round(v, 3) for v in x] for x in s["slowest"]]}), flush=True)
        del r
        srv.stop()
