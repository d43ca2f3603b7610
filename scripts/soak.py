#!/usr/bin/env python3
"""Soak of the reference's operating mode through the reference's own driver.

VERDICT r3 next #6.  The reference runs `execute_pb.sh <n>`: 48 workers
re-reading ~100 MB objects over gRPC (pool 1) and then over HTTP
(/root/reference/execute_pb.sh:1-9, main.go:36,38,52), exporting the
read-latency distribution every 30 s (metrics_exporter.go:44) and feeding the
latency files to the README histogram (README.md:15-35).  This driver runs
scripts/execute_pb.sh with

  -start-fake-server -worker 48 -sink gpu -duration <d> -metrics-jsonl ...

and, every --sample-s seconds, records the benchmark process's RSS and open
file descriptors (flat = no leak), then runs scripts/histogram.py on both
latency files.  One JSON line per sample on stdout, a summary in
<out>/soak.json:

  python scripts/soak.py --out gpurun_out/r4_soak --duration 120
"""
import argparse
import json
import os
import subprocess
import sys
import time

import psutil

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench_procs(root: psutil.Process) -> list:
    """The gcsbench python processes under the driver."""
    out = []
    try:
        for p in root.children(recursive=True):
            try:
                cmd = p.cmdline()
            except psutil.Error:
                continue
            if len(cmd) >= 3 and cmd[0].startswith("python") and "custom_go_client_benchmark_amd" in cmd:
                out.append(p)
    except psutil.Error:
        pass
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/soak")
    ap.add_argument("--duration", default="120s")
    ap.add_argument("--workers", type=int, default=48)
    ap.add_argument("--object-size", type=int, default=100 << 20)
    ap.add_argument("--sink", default="gpu")
    ap.add_argument("--metrics-interval", default="30s")
    ap.add_argument("--sample-s", type=float, default=10.0)
    ap.add_argument("--exp", default="soak")
    args = ap.parse_args()
    out = os.path.abspath(args.out)
    os.makedirs(out, exist_ok=True)
    gargs = (f"-start-fake-server -worker {args.workers} -read-call-per-worker 1000000 -duration {args.duration} "
             f"-fake-object-size {args.object_size} -sink {args.sink} -metrics-interval {args.metrics_interval} "
             f"-metrics-jsonl {out}/metrics_%p.jsonl -summary-json {out}/summary_%p.json")
    env = dict(os.environ, GCSB_ARGS=gargs, GCSB_RESULTS_DIR=os.path.join(out, "uploaded"), GCSB_RESULTS_URI="")
    env["PATH"] = "/nonexistent-gsutil:" + env.get("PATH", "")
    t0 = time.time()
    drv = subprocess.Popen(["bash", os.path.join(HERE, "scripts", "execute_pb.sh"), args.exp], cwd=out, env=env,
                           stderr=open(os.path.join(out, "driver.err"), "w"))
    root = psutil.Process(drv.pid)
    samples = []
    while drv.poll() is None:
        time.sleep(args.sample_s)
        for p in bench_procs(root):
            try:
                with p.oneshot():
                    proto = "grpc" if "grpc" in p.cmdline() else "http"
                    s = {"t_s": round(time.time() - t0, 1), "pid": p.pid, "protocol": proto,
                         "rss_mib": round(p.memory_info().rss / 2**20, 1), "fds": p.num_fds(),
                         "threads": p.num_threads()}
            except psutil.Error:
                continue
            samples.append(s)
            print(json.dumps(s), flush=True)
    rc = drv.wait()
    res = {"rc": rc, "wall_s": round(time.time() - t0, 1), "gcsb_args": gargs, "samples": samples}
    for proto in ("grpc", "http"):
        r = {}
        lat = os.path.join(out, f"{proto}_{args.exp}.txt")
        if os.path.exists(lat):
            h = subprocess.run([sys.executable, os.path.join(HERE, "scripts", "histogram.py"), lat],
                               capture_output=True, text=True, timeout=600)
            r["histogram"] = h.stdout.strip().splitlines()[1:]
            with open(os.path.join(out, f"histogram_{proto}.txt"), "w") as f:
                f.write(h.stdout)
        m = os.path.join(out, f"metrics_{proto}.jsonl")
        if os.path.exists(m):
            with open(m) as f:
                r["exporter_intervals"] = sum(1 for line in f if line.strip())
        sj = os.path.join(out, f"summary_{proto}.json")
        if os.path.exists(sj):
            with open(sj) as f:
                s = json.load(f)
            r.update({k: s.get(k) for k in ("reads", "errors", "verified", "bytes", "mib_per_s", "p50_ms", "p99_ms",
                                             "first_error")})
        ps = [x for x in samples if x["protocol"] == proto]
        if ps:
            r["rss_mib_first_last_max"] = [ps[0]["rss_mib"], ps[-1]["rss_mib"], max(x["rss_mib"] for x in ps)]
            r["fds_first_last_max"] = [ps[0]["fds"], ps[-1]["fds"], max(x["fds"] for x in ps)]
        res[proto] = r
    with open(os.path.join(out, "soak.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "samples"}), flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
