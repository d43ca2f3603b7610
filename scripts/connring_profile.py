#!/usr/bin/env python3
"""Connection-ring (ConnRing) profile: one multiplexed gRPC connection, every
worker's stream landing through one pinned ring -> H2D -> HBM with the CRC32C
kernel (csrc/gpu/engine.hip ConnRing).  VERDICT r4 item 4.

  run --block list_read   config 3: 8 workers read 1000 x 1 MiB objects
  run --block ref100      the reference's default at its object size:
                          48 workers x 100 MiB (main.go:36,52), pool 1
  summarize DIR [DIR..]   joins the run's JSON with rocprofv3's --stats CSVs:
                          H2D copies per MiB, mean copy size, CRC launches
                          per ring slot, kernel us per slot

Run under the profiler, the program itself after `--`:
  rocprofv3 --kernel-trace --memory-copy-trace --stats -d OUT -o run -- \\
      python3 scripts/connring_profile.py run --block ref100 --json OUT/run.json
"""
import argparse
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def run(args) -> None:
    sys.path.insert(0, ROOT)
    import torch  # noqa: F401

    import custom_go_client_benchmark_amd as pkg
    from custom_go_client_benchmark_amd.parallel import affinity
    from custom_go_client_benchmark_amd.utils import cpuacct

    n = pkg._native
    pl = affinity.plan(0, "same", 0)
    if pl.get("aux"):
        n.set_submitter_cpus(pl["aux"])
    srv = n.Server({"port": 0, "md5": False, "cpus": pl["server"], "retain_uploads": False})
    srv.start()
    cfg = {"protocol": "grpc", "endpoint": srv.url, "bucket": "b", "sink": "gpu", "device": 0,
           "grpc_conn_pool_size": 1, "conn_ring": True, "conn_ring_slots": 4, "conn_ring_slot_bytes": 1 << 20,
           "keep_records": False, "cpus": pl["client"], "retry_initial_s": 0.05, "tcp_congestion": "cubic",
           "loopback_rto_min": True, "reader_cpus": pl.get("reader_cpus")}
    if args.block == "list_read":
        srv.add_synthetic("b", "c3/file_", "", 0, 1000, 1 << 20)
        names = [f"c3/file_{i}" for i in range(1000)]
        cfg.update(workers=8, object_names=names, rcvbuf=64 << 20)
        warm, reads = 125, 125
    else:
        srv.add_synthetic("b", "r100/file_", "", 0, 48, 100 << 20)
        cfg.update(workers=48, object_prefix="r100/file_", rcvbuf=0)
        warm, reads = 1, args.reads
    r = n.Runner({**cfg, "reads_per_worker": warm})
    r.start()
    r.wait()
    r.reset_stats()
    cpuacct.label_runtime_threads()
    r.set_reads_per_worker(reads)
    t0 = cpuacct.thread_cpu()
    w0 = time.perf_counter()
    r.start()
    r.wait()
    el = time.perf_counter() - w0
    d = cpuacct.delta_by_name(t0, cpuacct.thread_cpu())
    s = r.summary()
    gib = max(s["bytes"], 1) / (1 << 30)
    out = {"block": args.block, "mib_s": round(s["bytes"] / el / (1 << 20), 1), "p50_ms": round(s["p50_ms"], 3),
           "p99_ms": round(s["p99_ms"], 3), "reads": s["reads"], "verified": s["verified"], "errors": s["errors"],
           "timed_bytes": s["bytes"], "cpu_s_per_gib": {k: round(v / gib, 4) for k, v in d.items() if v / gib > 5e-4},
           # the ring's counters cover the warm-up too (the profile does as well)
           "conn_ring": r.conn_ring_stats(), "warmup_bytes": warm * cfg["workers"] * (1 << 20 if args.block ==
                                                                                         "list_read" else 100 << 20)}
    srv.stop()
    text = json.dumps(out)
    print(text, flush=True)
    if args.json:
        with open(args.json, "w") as f:
            f.write(text + "\n")


def _stats(path: str) -> dict:
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            out[row["Name"]] = {"calls": int(row["Calls"]), "total_ns": int(row["TotalDurationNs"]),
                                "avg_ns": float(row["AverageNs"])}
    return out


def _db_stats(path: str) -> tuple[dict, dict]:
    """rocprofv3's SQLite output (its default format on ROCm 7): the same
    per-name calls / total / average as the --stats CSVs."""
    import sqlite3

    c = sqlite3.connect(path)
    k = {n: {"calls": cnt, "total_ns": int(tot), "avg_ns": tot / cnt}
         for n, cnt, tot in c.execute("select name, count(*), sum(duration) from kernels group by name")}
    m = {n: {"calls": cnt, "total_ns": int(tot), "avg_ns": tot / cnt, "bytes": int(b)}
         for n, cnt, tot, b in c.execute("select name, count(*), sum(duration), sum(size) from memory_copies "
                                         "group by name")}
    return k, m


def summarize(dirs) -> None:
    for d in dirs:
        runs = glob.glob(os.path.join(d, "**", "run.json"), recursive=True) or glob.glob(os.path.join(d, "*.json"))
        ks = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        ms = glob.glob(os.path.join(d, "**", "*memory_copy_stats.csv"), recursive=True)
        dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
        if not runs or not ((ks and ms) or dbs):
            print(json.dumps({"dir": d, "error": "missing run.json / kernel_stats / memory_copy_stats / .db"}))
            continue
        r = json.loads(open(runs[0]).read().strip().splitlines()[-1])
        k, m = (_stats(ks[0]), _stats(ms[0])) if ks and ms else _db_stats(dbs[0])
        crc = {name: v for name, v in k.items() if "crc32c" in name}
        h2d = m.get("MEMORY_COPY_HOST_TO_DEVICE", {"calls": 0, "total_ns": 0, "avg_ns": 0})
        mib = (r["timed_bytes"] + r["warmup_bytes"]) / (1 << 20)
        slots = (r["conn_ring"] or {}).get("slots_filled", 0) or 1
        crc_calls = sum(v["calls"] for v in crc.values())
        crc_ns = sum(v["total_ns"] for v in crc.values())
        print(json.dumps({
            "dir": d, "block": r["block"], "mib_s_under_profiler": r["mib_s"], "mib_moved": round(mib, 1),
            "h2d_copies": h2d["calls"], "h2d_copies_per_mib": round(h2d["calls"] / mib, 3),
            "mean_copy_kib": round((h2d.get("bytes") or mib * (1 << 20)) / 1024 / max(1, h2d["calls"]), 1),
            "h2d_avg_us": round(h2d["avg_ns"] / 1e3, 2),
            "h2d_gbps_per_copy": round((h2d.get("bytes") or mib * (1 << 20)) / max(1, h2d["total_ns"]), 2),
            "ring_slots_filled": slots, "crc_launches": crc_calls,
            "crc_launches_per_slot": round(crc_calls / slots, 3),
            "crc_kernel_us_per_slot": round(crc_ns / 1e3 / slots, 2),
            "crc_kernel_avg_us": round(crc_ns / 1e3 / max(1, crc_calls), 2),
            "segments_per_slot": round((r["conn_ring"] or {}).get("segments", 0) / slots, 3),
            "cpu_s_per_gib": r["cpu_s_per_gib"]}))


def main() -> None:
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("run")
    a.add_argument("--block", choices=["list_read", "ref100"], default="list_read")
    a.add_argument("--reads", type=int, default=2, help="ref100: timed reads per worker")
    a.add_argument("--json", default="")
    b = sub.add_parser("summarize")
    b.add_argument("dirs", nargs="+")
    args = ap.parse_args()
    run(args) if args.cmd == "run" else summarize(args.dirs)


if __name__ == "__main__":
    main()
