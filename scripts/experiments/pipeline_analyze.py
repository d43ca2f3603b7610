#!/usr/bin/env python3
"""Reads a rocprofv3 kernel + memory-copy + marker trace of the one-stream
bench (scripts/experiments/pipeline_trace.sh) and reports, per object read
(gcsb.read_object marker): H2D copies and slot CRC kernels, their durations,
how much of the copy time overlaps the receive, and the tail from the last
H2D copy's end to the last CRC kernel's end."""
import csv
import json
import statistics
import sys
from pathlib import Path

d = Path(sys.argv[1])


def rows(name):
    return list(csv.DictReader(open(next(d.glob(f"*{name}.csv")))))


copies = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows("memory_copy_trace")
          if r["Direction"].endswith("HOST_TO_DEVICE")]
kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows("kernel_trace")
        if "slot_kernel" in r["Kernel_Name"]]
reads = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows("marker_api_trace")
               if r["Function"] == "gcsb.read_object")
out = []
for i, (a, b) in enumerate(reads):
    nxt = reads[i + 1][0] if i + 1 < len(reads) else b + 50_000_000
    cs = [c for c in copies if a <= c[0] < nxt]
    ks = [k for k in kern if a <= k[0] < nxt]
    if not cs or not ks:
        continue
    last_copy_end = max(e for _, e in cs)
    last_kernel_end = max(e for _, e in ks)
    out.append({
        "read_ms": (b - a) / 1e6,
        "copies": len(cs),
        "copy_us_p50": statistics.median((e - s) / 1e3 for s, e in cs),
        "copy_GBps_p50": statistics.median(2 * 2**20 / max(e - s, 1) for s, e in cs),
        "crc_kernels": len(ks),
        "crc_us_p50": statistics.median((e - s) / 1e3 for s, e in ks),
        "gpu_busy_fraction": (sum(e - s for s, e in cs) + sum(e - s for s, e in ks)) / max(b - a, 1),
        "tail_last_copy_to_last_crc_us": (last_kernel_end - last_copy_end) / 1e3,
        "read_end_minus_last_crc_us": (b - last_kernel_end) / 1e3,
        "first_copy_after_read_start_us": (min(s for s, _ in cs) - a) / 1e3,
    })
summary = {k: round(statistics.median(o[k] for o in out), 3) for k in out[0]} if out else {}
print(json.dumps({"reads": len(out), "median": summary}, indent=1))
