#!/usr/bin/env python3
"""Markdown table from scripts/measure_configs.sh summaries.

usage: configs_table.py <dir with *.json>   (prints the table to stdout)
"""
import glob
import json
import os
import sys


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/configs"
    rows = []
    for p in sorted(glob.glob(os.path.join(d, "*.json"))):
        s = json.load(open(p))
        name = os.path.splitext(os.path.basename(p))[0]
        ops = s.get("reads", 0) or s.get("writes", 0)
        size = s["bytes"] / ops if ops else 0
        host = ""
        if s.get("sink") == "gpu" and s.get("host_p50_ms"):
            host = f"{s['host_p50_ms']:.3f}"
        extra = s.get("extra") or {}
        note = f"list {extra['listed']} objs in {extra['list_ms']:.1f} ms" if "listed" in extra else ""
        rows.append((name, s.get("protocol", ""), s.get("sink", ""), s.get("workers", ""), ops,
                     f"{size / 2**20:.0f} MiB", f"{s['p50_ms']:.3f}", f"{s['p99_ms']:.3f}", host,
                     f"{s.get('mib_per_s', 0):.0f}", s.get("errors", 0), note))
    hdr = ("run", "protocol", "sink", "workers", "ops", "object", "p50 ms", "p99 ms", "host-landed p50 ms",
           "MiB/s", "errors", "note")
    print("| " + " | ".join(hdr) + " |")
    print("|" + "---|" * len(hdr))
    for r in rows:
        print("| " + " | ".join(str(x) for x in r) + " |")


if __name__ == "__main__":
    main()
