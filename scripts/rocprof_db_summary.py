#!/usr/bin/env python3
"""Per-name kernel and memory-copy statistics from rocprofv3's SQLite output
(its default format on ROCm 7; `--kernel-trace --memory-copy-trace`).

  rocprof_db_summary.py OUT_DIR [--md]   -> JSON (or a markdown table) on stdout
"""
import glob
import json
import os
import sqlite3
import sys


def summary(path: str) -> dict:
    c = sqlite3.connect(path)
    out = {"db": os.path.basename(path), "kernels": [], "memory_copies": []}
    for name, cnt, tot, mn, mx in c.execute(
            "select name, count(*), sum(duration), min(duration), max(duration) from kernels group by name "
            "order by sum(duration) desc"):
        out["kernels"].append({"name": name[:100], "calls": cnt, "total_ms": round(tot / 1e6, 3),
                               "avg_us": round(tot / cnt / 1e3, 2), "min_us": round(mn / 1e3, 2),
                               "max_us": round(mx / 1e3, 2)})
    for name, cnt, tot, b in c.execute(
            "select name, count(*), sum(duration), sum(size) from memory_copies group by name "
            "order by sum(duration) desc"):
        out["memory_copies"].append({"name": name, "calls": cnt, "total_ms": round(tot / 1e6, 3),
                                     "avg_us": round(tot / cnt / 1e3, 2), "mean_kib": round(b / cnt / 1024, 1),
                                     "gbps_per_copy": round(b / max(1, tot), 2)})
    return out


def main() -> None:
    dbs = sorted(glob.glob(os.path.join(sys.argv[1], "**", "*.db"), recursive=True))
    res = [summary(p) for p in dbs]
    if "--md" not in sys.argv:
        print(json.dumps(res, indent=1))
        return
    for r in res:
        print(f"### {r['db']}\n\n| kernel | calls | avg us | min / max us | total ms |\n|---|---|---|---|---|")
        for k in r["kernels"][:12]:
            print(f"| `{k['name']}` | {k['calls']} | {k['avg_us']} | {k['min_us']} / {k['max_us']} | {k['total_ms']} |")
        print("\n| copy | calls | mean KiB | avg us | GB/s per copy | total ms |\n|---|---|---|---|---|---|")
        for m in r["memory_copies"]:
            print(f"| {m['name']} | {m['calls']} | {m['mean_kib']} | {m['avg_us']} | {m['gbps_per_copy']} | "
                  f"{m['total_ms']} |")
        print()


if __name__ == "__main__":
    main()
