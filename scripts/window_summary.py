#!/usr/bin/env python3
"""Summarize the paired headline's per-chunk windows over many bench runs
(VERDICT r4 item 6): for every run, the 4 headline chunks' MiB/s and the
base / nodma arms beside them, the receiving thread's CPU-s/GiB, its core's
clock and the host's NUMA migrations / compaction stalls during each chunk,
and the slow windows benchmark/report.attribute_windows named.

  python3 scripts/window_summary.py DIAG.json [DIAG.json ...]   (bench --diag-out files)
"""
import json
import sys


def main(paths):
    runs = []
    for p in paths:
        try:
            d = json.load(open(p))
        except (OSError, ValueError) as e:
            print(f"{p}: {e}", file=sys.stderr)
            continue
        pr = d.get("paired") or {}
        line = d.get("line") or {}
        runs.append((p, line, pr))
    slow_total = 0
    print(f"{'run':<40} {'value':>9} {'vs_base':>7} {'paired':>7} {'nodma':>6} {'frac':>6}  chunks head/base/nodma MiB/s")
    for p, line, pr in runs:
        chunks = " | ".join(
            "/".join(str(int(x)) for x in (h, b, n))
            for h, b, n in zip(pr.get("head_mib_s", []), pr.get("base_mib_s", []),
                               pr.get("nodma_mib_s", [0] * len(pr.get("head_mib_s", [])))))
        print(f"{p[-40:]:<40} {line.get('value', 0):>9.0f} {line.get('vs_baseline') or 0:>7.3f} "
              f"{line.get('vs_baseline_paired') or 0:>7.3f} {line.get('headline_vs_nodma') or 0:>6.3f} "
              f"{line.get('headline_frac_of_ceiling') or 0:>6.3f}  {chunks}")
        for w in pr.get("slow_windows", []):
            slow_total += 1
            print(f"    slow chunk {w['chunk']}: {w['mib_s']} MiB/s vs median {w['median_mib_s']}: {w['cause']}")
    vals = sorted(line.get("vs_baseline_paired") for _, line, _ in runs if line.get("vs_baseline_paired"))
    nod = sorted(line.get("headline_vs_nodma") for _, line, _ in runs if line.get("headline_vs_nodma"))
    if vals:
        print(f"\n{len(runs)} runs; vs_baseline_paired median {vals[len(vals) // 2]:.3f} "
              f"(min {vals[0]:.3f}, max {vals[-1]:.3f}); headline_vs_nodma median "
              f"{nod[len(nod) // 2] if nod else 0:.3f}; slow windows named: {slow_total}")
    # every window's fields, for the record
    print("\nwindows (run, chunk, arm, MiB/s, recv CPU-s/GiB, run-queue ms, clock MHz, numa migrated, compact stalls):")
    for p, _, pr in runs:
        for w in pr.get("windows", []):
            print(f"  {p[-24:]:<24} {w['chunk']} {w['arm']:<5} {w['mib_s']:>8} {w.get('recv_cpu_s_per_gib')} "
                  f"{w.get('run_delay_ms')} {w.get('clock_mhz')} {w.get('numa_pages_migrated')} {w.get('compact_stall')}")


if __name__ == "__main__":
    main(sys.argv[1:])
