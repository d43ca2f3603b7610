#!/usr/bin/env python3
"""Ranges and medians of bench.py lines over several runs (the README /
BASELINE.md round tables).

  bench_ranges.py profiles/r6_k/bench1.json profiles/r6_v/bench*.json ...

Each file holds bench.py's stdout (its last line is the JSON line).  Prints
one row per quantity: min – max (median) over the files that carry it.
"""
import json
import sys

TOP = ["value", "vs_baseline_paired", "vs_baseline", "headline_vs_nodma", "headline_vs_tcp_paired",
       "headline_vs_ref_effective"]
BLOCKS = ["ref_framing", "cpu_baseline", "compare", "sliced", "ref_default_grpc", "ref_default_grpc_ref",
          "ref_default_http", "ref_default_100m_grpc_gpu", "ref_default_100m_http_gpu", "list_read_grpc",
          "list_read_grpc_ref", "list_read_http", "c1_http_cpu", "write", "write_composite"]


def line(path: str) -> dict:
    return json.loads(open(path).read().strip().splitlines()[-1])


def rng(vals, nd):
    v = sorted(x for x in vals if isinstance(x, (int, float)))
    if not v:
        return "-"
    f = (lambda x: f"{x:,.0f}") if nd == 0 else (lambda x: f"{x:.{nd}f}")
    return f"{f(v[0])} – {f(v[-1])} ({f(v[len(v) // 2])}), n={len(v)}"


def main() -> None:
    runs = [line(p) for p in sys.argv[1:]]
    print(f"{len(runs)} runs")
    for k in TOP:
        print(f"{k}: {rng([r.get(k) for r in runs], 0 if k == 'value' else 3)}")
    print(f"p99/p50: {rng([r['p99_ms'] / r['p50_ms'] for r in runs if r.get('p50_ms')], 2)}")
    for b in BLOCKS:
        blk = [r.get(b) or {} for r in runs]
        print(f"{b}: MiB/s {rng([x.get('mib_s') for x in blk], 0)}; frac_of_bound "
              f"{rng([x.get('frac_of_bound') for x in blk], 2)}")
    print(f"ref_framing paired: {rng([(r.get('ref_framing') or {}).get('vs_baseline_paired') for r in runs], 3)}")
    print(f"100m gRPC GPU vs discard twin: "
          f"{rng([(r.get('ref_default_100m_grpc_gpu') or {}).get('vs_discard_twin') for r in runs], 2)}")
    wc = [(r.get("write_composite") or {}).get("mib_s", 0) / r["write"]["mib_s"]
          for r in runs if (r.get("write") or {}).get("mib_s")]
    print(f"write_composite / write: {rng(wc, 2)}")


if __name__ == "__main__":
    main()
