#!/usr/bin/env python3
"""Merge per-rank latency files into exact node-level statistics.

SURVEY.md §2.4: "Exact global percentiles come from merging per-rank latency
files on the host, not from collectives."  Each input holds one "<ms>ms" line
per read (the reference's output contract, execute_pb.sh / README histogram);
the output uses the reference's FS-tool stats (ssd_test/main.go:144-164):
Average / P20 / P50 / P90 / p99 / Min / Max, floor-index nearest rank.

    python scripts/merge_latency.py lat.rank*.txt [--json]
"""
import json
import sys


def read_ms(path):
    out = []
    with open(path) as f:
        for line in f:
            t = line.strip()
            if t.endswith("ms"):
                t = t[:-2]
            if t:
                out.append(float(t))
    return out


def stats(v):
    v = sorted(v)
    n = len(v)
    if n == 0:
        return {"count": 0}

    def pct(k):
        return v[n * k // 100]

    return {"count": n, "avg_ms": sum(v) / n, "p20_ms": pct(20), "p50_ms": pct(50), "p90_ms": pct(90),
            "p99_ms": pct(99), "min_ms": v[0], "max_ms": v[-1]}


def main(argv):
    as_json = "--json" in argv
    files = [a for a in argv if a != "--json"]
    if not files:
        print(__doc__, file=sys.stderr)
        return 2
    per = {f: stats(read_ms(f)) for f in files}
    allv = []
    for f in files:
        allv.extend(read_ms(f))
    node = stats(allv)
    if as_json:
        print(json.dumps({"node": node, "per_file": per}))
    else:
        for k in ("count", "avg_ms", "p20_ms", "p50_ms", "p90_ms", "p99_ms", "min_ms", "max_ms"):
            val = node.get(k)
            print(f"{k}: {val:.3f}" if isinstance(val, float) else f"{k}: {val}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
