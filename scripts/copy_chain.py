#!/usr/bin/env python3
"""Per-burst H2D copy and CRC-kernel timing from a rocprofv3 SQLite trace
(`--kernel-trace --memory-copy-trace`): for every burst of host-to-device
copies (bursts split at gaps > 20 ms, i.e. per bench block or pass) the
copies' rate, their duration percentiles, how many were in flight at once
(fraction of the burst's span at each concurrency), and the gap from a
copy's end to the start of the next kernel on the same stream (the slot's
CRC launch queued behind it).

  copy_chain.py OUT_DIR_OR_DB [--min-copies 500]
"""
import bisect
import glob
import os
import sqlite3
import sys


def pct(v, q):
    return v[min(len(v) - 1, int(len(v) * q))] if v else 0.0


def bursts(rows, gap_ns=20e6):
    out, cur = [], []
    for r in rows:
        if cur and r[0] - cur[-1][1] > gap_ns:
            out.append(cur)
            cur = []
        cur.append(r)
    if cur:
        out.append(cur)
    return out


def analyse(db: str, min_copies: int) -> list[dict]:
    c = sqlite3.connect(db)
    copies = list(c.execute("select start, end, size, stream_id from memory_copies "
                            "where name like '%HOST_TO_DEVICE%' order by start"))
    kernels = list(c.execute("select start, end, stream_id from kernels order by start"))
    by_stream = {}
    for k in kernels:
        by_stream.setdefault(k[2], []).append(k)
    starts = {s: [k[0] for k in ks] for s, ks in by_stream.items()}
    res = []
    for b in bursts(copies):
        if len(b) < min_copies:
            continue
        t0, t1 = b[0][0], max(r[1] for r in b)
        ev = sorted([(r[0], 1) for r in b] + [(r[1], -1) for r in b])
        conc, last, hist = 0, t0, {}
        for t, d in ev:
            hist[conc] = hist.get(conc, 0) + (t - last)
            conc += d
            last = t
        durs = sorted((r[1] - r[0]) / 1e3 for r in b)
        gaps = []
        for s, e, _, st in b:
            ks, ss = by_stream.get(st, []), starts.get(st, [])
            i = bisect.bisect_left(ss, e)
            if i < len(ks):
                gaps.append((ks[i][0] - e) / 1e3)
        gaps.sort()
        res.append({"copies": len(b), "span_ms": round((t1 - t0) / 1e6, 2),
                    "gbps": round(sum(r[2] for r in b) / (t1 - t0), 2),
                    "mean_kib": round(sum(r[2] for r in b) / len(b) / 1024, 1),
                    "streams": len(set(r[3] for r in b)),
                    "copy_us_p10_p50_p90": [round(pct(durs, q), 1) for q in (0.1, 0.5, 0.9)],
                    "in_flight_frac": {k: round(v / (t1 - t0), 3) for k, v in sorted(hist.items())},
                    "copy_end_to_kernel_us_p50_p90": [round(pct(gaps, q), 1) for q in (0.5, 0.9)]})
    return res


def main():
    import json

    a = sys.argv[1] if len(sys.argv) > 1 else "."
    m = int(sys.argv[sys.argv.index("--min-copies") + 1]) if "--min-copies" in sys.argv else 500
    dbs = [a] if a.endswith(".db") else sorted(glob.glob(os.path.join(a, "**", "*.db"), recursive=True))
    for db in dbs:
        for r in analyse(db, m):
            print(json.dumps({"db": os.path.basename(db), **r}))


if __name__ == "__main__":
    main()
