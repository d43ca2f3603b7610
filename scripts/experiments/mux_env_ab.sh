#!/bin/bash
# Env A/B for multiplexed discard-sink reads (one connection, pool 1),
# interleaved, 48 x 1 MiB, 8 x 1 MiB, 1 x 256 MiB.  AB_VAR (default
# GCSB_DEFER_CRC: 1 = host CRC on each worker thread, 0 = inline on the
# connection's reader thread; GCSB_CONN_CORE: 1 = the reader thread gets a
# physical core of its own) is set to 1 and 0.  PROTO = grpc | http2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
AB_VAR=${AB_VAR:-GCSB_DEFER_CRC}
OUT=${OUT:-gpurun_out/${PROTO:-grpc}_${AB_VAR}}
mkdir -p "$OUT"
export TMPDIR=/tmp
M=1048576
CASES=("w48|-worker 48 -read-call-per-worker 400 -fake-object-size $M"
       "w8|-worker 8 -read-call-per-worker 1000 -fake-object-size $M"
       "w1_256m|-worker 1 -read-call-per-worker 20 -fake-object-size $((256 * M))")
for rep in 1 2 3; do
  for c in "${CASES[@]}"; do
    name=${c%%|*}; args=${c#*|}
    for d in 1 0; do
      env $AB_VAR=$d timeout -k 10 200 ./gcsbench -start-fake-server -latency-file /dev/null \
        -summary-json "$OUT/run.json" -client-protocol ${PROTO:-grpc} $args > "$OUT/run.log" 2>&1 \
        || { tail -n 5 "$OUT/run.log"; exit 1; }
      python3 - "$name" "$d" "$OUT/run.json" <<'PY' | tee -a "$OUT/runs.jsonl"
import json, sys
d = json.load(open(sys.argv[3]))
print(json.dumps({"case": sys.argv[1], "defer": int(sys.argv[2]),
                  **{k: round(d[k], 3) for k in ("mib_per_s", "p50_ms", "p99_ms")},
                  "verified": d["verified"], "reads": d["reads"]}))
PY
    done
  done
done
python3 - "$OUT/runs.jsonl" <<'PY' | tee "$OUT/summary.txt"
import json, sys, statistics, collections
v = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); v[(d["case"], d["defer"])].append((d["mib_per_s"], d["p50_ms"], d["p99_ms"]))
for k in sorted(v):
    xs = v[k]
    print("%-8s defer=%d MiB/s median %8.1f (%s)  p50 %.3f  p99 %.3f" % (k[0], k[1], statistics.median(x[0] for x in xs),
          ", ".join("%.0f" % x[0] for x in xs), statistics.median(x[1] for x in xs), statistics.median(x[2] for x in xs)))
PY
