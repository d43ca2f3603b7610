#!/bin/bash
# 48-worker 1 MiB reads (the reference's default concurrency) at two run
# lengths: with 100 reads per worker each worker's first read (connection
# dial) is 1 % of the reads, i.e. the p99; the summary splits first reads
# from steady-state reads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/tail}
mkdir -p "$OUT"
export TMPDIR=/tmp
MIB=1048576
for p in http grpc; do
  for n in 100 2000; do
    name=c1_${p}_w48_n$n
    timeout -k 10 200 ./gcsbench -start-fake-server -latency-file /dev/null -summary-json "$OUT/$name.json" \
      -client-protocol $p -worker 48 -read-call-per-worker $n -fake-object-size $MIB > "$OUT/$name.log" 2>&1 \
      || { tail -n 5 "$OUT/$name.log"; exit 1; }
    python3 - "$name" "$OUT/$name.json" <<'PY' | tee -a "$OUT/summary.txt"
import json, sys
d = json.load(open(sys.argv[2]))
keys = ("mib_per_s", "p50_ms", "p99_ms", "first_read_p50_ms", "first_read_max_ms", "steady_p50_ms", "steady_p99_ms")
print(f"{sys.argv[1]:20s}", {k: round(d[k], 3) for k in keys}, "p99/p50", round(d["p99_ms"] / d["p50_ms"], 2),
      "steady", round(d["steady_p99_ms"] / d["steady_p50_ms"], 2))
PY
  done
done
