#!/bin/bash
# Named gcsbench runs against the in-process synthetic endpoint, one summary
# line each.   RUNS="name|args;name|args"  REPS=1  OUT=gpurun_out/cli
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/cli}
mkdir -p "$OUT"
export TMPDIR=/tmp
IFS=';' read -ra RS <<< "$RUNS"
for rep in $(seq 1 ${REPS:-1}); do
  for r in "${RS[@]}"; do
    name=${r%%|*}; args=${r#*|}
    timeout -k 10 200 ./gcsbench -start-fake-server -latency-file /dev/null -summary-json "$OUT/$name.json" \
      $args > "$OUT/$name.log" 2>&1 || { tail -n 5 "$OUT/$name.log"; exit 1; }
    python3 - "$name" "$OUT/$name.json" <<'PY' | tee -a "$OUT/summary.txt"
import json, sys
d = json.load(open(sys.argv[2]))
keys = ("mib_per_s", "p50_ms", "p99_ms", "steady_p99_ms", "first_read_p50_ms", "verified", "reads")
print(f"{sys.argv[1]:24s}", {k: (round(d[k], 3) if isinstance(d.get(k), float) else d.get(k)) for k in keys})
PY
  done
done
