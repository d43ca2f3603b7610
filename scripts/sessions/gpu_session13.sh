#!/bin/bash
# bench --event-wait spin (new bench default) vs block, interleaved x3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/s13
mkdir -p "$OUT"
for rep in 1 2 3; do
  for ew in block spin; do
    name=${ew}_r$rep
    timeout -k 10 300 python bench.py --event-wait $ew --steps 20 --warmup 3 --single-stream-steps 0 --compare-steps 0 \
      --json-out $OUT/$name.json > $OUT/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $OUT/$name.log; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], d['p50_ms'], d['p99_ms'], d['config']['event_wait'])"
  done
done
echo "session done"
