#!/bin/bash
# Headline bench with the HTTP comparison (`compare`), twice, and an HTTP-headline run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/s11
mkdir -p "$OUT"
for name in grpc_r1 grpc_r2 http_r1; do
  proto=${name%_r*}
  timeout -k 10 300 python bench.py --protocol $proto --json-out $OUT/$name.json > $OUT/$name.log 2>&1 \
    || { echo "$name rc=$?"; tail -5 $OUT/$name.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], d['p50_ms'], d['p99_ms'], 'single', d.get('single_stream_mib_s'), 'compare', d.get('compare'))"
done
echo "session done"
