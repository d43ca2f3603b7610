#!/bin/bash
# Targeted GPU debug session: the conn-ring tests over the HTTP/2 framings,
# then the framing-twin bench block under faulthandler.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dbg
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_conn_ring.py -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "many_streams" > $OUT/connring.log 2>&1
echo "connring rc=$?"; grep -E "PASS|FAIL" $OUT/connring.log | tail -40
timeout -k 10 300 env MALLOC_CHECK_=3 python -X faulthandler -u bench.py --steps 8 --warmup 2 \
  --blocks framing_twin --diag-out $OUT/diag.json > $OUT/bench_twin.log 2>&1
rc=$?
echo "bench twin rc=$rc"; tail -40 $OUT/bench_twin.log
