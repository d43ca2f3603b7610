#!/bin/bash
# A/B of GpuSink hand-off modes on the headline bench (interleaved rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for r in 1 2 3; do
  for mode in "1 0" "0 0" "1 1" "0 1"; do
    set -- $mode
    name=async$1_spin$2_r$r
    GCSB_ASYNC_SUBMIT=$1 GCSB_EVENT_SPIN=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 \
      --json-out "$OUT/$name.json" > "$OUT/$name.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -3 "$OUT/$name.log"; exit $rc; fi
    python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], d['p50_ms'], d['p99_ms'], d.get('single_stream_mib_s'), d.get('single_stream_p50_ms'))"
  done
done
