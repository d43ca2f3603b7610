#!/bin/bash
# Piece-mode A/B of the opt-in submit/wait knobs, interleaved x3:
# default vs GCSB_ASYNC_SUBMIT=1 (one submitter thread per device) vs GCSB_EVENT_SPIN=1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/s12
mkdir -p "$OUT"
b() {  # b <name> env...
  local name=$1; shift
  timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 --single-stream-steps 0 --compare-steps 0 \
    --json-out $OUT/$name.json > $OUT/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $OUT/$name.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], d['p50_ms'], d['p99_ms'], d.get('host_landed_p50_ms'))"
}
for rep in 1 2 3; do
  b def_r$rep GCSB_NOOP=1
  b async_r$rep GCSB_ASYNC_SUBMIT=1

  b spin_r$rep GCSB_EVENT_SPIN=1
done
echo "session done"
