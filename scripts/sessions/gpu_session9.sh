#!/bin/bash
# (1) raw pinned->HBM copy ceiling, SDMA vs blit kernels;
# (2) bench piece mode with smaller ring slots, and with HSA_ENABLE_SDMA=0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/s9
mkdir -p "$OUT"
timeout -k 10 180 python scripts/h2d_ceiling.py > $OUT/h2d_sdma.log 2>&1 || { echo "h2d rc=$?"; cat $OUT/h2d_sdma.log; exit 1; }
cat $OUT/h2d_sdma.log
HSA_ENABLE_SDMA=0 timeout -k 10 180 python scripts/h2d_ceiling.py > $OUT/h2d_blit.log 2>&1 || { echo "h2d blit rc=$?"; cat $OUT/h2d_blit.log; exit 1; }
cat $OUT/h2d_blit.log
b() {  # b <name> [env...] -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" --json-out $OUT/$name.json > $OUT/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $OUT/$name.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], d['p50_ms'], d['p99_ms'], d.get('host_landed_p50_ms'))"
}
for rep in 1 2; do
  b def_r$rep python bench.py --steps 20 --warmup 3 --single-stream-steps 0
  b s2x8_r$rep python bench.py --steps 20 --warmup 3 --single-stream-steps 0 --slot-bytes 2MiB --slots 8
  b s1x16_r$rep python bench.py --steps 20 --warmup 3 --single-stream-steps 0 --slot-bytes 1MiB --slots 16
  b blit_r$rep HSA_ENABLE_SDMA=0 python bench.py --steps 20 --warmup 3 --single-stream-steps 0
done
echo "session done"
