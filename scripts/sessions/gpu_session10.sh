#!/bin/bash
# Tapered (guided) piece schedule A/B on the headline bench, interleaved x3:
# fixed 8 MiB pieces vs taper floors 2 / 4 MiB, and 16 MiB pieces tapered to 2 MiB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/s10
mkdir -p "$OUT"
b() {  # b <name> bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --single-stream-steps 0 "$@" --json-out $OUT/$name.json \
    > $OUT/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $OUT/$name.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], d['p50_ms'], d['p99_ms'], d.get('host_landed_p50_ms'), d.get('slice_skew_ms'))"
}
for rep in 1 2 3; do
  b fixed8_r$rep
  b taper2_r$rep --piece-min-bytes 2MiB
  b taper4_r$rep --piece-min-bytes 4MiB
  b p16taper2_r$rep --piece-bytes 16MiB --piece-min-bytes 2MiB
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_sink.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu_sink.log 2>&1 || { echo "pytest rc=$?"; tail -20 $OUT/pytest_gpu_sink.log; exit 1; }
tail -2 $OUT/pytest_gpu_sink.log
echo "session done"
