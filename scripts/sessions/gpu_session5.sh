#!/bin/bash
# Piece-mode (dynamic load balance) sliced reads: GPU tests, then the headline
# bench at piece sizes 0 (fixed shares) / 4 / 8 / 16 MiB, interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/s5
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -20 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for rep in 1 2; do
  for pb in 0 4MiB 8MiB 16MiB; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --single-stream-steps 0 --piece-bytes $pb \
      --json-out $OUT/bench_p${pb}_r$rep.json > $OUT/bench_p${pb}_r$rep.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench_p${pb}_r$rep.log; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_p${pb}_r$rep.json'));print('piece=$pb rep=$rep', d['value'], d['p50_ms'], d['p99_ms'], d['slice_skew_ms'], d['rank0_cpu']['cpu_s_per_gib_by_thread'])"
  done
done
for pb in 4MiB 8MiB; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --single-stream-steps 0 --piece-bytes $pb --protocol http \
    --json-out $OUT/bench_http_p${pb}.json > $OUT/bench_http_p${pb}.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_http_p${pb}.json'));print('http piece=$pb', d['value'], d['p50_ms'], d['p99_ms'], d['slice_skew_ms'])"
done
echo "session done"
