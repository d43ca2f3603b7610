#!/bin/bash
# CRC kernel check on the GPU box: GPU CRC/sink tests, the kernel bench
# (bulk rate + per-launch time of slot-sized batches), and rocprofv3 kernel
# stats of the headline bench.  Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/crc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_crc32c.py tests/test_gpu_sink.py tests/test_gpu_large_object.py \
  -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python scripts/crc_kernel_bench.py > $OUT/crc_bench.jsonl 2>&1 || { tail $OUT/crc_bench.jsonl; exit 1; }
cat $OUT/crc_bench.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
  python bench.py --steps 10 --warmup 2 --side-steps 0 > $OUT/bench_prof.log 2>&1 || { tail $OUT/bench_prof.log; exit 1; }
grep '^{' $OUT/bench_prof.log | cut -c1-400
cut -d, -f1-4,6,7 $OUT/prof/bench_kernel_stats.csv | head -6
echo done
