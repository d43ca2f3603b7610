#!/bin/bash
# Slot CRC kernel in the read pipeline: correctness, back-to-back launch time,
# then rocprofv3 kernel stats of short single-stream benches (fresh slot bytes
# from SDMA, L2-cold tables) for waves-per-workgroup 2 / 4 / 8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/crc_pipe}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_crc32c.py tests/test_gpu_sink.py tests/test_gpu_large_object.py -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
PROBES=0 timeout -k 10 120 python scripts/experiments/crc_latency_probe.py 2>/dev/null | grep '^{' | tee $OUT/probe.jsonl | cut -c1-100 || exit 1
for w in 2 4 8; do
  GCSB_CRC_SLOT_WAVES=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_w$w -o b -- \
    python bench.py --steps 10 --warmup 2 --side-steps 0 > $OUT/prof_w$w.log 2>&1 || { tail -10 $OUT/prof_w$w.log; exit 1; }
  echo "waves $w"; grep -h slot_kernel $(find $OUT/prof_w$w -name '*kernel_stats.csv') | cut -d, -f2-7
done
echo done
