#!/bin/bash
# int8-MFMA tile CRC: correctness (GPU CRC tests with every batch on 4 KiB
# tiles and the MFMA tile kernel) and bulk throughput vs the LDS kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/crc_mfma}
mkdir -p $OUT
GCSB_CRC_MFMA=1 GCSB_CRC_TILE=4k timeout -k 10 300 python -u -m pytest tests/test_gpu_crc32c.py -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in 0 1; do
  GCSB_CRC_MFMA=$v CRC_ITERS=20 timeout -k 10 200 python scripts/crc_kernel_bench.py 2>/dev/null | grep '"bulk"' \
    | sed "s/^{/{\"mfma\": $v, /" | tee -a $OUT/bulk.jsonl || exit 1
done
GCSB_CRC_MFMA=1 timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o crc -- \
  python scripts/crc_kernel_bench.py > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
grep -h "mfma\|tiles_kernel\|fold" $(find $OUT/prof -name '*kernel_stats.csv') | cut -c1-200
echo done
