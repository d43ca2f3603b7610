#!/bin/bash
# CRC32C kernel throughput + rocprofv3 kernel stats and PMC counters.
# Each GPU step has its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
timeout -k 10 300 python scripts/crc_kernel_bench.py > $OUT/crc_bench.log 2>&1 || exit $?
cat $OUT/crc_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_crc -o crc -- \
  python scripts/crc_kernel_bench.py > $OUT/prof_crc.log 2>&1 || exit $?
CRC_ITERS=3 timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES \
  SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_crc -o crc -- python scripts/crc_kernel_bench.py \
  > $OUT/pmc_crc.log 2>&1 || exit $?
CRC_ITERS=3 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_crc2 -o crc -- \
  python scripts/crc_kernel_bench.py > $OUT/pmc_crc2.log 2>&1 || exit $?
echo done
