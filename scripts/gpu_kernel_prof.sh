#!/bin/bash
# CRC32C kernel throughput + rocprofv3 kernel stats and PMC counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/crc_kernel_bench.py > gpurun_out/crc_bench.log 2>&1 || exit $?
cat gpurun_out/crc_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_crc -o crc -- \
  python scripts/crc_kernel_bench.py > gpurun_out/prof_crc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/pmc_crc -o crc -- python scripts/crc_kernel_bench.py > gpurun_out/pmc_crc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_crc2 -o crc -- \
  python scripts/crc_kernel_bench.py > gpurun_out/pmc_crc2.log 2>&1 || exit $?
echo done
