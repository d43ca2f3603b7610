#!/bin/bash
# Multi-rank rehearsal of the driver's scaling run on a 1-GPU box (2 and 4
# ranks sharing the GPU, control plane over gloo since RCCL rejects two ranks
# on one device), with the piece-mode default; plus piece sizes 6/12 MiB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/s7
mkdir -p "$OUT"
for n in 2 4; do
  GCSB_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 10 --warmup 2 \
    --single-stream-steps 0 > $OUT/rehearsal_${n}rank.log 2>&1 || { echo "rehearsal $n rc=$?"; tail -20 $OUT/rehearsal_${n}rank.log; exit 1; }
  grep '^{' $OUT/rehearsal_${n}rank.log | tail -1 | cut -c1-400
done
for pb in 6MiB 12MiB 8MiB; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --single-stream-steps 0 --piece-bytes $pb \
    --json-out $OUT/bench_p$pb.json > $OUT/bench_p$pb.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_p$pb.json'));print('piece=$pb', d['value'], d['p50_ms'], d['p99_ms'], d['slice_skew_ms'])"
done
echo "session done"
