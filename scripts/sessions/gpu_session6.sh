#!/bin/bash
# Final checks for the round: the standard GPU check (tests, smoke, default
# bench, rocprof kernel stats) and config-5 uploads with the new defaults.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_check.sh || exit $?
OUT=gpurun_out/s6
mkdir -p "$OUT"
MIB=1048576
for p in grpc http; do
  for sl in 1 8; do
    name=c5_${p}_s${sl}
    timeout -k 10 300 ./gcsbench -start-fake-server -summary-json "$OUT/$name.json" -workload write -slices $sl \
      -client-protocol $p -sink gpu -worker 1 -write-objects 20 -fake-retain-uploads=false \
      -write-size $((64 * MIB)) -fake-objects 1 -fake-object-size $MIB > "$OUT/$name.log" 2>&1
    rc=$?
    echo "$name rc=$rc $(grep -o 'p50 [0-9.]* ms, p99 [0-9.]* ms, [0-9.]* MiB/s' $OUT/$name.log | head -1)"
    [ $rc -ne 0 ] && { tail -5 "$OUT/$name.log"; exit $rc; }
  done
done
echo "session done"
