#!/bin/bash
# Upload-path analysis: config-5 WriteObject vs resumable HTTP under different
# CPU placements, with per-thread CPU accounting in each summary; plus the
# headline bench (slice_skew_ms = sliced-read load balance).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/s4
mkdir -p "$OUT"
MIB=1048576
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
for aff in same split numa none; do
  for p in grpc http; do
    name=c5_${p}_${aff}
    timeout -k 10 300 ./gcsbench -start-fake-server -summary-json "$OUT/$name.json" -workload write -affinity $aff \
      -client-protocol $p -sink gpu -worker 1 -write-objects 20 -fake-retain-uploads=false \
      -write-size $((64 * MIB)) -fake-objects 1 -fake-object-size $MIB > "$OUT/$name.log" 2>&1
    rc=$?
    echo "$name rc=$rc $(grep -o 'p50 [0-9.]* ms' $OUT/$name.log | head -1)"
    [ $rc -ne 0 ] && { tail -5 "$OUT/$name.log"; exit $rc; }
  done
done
echo "session done"
