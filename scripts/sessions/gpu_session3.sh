#!/bin/bash
# GPU session: the standard check (tests, smoke, bench, rocprof) plus the
# config-5 upload runs (HBM -> pinned -> resumable / WriteObject).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh || exit $?
OUT=gpurun_out/configs
mkdir -p "$OUT"
MIB=1048576
for p in grpc http; do
  name=c5_${p}_write64m
  echo "=== $name ($(date +%T))"
  timeout -k 10 300 ./gcsbench -start-fake-server -summary-json "$OUT/$name.json" -workload write \
    -client-protocol $p -sink gpu -worker 1 -write-objects 20 -fake-retain-uploads=false \
    -write-size $((64 * MIB)) -fake-objects 1 -fake-object-size $MIB > "$OUT/$name.log" 2>&1
  rc=$?; tail -n 2 "$OUT/$name.log"
  [ $rc -ne 0 ] && { echo "fatal rc=$rc in $name"; exit $rc; }
done
echo "session done"
