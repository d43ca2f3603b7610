#!/bin/bash
# Config 3 (1000 x 1 MiB list + read -> HBM, 8 workers) under hand-off variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/small}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  name=$1; shift
  env "$@" timeout -k 10 120 ./gcsbench -start-fake-server -workload list-read -client-protocol http -sink gpu \
    -worker 8 -read-call-per-worker 3 -fake-objects 1000 -fake-object-size 1048576 -affinity numa \
    -latency-file "$OUT/$name.lat" -summary-json "$OUT/$name.json" $EXTRA > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -3 "$OUT/$name.log"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', round(d['p50_ms'],3), round(d['p99_ms'],3), round(d['host_p50_ms'],3), round(d['mib_per_s']))"
}
for r in 1 2; do
  EXTRA="" run base_r$r GCSB_X=0
  EXTRA="" run spin_r$r GCSB_EVENT_SPIN=1
  EXTRA="-ring-slot-bytes 262144 -ring-slots 8" run slot256k_r$r GCSB_X=0
  EXTRA="-ring-slot-bytes 262144 -ring-slots 8" run slot256k_spin_r$r GCSB_EVENT_SPIN=1
  EXTRA="" run async_r$r GCSB_ASYNC_SUBMIT=1
done
