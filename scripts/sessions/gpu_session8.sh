#!/bin/bash
# (1) piece size 8 vs 12 MiB, interleaved x3 (run-to-run spread is ~10%);
# (2) WriteObject upload pinned vs unpinned with per-thread CPU accounting.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/s8
mkdir -p "$OUT"
MIB=1048576
for rep in 1 2 3; do
  for pb in 8MiB 12MiB; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --single-stream-steps 0 --piece-bytes $pb \
      --json-out $OUT/bench_p${pb}_r$rep.json > $OUT/bench_p${pb}_r$rep.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_p${pb}_r$rep.json'));print('piece=$pb rep=$rep', d['value'], d['p50_ms'], d['p99_ms'], d['slice_skew_ms'])"
  done
done
for aff in same none; do
  name=c5_grpc_$aff
  timeout -k 10 300 ./gcsbench -start-fake-server -summary-json "$OUT/$name.json" -workload write -affinity $aff \
    -client-protocol grpc -sink gpu -worker 1 -write-objects 20 -fake-retain-uploads=false \
    -write-size $((64 * MIB)) -fake-objects 1 -fake-object-size $MIB > "$OUT/$name.log" 2>&1 || { echo "$name failed"; exit 1; }
  python -c "
import json;d=json.load(open('$OUT/$name.json'))
def f(x):
    if isinstance(x,dict):
        for k,v in x.items():
            if k in ('p50_ms','cpu_s_per_gib_by_thread'): print('$name',k,v)
            f(v)
f(d)"
done
echo "session done"
