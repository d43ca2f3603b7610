#!/bin/bash
# Round-2 session C on one MI355X box: the BASELINE configs after the
# host-memory placement fix (endpoint memfd on the GPU's NUMA node), the slot
# CRC kernel and the HTTP/2 media path.  Every GPU step has its own limit;
# a crash / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/r2c}
mkdir -p "$OUT"
export TMPDIR=/tmp
MIB=1048576

run() {  # run <name> <timeout> <gcsbench args...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" ./gcsbench -start-fake-server -latency-file /dev/null \
    -summary-json "$OUT/$name.json" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then tail -n 5 "$OUT/$name.log"; echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
  python3 - "$name" "$OUT/$name.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
keys = ("mib_per_s", "p50_ms", "p99_ms", "verified", "reads", "errors", "cgroup_nr_throttled")
print(f"{sys.argv[1]:28s}", {k: (round(d[k], 3) if isinstance(d[k], float) else d[k]) for k in keys if k in d})
PY
}

for p in http http2 grpc; do
  run c1_${p}_w1 200 -client-protocol $p -worker 1 -read-call-per-worker 2000 -fake-object-size $MIB
  run c1_${p}_w48 200 -client-protocol $p -worker 48 -read-call-per-worker 100 -fake-object-size $MIB
done
for p in http http2 grpc; do
  run c3_${p}_hbm 200 -workload list-read -client-protocol $p -sink gpu -worker 8 -read-call-per-worker 3 \
    -fake-objects 1000 -fake-object-size $MIB
done
run c3_grpc_pool8_hbm 200 -workload list-read -client-protocol grpc -grpc-conn-pool-size 8 -sink gpu -worker 8 \
  -read-call-per-worker 3 -fake-objects 1000 -fake-object-size $MIB
for p in http2 grpc http; do
  run c2_${p}_256m_hbm 200 -client-protocol $p -sink gpu -worker 1 -read-call-per-worker 20 \
    -fake-object-size $((256 * MIB))
done
for rep in 1 2; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 3 > $OUT/bench_$rep.log 2>&1 || { tail -20 $OUT/bench_$rep.log; exit 1; }
  grep -h '^{' $OUT/bench_$rep.log >> $OUT/bench_runs.jsonl
  python3 -c "
import json,sys
d=json.loads(open('$OUT/bench_runs.jsonl').read().splitlines()[-1])
print('bench', d['value'], d['p50_ms'], d['p99_ms'], d['numa'], 'compare', d['compare']['mib_s'], 'sliced', d['sliced']['mib_s'], d['sliced']['p99_ms'], 'write', d['write']['mib_s'], d['write']['p50_ms'])"
done
GCSB_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 4 --steps 10 --warmup 2 --side-steps 0 \
  > $OUT/rehearsal4.log 2>&1 || { tail -30 $OUT/rehearsal4.log; exit 1; }
grep -h '^{' $OUT/rehearsal4.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('rehearsal4', d['value'], 'per_rank', d['per_rank_mib_s'], 'p50', d['p50_ms'], 'p99', d['p99_ms'], 'n_gpus', d['n_gpus'], 'ranks', d['ranks'])"
echo done
