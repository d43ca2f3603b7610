#!/bin/bash
# GPU box session: GPU tests, config 3 (1000 x 1 MiB list + read into HBM),
# the default bench twice, and a 4-rank shared-GPU rehearsal (gloo control
# plane, 4 ranks on the box's one GPU) next to N=1 for the per-rank rate.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/r2a}
mkdir -p "$OUT"
export TMPDIR=/tmp
MIB=1048576
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for p in grpc http; do
  timeout -k 10 200 ./gcsbench -start-fake-server -latency-file /dev/null -summary-json $OUT/c3_$p.json \
    -workload list-read -client-protocol $p -sink gpu -worker 8 -read-call-per-worker 3 -fake-objects 1000 \
    -fake-object-size $MIB > $OUT/c3_$p.log 2>&1 || { tail -5 $OUT/c3_$p.log; exit 1; }
  python -c "
import json; d = json.load(open('$OUT/c3_$p.json'))
print('c3 $p', {k: round(d[k], 3) if isinstance(d[k], float) else d[k] for k in
      ('mib_per_s', 'p50_ms', 'p99_ms', 'verified', 'reads', 'cgroup_nr_throttled', 'cpu_s_by_group') if k in d})"
done
for rep in 1 2; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 3 > $OUT/bench_$rep.log 2>&1 || { tail -20 $OUT/bench_$rep.log; exit 1; }
  grep -h '^{' $OUT/bench_$rep.log | tee -a $OUT/bench_runs.jsonl | cut -c1-160
done
timeout -k 10 240 python bench.py --steps 10 --warmup 2 --side-steps 0 > $OUT/n1.log 2>&1 || { tail -20 $OUT/n1.log; exit 1; }
grep -h '^{' $OUT/n1.log | cut -c1-160
GCSB_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 4 --steps 10 --warmup 2 --side-steps 0 \
  > $OUT/rehearsal4.log 2>&1 || { tail -30 $OUT/rehearsal4.log; exit 1; }
grep -h '^{' $OUT/rehearsal4.log | python -c "
import json, sys
d = json.loads(sys.stdin.read())
print('rehearsal4', d['value'], 'per_rank', d['per_rank_mib_s'], 'p50', d['p50_ms'], 'p99', d['p99_ms'], 'n_gpus', d['n_gpus'], 'ranks', d['ranks'])"
echo done
