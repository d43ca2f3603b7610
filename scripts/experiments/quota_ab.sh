#!/bin/bash
# GPU box session: quota-aware placement A/B.  Small-object configs at the
# reference's default concurrency (48 workers, main.go:36) and at 8, with
# threads unpinned (-affinity none) vs held to the CPU quota's worth of cores
# (-affinity quota, the discard-sink default), plus the headline bench
# (share placement, now trimmed to the quota) three times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/quota}
mkdir -p "$OUT"
export TMPDIR=/tmp
MIB=1048576
one() {  # one <name> <args...>
  local name=$1; shift
  timeout -k 10 200 ./gcsbench -start-fake-server -latency-file /dev/null -summary-json $OUT/$name.json "$@" \
    > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
  python -c "
import json; d = json.load(open('$OUT/$name.json'))
print('$name'.ljust(30), {k: round(d[k], 3) if isinstance(d[k], float) else d[k] for k in
      ('mib_per_s', 'p50_ms', 'p99_ms', 'max_ms', 'cgroup_nr_periods', 'cgroup_nr_throttled', 'cgroup_throttled_ms',
       'cpu_s_by_group') if k in d})
" | tee -a $OUT/quota.txt
}
for rep in 1 2; do
  for p in http grpc; do
    for w in 48 8; do
      for aff in quota none; do
        one c1_${p}_w${w}_${aff}_$rep -client-protocol $p -worker $w -read-call-per-worker 400 \
          -fake-object-size $MIB -affinity $aff
      done
    done
  done
done
for p in http grpc; do
  one c3_${p}_list1000_hbm -workload list-read -client-protocol $p -sink gpu -worker 8 -read-call-per-worker 3 \
    -fake-objects 1000 -fake-object-size $MIB
done
for rep in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 3 --side-steps 20 > $OUT/bench_$rep.log 2>&1 \
    || { tail -20 $OUT/bench_$rep.log; exit 1; }
  grep -h '^{' $OUT/bench_$rep.log | tee -a $OUT/bench_runs.jsonl | cut -c1-200
done
echo done
