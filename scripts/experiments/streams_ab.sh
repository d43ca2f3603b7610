#!/bin/bash
# GPU box session: full GPU tests, then A/B of the per-device stream pool size
# (GCSB_STREAMS) on the headline bench (one stream per read) and the sliced
# extension, then the 48-worker small-object configs with the container's CFS
# throttling counters (the reference's default concurrency, main.go:36).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/streams}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
summ() {  # summ <label> <json file>
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
s = d.get("sliced", {})
print(f"{sys.argv[1]:24s} single={d['value']:9.1f} p50={d['p50_ms']:.2f} p99={d['p99_ms']:.2f} "
      f"host_p50={d.get('host_landed_p50_ms', 0):.2f} | sliced={s.get('mib_s', 0):9.1f} p50={s.get('p50_ms', 0):.2f} "
      f"p99={s.get('p99_ms', 0):.2f} host_p50={s.get('host_landed_p50_ms', 0):.2f}")
PY
}
for n in 0 4 8 0 4 8 0 4 8; do
  GCSB_STREAMS=$n timeout -k 10 240 python bench.py --steps 20 --warmup 3 --side-steps 20 \
    > $OUT/bench_s$n.log 2>&1 || { tail -20 $OUT/bench_s$n.log; exit 1; }
  summ "streams=$n" $OUT/bench_s$n.log | tee -a $OUT/ab.txt
  grep -h '^{' $OUT/bench_s$n.log >> $OUT/ab_runs.jsonl
done
MIB=1048576
for p in http grpc; do
  for w in 8 48; do
    timeout -k 10 200 ./gcsbench -start-fake-server -latency-file /dev/null -summary-json $OUT/c1_${p}_w$w.json \
      -client-protocol $p -worker $w -read-call-per-worker 200 -fake-object-size $MIB > $OUT/c1_${p}_w$w.log 2>&1 \
      || { tail -5 $OUT/c1_${p}_w$w.log; exit 1; }
    python -c "
import json; d = json.load(open('$OUT/c1_${p}_w$w.json'))
print('c1 $p w$w', {k: round(d[k], 3) if isinstance(d[k], float) else d[k] for k in
      ('mib_per_s', 'p50_ms', 'p99_ms', 'max_ms', 'elapsed_s', 'cgroup_nr_periods', 'cgroup_nr_throttled', 'cgroup_throttled_ms', 'cpu_s_by_group') if k in d})
" | tee -a $OUT/w48.txt
  done
done
echo done
