#!/bin/bash
# A/B on one box: pinned ring page size (hipHostMalloc 4 KiB pages vs THP +
# hipHostRegister) x submitter-thread placement (inherits the receiving
# thread's SMT pair vs a core of its own), one gRPC stream per 256 MiB read.
# Also the raw loopback stream into a ring of default / huge / small pages.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/ring_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
B=custom_go_client_benchmark_amd/bin/loopback_ceiling
{ cat /sys/kernel/mm/transparent_hugepage/enabled; cat /sys/kernel/mm/transparent_hugepage/defrag; } > $OUT/thp.txt 2>&1
cat $OUT/thp.txt
PAIR=$(timeout -k 5 120 python3 -c "
from custom_go_client_benchmark_amd.parallel import affinity
p = affinity.plan(0, 'pair'); print(p['client'][0], p['server'][0], p.get('aux'))") || exit 1
echo "pair plan: $PAIR" | tee $OUT/plan.txt
set -- $PAIR
for rep in 1 2; do
  for pg in 0 1 2; do
    echo "== ceiling ring-pages $pg"
    timeout -k 5 60 $B -mode tcp -reads 6 -ring-kib 16384 -ring-pages $pg -recv-cpu $1 -send-cpu $2 \
      | sed "s/^{/{\"ring_pages\": $pg, /" | tee -a $OUT/ceiling.jsonl || exit 1
  done
done
for rep in ${REPS:-1 2}; do
  for alloc in hip thp; do
    for sub in inherit aux; do
      GCSB_RING_ALLOC=$alloc timeout -k 10 180 python bench.py --steps 20 --warmup 3 --side-steps 0 \
        --submit-cpus $sub > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
      python - "$alloc" "$sub" <<'PY' | tee -a $OUT/ab.txt
import json, sys
line = [l for l in open("gpurun_out/ring_ab/bench.log") if l.startswith("{")][-1]
d = json.loads(line)
c = d["rank0_cpu"]
print(f"alloc={sys.argv[1]:4s} submit={sys.argv[2]:7s} MiB/s={d['value']:9.1f} p50={d['p50_ms']:.2f} "
      f"p99={d['p99_ms']:.2f} host_p50={d['host_landed_p50_ms']:.2f} cpu/GiB={c['process_cpu_s_per_gib']} "
      f"by_thread={c.get('cpu_s_per_gib_by_thread')}")
PY
    done
  done
done
echo done
