#!/bin/bash
# GPU box session: CPU placement of the client / endpoint threads for the
# headline read (one gRPC stream per 256 MiB read into HBM), interleaved reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/placement}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 python -c "
from custom_go_client_benchmark_amd.parallel import affinity as a
for m in ('pair', 'same', 'split', 'share'): print(m, a.plan(0, m))" > $OUT/plans.txt 2>&1 || exit 1
cut -c1-200 $OUT/plans.txt
for rep in 1 2 3; do
  for aff in share pair same split none; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 3 --side-steps 0 --affinity $aff > $OUT/b.log 2>&1 \
      || { tail -20 $OUT/b.log; exit 1; }
    python - $aff <<'PY' | tee -a $OUT/placement.txt
import json, sys
d = json.loads([l for l in open("gpurun_out/placement/b.log") if l.startswith("{")][-1])
c = d["rank0_cpu"]
print(f"{sys.argv[1]:6s} MiB/s={d['value']:9.1f} p50={d['p50_ms']:.2f} p99={d['p99_ms']:.2f} "
      f"cpu/GiB={c['process_cpu_s_per_gib']} busy={c['cpus_busy']} {c.get('cpu_s_per_gib_by_thread')}")
PY
  done
done
echo done
