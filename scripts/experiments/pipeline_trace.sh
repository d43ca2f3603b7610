#!/bin/bash
# Timeline of the one-stream read pipeline: rocprofv3 kernel + memory-copy +
# marker (roctx) traces of a short single-stream bench, and five plain bench
# runs for the run-to-run distribution at this HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pipe}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --stats --output-format csv \
  -d $OUT/trace -o b -- python3 bench.py --steps 5 --warmup 1 --side-steps 0 > $OUT/trace.log 2>&1 \
  || { tail -20 $OUT/trace.log; exit 1; }
ls $OUT/trace
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --side-steps 0 > $OUT/b$i.log 2>&1 || { tail -20 $OUT/b$i.log; exit 1; }
  grep -h '^{' $OUT/b$i.log >> $OUT/runs.jsonl
done
python3 - <<'PY'
import json
for l in open("gpurun_out/pipe/runs.jsonl"):
    d = json.loads(l)
    print(d["value"], d["p50_ms"], d["p99_ms"], d["ttfb_p50_ms"], d["host_landed_p50_ms"], d["rank0_cpu"]["cpu_s_per_gib_by_thread"])
PY
echo done
