#!/bin/bash
# Interleaved A/B of bench variants on one box (identical runs vary up to 2x
# between and within boxes, so variants alternate within each rep).
#   VARIANTS="A=ENV1=x,ENV2=y;B=ENV1=z|--rcvbuf 32MiB"  REPS=4  ARGS="--side-steps 0"
# Each variant is "<label>=<comma-separated env assignments>[|extra bench args]"
# (either part may be empty).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/env_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${ARGS:---steps 20 --warmup 3 --side-steps 0}
IFS=';' read -ra VS <<< "$VARIANTS"
for rep in $(seq 1 ${REPS:-3}); do
  for v in "${VS[@]}"; do
    label=${v%%=*}; rest=${v#*=}; envs=${rest%%|*}; extra=""
    [[ "$rest" == *"|"* ]] && extra=${rest#*|}
    IFS=',' read -ra EA <<< "$envs"
    env "${EA[@]}" timeout -k 10 180 python bench.py $ARGS $extra > $OUT/bench.log 2>&1 \
      || { tail -20 $OUT/bench.log; exit 1; }
    grep -h '^{' $OUT/bench.log | sed "s/^{/{\"variant\": \"$label\", /" >> $OUT/runs.jsonl
    python3 - "$label" "$OUT/bench.log" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
c = d.get("rank0_cpu") or {}
print(f"{sys.argv[1]:12s} MiB/s={d['value']:9.1f} p50={d['p50_ms']:.2f} p99={d['p99_ms']:.2f} "
      f"host_p50={d.get('host_landed_p50_ms', 0):.2f} cpu/GiB={c.get('process_cpu_s_per_gib')} "
      f"by_thread={c.get('cpu_s_per_gib_by_thread')} placement={d.get('placement')}")
PY
  done
done
python3 - "$OUT/runs.jsonl" <<'PY' | tee -a $OUT/ab.txt
import json, statistics, sys
from collections import defaultdict
v = defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); v[d["variant"]].append(d["value"])
for k, xs in v.items():
    print(f"summary {k:12s} n={len(xs)} median={statistics.median(xs):9.1f} min={min(xs):9.1f} max={max(xs):9.1f}")
PY
echo done
