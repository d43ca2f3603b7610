#!/bin/bash
# Generic interleaved A/B of bench.py arguments, order alternating per pair.
#   A="--mux-send shared" B="--mux-send isolate" COMMON="--blocks ref_default,list_read" \
#   KEYS="ref_default_grpc list_read_grpc" NAME=muxsend bash scripts/experiments/bench_ab.sh
# Every run has its own time limit; a failing run ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
NAME=${NAME:-ab}
OUT=gpurun_out/$NAME
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
PAIRS=${PAIRS:-5}
KEYS=${KEYS:-}
for i in $(seq 1 "$PAIRS"); do
  order="A B"
  [ $((i % 2)) -eq 0 ] && order="B A"
  for arm in $order; do
    if [ "$arm" = A ]; then args=${A:-}; else args=${B:-}; fi
    # shellcheck disable=SC2086
    timeout -k 10 ${RUN_TIMEOUT:-300} python bench.py --steps ${STEPS:-5} --warmup ${WARMUP:-2} ${COMMON:-} $args \
      --json-out "$OUT/${arm}_$i.json" --diag-out "$OUT/diag_${arm}_$i.json" > "$OUT/${arm}_$i.out" 2> "$OUT/${arm}_$i.err"
    rc=$?
    echo "pair $i arm=$arm rc=$rc $(KEYS="$KEYS" python3 -c "
import json, os
d = json.load(open('$OUT/${arm}_$i.json'))
ks = os.environ['KEYS'].split()
parts = [f\"head={d['value']:.0f} paired={d.get('vs_baseline_paired')} nodma={d.get('headline_vs_nodma')}\"]
parts += [f\"{k}={d[k].get('mib_s', 0):.0f}/{d[k].get('recv_cpu_s_per_gib')}\" for k in ks if isinstance(d.get(k), dict)]
print(' '.join(parts))" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
exit 0
