#!/bin/bash
# Headline ring A/B: cached THP ring (off) vs write-combined pinned ring (on),
# interleaved, each run the paired headline only (baseline + nodma arms
# between its chunks).  Every run has its own time limit; a crash ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/ringwc
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
PAIRS=${PAIRS:-6}
for i in $(seq 1 "$PAIRS"); do
  for wc in off on; do
    [ $((i % 2)) -eq 0 ] && wc=$([ "$wc" = off ] && echo on || echo off)
    timeout -k 10 240 python bench.py --steps 20 --warmup 3 --blocks cpu_baseline --ring-wc "$wc" \
      --json-out "$OUT/wc_${wc}_$i.json" --diag-out "$OUT/diag_${wc}_$i.json" > "$OUT/wc_${wc}_$i.out" 2> "$OUT/wc_${wc}_$i.err"
    rc=$?
    echo "pair $i wc=$wc rc=$rc $(python3 -c "import json,sys; d=json.load(open('$OUT/wc_${wc}_$i.json')); print(d['value'], d.get('vs_baseline_paired'), d.get('headline_vs_nodma'))" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
