#!/bin/bash
# bench.py over protocol x slices x placement on one GPU (each step time-limited).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/slices}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for p in grpc http; do
  for aff in same split; do
    for sl in 1 2 4 8; do
      name=${p}_${aff}_s${sl}
      timeout -k 10 120 python bench.py --protocol $p --affinity $aff --slices $sl --steps 15 --warmup 2 \
        --json-out "$OUT/$name.json" > "$OUT/$name.log" 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -3 "$OUT/$name.log"; [ $rc -ne 1 ] && exit $rc; fi
      python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], d['p50_ms'], d['p99_ms'])"
    done
  done
done
