#!/bin/bash
# Sliced-read tuning on one GPU: slices x placement x ring geometry (bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/slices2}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for p in grpc http; do
  for aff in split numa; do
    for sl in 4 8; do
      for geo in 8MiB:4 4MiB:4 2MiB:8; do
        sb=${geo%:*}; ns=${geo#*:}
        name=${p}_${aff}_s${sl}_${sb}x${ns}
        timeout -k 10 120 python bench.py --protocol $p --affinity $aff --slices $sl --slot-bytes $sb --slots $ns \
          --steps 15 --warmup 2 --single-stream-steps 0 --json-out "$OUT/$name.json" > "$OUT/$name.log" 2>&1
        rc=$?
        if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -3 "$OUT/$name.log"; [ $rc -ne 1 ] && exit $rc; fi
        python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], d['p50_ms'], d['p99_ms'])"
      done
    done
  done
done
