#!/bin/bash
# bench.py defaults and neighbours (share placement) on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/slices3}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  name=$1; shift
  timeout -k 10 120 python bench.py "$@" --json-out "$OUT/$name.json" > "$OUT/$name.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -3 "$OUT/$name.log"; [ $rc -ne 1 ] && exit $rc; return; fi
  python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], d['p50_ms'], d['p99_ms'], d.get('single_stream_mib_s'))"
}
run default --steps 20 --warmup 3
run default_http --protocol http --steps 20 --warmup 3
for sl in 6 8 12 16; do
  for geo in 4MiB:4 2MiB:8 2MiB:4; do
    sb=${geo%:*}; ns=${geo#*:}
    run grpc_s${sl}_${sb}x${ns} --slices $sl --slot-bytes $sb --slots $ns --steps 15 --warmup 2 --single-stream-steps 0
  done
done
run default_again --steps 20 --warmup 3
