#!/bin/bash
# Multiplexed gRPC blocks A/B: the connection's reader wakes each finished
# read's worker itself (0) vs a notifier thread polling every N us does
# (core/waker.h), interleaved, order alternating per pair.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/notify
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
PAIRS=${PAIRS:-5}
US=${US:-20}
for i in $(seq 1 "$PAIRS"); do
  order="0 $US"
  [ $((i % 2)) -eq 0 ] && order="$US 0"
  for n in $order; do
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --blocks ref_default,list_read --mux-notify-us "$n" \
      --json-out "$OUT/n${n}_$i.json" --diag-out "$OUT/diag_n${n}_$i.json" > "$OUT/n${n}_$i.out" 2> "$OUT/n${n}_$i.err"
    rc=$?
    echo "pair $i notify_us=$n rc=$rc $(python3 -c "
import json
d=json.load(open('$OUT/n${n}_$i.json'))
print(' '.join(f\"{k}={d[k]['mib_s']:.0f}/{d[k].get('recv_cpu_s_per_gib')}\" for k in ('ref_default_grpc','list_read_grpc') if k in d))" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
exit 0
