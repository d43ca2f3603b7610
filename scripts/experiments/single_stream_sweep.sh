#!/bin/bash
# Single-stream ceiling on the GPU box: the raw loopback TCP copy bound
# (csrc/tools/loopback_ceiling.cc, no GPU) next to the bench's single-stream
# gRPC read into HBM under a few ring geometries / submit modes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/single}
mkdir -p "$OUT"
export TMPDIR=/tmp
B=custom_go_client_benchmark_amd/bin/loopback_ceiling
PLAN=$(timeout -k 5 120 python -c "
from custom_go_client_benchmark_amd.parallel import affinity
p = affinity.plan(0, 'share'); print(' '.join(map(str, p['client'])))") || exit 1
echo "share plan cpus: $PLAN" | tee $OUT/plan.txt
set -- $PLAN
C0=$1; C1=$2; C8=${9:-$2}
for args in "-ring-kib 16384" "-ring-kib 4096" "-ring-kib 1024 -recv-kib 1024" "-ring-kib 16384 -recv-kib 256" \
            "-ring-kib 16384 -recv-cpu $C0 -send-cpu $C1" "-ring-kib 4096 -recv-cpu $C0 -send-cpu $C1" \
            "-ring-kib 16384 -recv-cpu $C0 -send-cpu $C8" "-ring-kib 16384 -rcvbuf-kib 32768" \
            "-ring-kib 16384 -zerocopy-send=false"; do
  echo "== $args"
  timeout -k 5 120 $B -reads 10 $args | tee -a $OUT/ceiling.jsonl || exit 1
done
for cfg in "--slot-bytes 4MiB --slots 4" "--slot-bytes 1MiB --slots 8" "--slot-bytes 2MiB --slots 8" \
           "--slot-bytes 8MiB --slots 4" "--slot-bytes 16MiB --slots 2"; do
  for asy in 0 1; do
    echo "== bench $cfg async=$asy"
    GCSB_ASYNC_SUBMIT=$asy timeout -k 10 180 python bench.py --steps 20 --warmup 3 --side-steps 0 $cfg \
      > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
    python - "$cfg" "$asy" <<'PY' | tee -a $OUT/bench_sweep.txt
import json, sys
line = [l for l in open("gpurun_out/single/bench.log") if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[1]:32s} async={sys.argv[2]} MiB/s={d['value']:9.1f} p50={d['p50_ms']:.2f} p99={d['p99_ms']:.2f} "
      f"host_p50={d['host_landed_p50_ms']:.2f} cpu/GiB={d['rank0_cpu']['process_cpu_s_per_gib']} "
      f"by_thread={d['rank0_cpu'].get('cpu_s_per_gib_by_thread')}")
PY
  done
done
echo done
