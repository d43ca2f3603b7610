#!/bin/bash
# Sliced-read extension A/B on one box: streams per read x piece size, the
# sliced block only (headline 1 step), interleaved reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/sliced_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "base::" "streams4:GCSB_STREAMS=4:" "streams16:GCSB_STREAMS=16:" "slot8x2::--sliced-slot-bytes 8MiB --sliced-slots 2" \
           "slot2x8::--sliced-slot-bytes 2MiB --sliced-slots 8" "async::--sliced-async-submit 1"; do
    label=${v%%:*}; rest=${v#*:}; envs=${rest%%:*}; extra=${rest#*:}
    env $envs timeout -k 10 180 python bench.py --steps 2 --warmup 1 --side-steps 20 $extra \
      > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
    python3 - "$label" "$OUT/bench.log" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
s = d["sliced"]
print(f"{sys.argv[1]:10s} MiB/s={s['mib_s']:9.1f} p50={s['p50_ms']:.2f} p99={s['p99_ms']:.2f} "
      f"host_p50={s['host_landed_p50_ms']:.2f} cpu/GiB={s.get('process_cpu_s_per_gib')} skew={s['slice_skew_ms']} "
      f"cpus={s.get('cpus_busy')} throttled={s.get('cgroup_nr_throttled')}")
PY
  done
done
echo done
