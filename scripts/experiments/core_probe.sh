#!/bin/bash
# Which cores of a shared GPU host are fast for one loopback stream?
# Prints topology, the cgroup's CPU limits, per-CPU busy fraction from
# /proc/stat over 2 s, per-core clock, then runs loopback_ceiling (no GPU)
# pinned to receiver/sender core pairs spread over the GPU's NUMA node.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/cores}
mkdir -p "$OUT"
export TMPDIR=/tmp
B=custom_go_client_benchmark_amd/bin/loopback_ceiling
{
  echo "nproc=$(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null
  lscpu | head -30
} > $OUT/topo.txt 2>&1
timeout -k 5 60 python3 - <<'PY' > $OUT/busy.txt 2>&1
import time
def snap():
    out = {}
    for l in open("/proc/stat"):
        if l.startswith("cpu") and l[3].isdigit():
            p = l.split(); c = int(p[0][3:]); v = list(map(int, p[1:]))
            out[c] = (sum(v), v[3] + v[4])
    return out
a = snap(); time.sleep(2.0); b = snap()
busy = {c: 1.0 - (b[c][1] - a[c][1]) / max(1, b[c][0] - a[c][0]) for c in b}
def freq(c):
    try: return int(open(f"/sys/devices/system/cpu/cpu{c}/cpufreq/scaling_cur_freq").read()) // 1000
    except OSError: return -1
print("cpus", len(busy), "mean_busy", round(sum(busy.values()) / len(busy), 3))
for c in sorted(busy):
    print(c, round(busy[c], 3), freq(c))
PY
head -3 $OUT/busy.txt
PAIRS=$(timeout -k 5 120 python3 -c "
from custom_go_client_benchmark_amd.parallel import affinity
cpus = affinity.gpu_local_cpus(0)
groups = affinity.l3_groups(cpus)
out = []
for g in groups:
    f = affinity.core_first(g)
    if len(f) >= 4: out.append(f'{f[0]}:{f[1]}'); out.append(f'{f[2]}:{f[3]}')
print(' '.join(out))") || exit 1
echo "pairs: $PAIRS" | tee $OUT/pairs.txt
for p in $PAIRS; do
  r=${p%%:*}; s=${p##*:}
  echo "== recv $r send $s"
  timeout -k 5 60 $B -reads 4 -ring-kib 16384 -recv-cpu $r -send-cpu $s | tee -a $OUT/pairs.jsonl || exit 1
done
echo "== unpinned x3"
for i in 1 2 3; do timeout -k 5 60 $B -reads 4 -ring-kib 16384 | tee -a $OUT/unpinned.jsonl || exit 1; done
echo done
