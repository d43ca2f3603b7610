#!/bin/bash
# Endpoint send path A/B on one loopback stream (no GPU): sendfile() from the
# memfd page cache (receiver's copy reads DRAM) vs send() from a 2 MiB
# buffer the sender just filled (the skb pages are written by a core of the
# same L3 domain, so the receiver's copy_to_user reads them from L3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-gpurun_out/sendpath}
mkdir -p "$OUT"
B=custom_go_client_benchmark_amd/bin/loopback_ceiling
PAIRS=$(timeout -k 5 120 python3 -c "
from custom_go_client_benchmark_amd.parallel import affinity
cpus = affinity.gpu_local_cpus(0)
groups = affinity.l3_groups(cpus)
out = []
for g in groups[:3]:
    f = affinity.core_first(g)
    if len(f) >= 2: out.append(f'{f[0]}:{f[1]}')
print(' '.join(out))") || exit 1
echo "pairs: $PAIRS"
for rep in 1 2 3; do
  for p in $PAIRS; do
    r=${p%%:*}; s=${p##*:}
    for zc in 1 0; do
      timeout -k 5 60 $B -mode tcp -reads 6 -ring-kib 16384 -ring-pages 1 -recv-cpu $r -send-cpu $s -zerocopy-send=$([ $zc = 1 ] && echo true || echo false) \
        | sed "s/^{/{\"zc\": $zc, \"pair\": \"$p\", /" | tee -a $OUT/runs.jsonl || exit 1
    done
  done
done
python3 - $OUT/runs.jsonl <<'PY' | tee $OUT/summary.txt
import json, sys, statistics, collections
v = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); v[d["zc"]].append(d["tcp_gbps"])
for k, xs in sorted(v.items()):
    print("zerocopy_send=%d n=%d median %.2f GB/s min %.2f max %.2f" % (k, len(xs), statistics.median(xs), min(xs), max(xs)))
PY
