#!/bin/bash
# Does reading each slot one or two slots LATER (lines out of the writer's
# private L2, still in the L3) remove what the copy engine's read costs the
# writing core?  ring_dma_probe with small rings and lag 0 / 1 / 2, tcp and
# rep writers, idle vs sdma, placement of the bench headline (pair).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/dmalag
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
read -r W S X < <(python3 -c "
import sys; sys.path.insert(0, '.')
from custom_go_client_benchmark_amd.parallel import affinity as a
p = a.plan(0, 'pair')
print(p['client'][0], (p.get('aux') or p['server'])[0], p['server'][0])")
echo "writer=$W submitter=$S sender=$X"
P=custom_go_client_benchmark_amd/bin/ring_dma_probe
V=tcp/idle,tcp/sdma,rep/idle,rep/sdma
for geo in "4 0" "4 1" "4 2" "8 2" "8 4"; do
  set -- $geo
  timeout -k 10 120 "$P" slots=$1 slot=1048576 total=2147483648 reps=5 writer=$W submitter=$S sender=$X lag=$2 \
    variants=$V > "$OUT/s$1_lag$2.jsonl" 2> "$OUT/s$1_lag$2.err" || { echo "slots=$1 lag=$2 rc=$?"; exit 1; }
  echo "slots=$1 lag=$2"
  python3 scripts/experiments/dmaprobe_summary.py "$OUT/s$1_lag$2.jsonl"
done
