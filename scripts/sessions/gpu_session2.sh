#!/bin/bash
# GPU box: environment facts (cgroup CPU quota), 2-rank gloo rehearsal of
# bench.py on one GPU, and a marker+kernel+copy trace of the headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s2
mkdir -p $OUT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
{
  echo "nproc: $(nproc)"; python -c "import os;print('affinity', len(os.sched_getaffinity(0)))"
  cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cpu.max"
  cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null || true
  cat /proc/self/cgroup
  grep -c processor /proc/cpuinfo; grep -m1 "model name" /proc/cpuinfo
} > $OUT/env.txt 2>&1
cat $OUT/env.txt
timeout -k 10 600 make -j16 all > $OUT/build.log 2>&1 || exit 1
GCSB_DIST_BACKEND=gloo timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 2 > $OUT/rehearsal2.log 2>&1
rc=$?; echo "rehearsal rc=$rc"; grep metric $OUT/rehearsal2.log | head -c 1500; echo
[ $rc -ne 0 ] && { tail -20 $OUT/rehearsal2.log; exit $rc; }
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --memory-copy-trace --stats --output-format csv \
  -d $OUT/prof -o bench -- python bench.py --steps 8 --warmup 2 > $OUT/prof.log 2>&1
echo "rocprof rc=$?"; ls $OUT/prof
