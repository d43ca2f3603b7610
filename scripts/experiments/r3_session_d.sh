# Headline-phase diagnosis: three full bench runs back to back (host vmstat,
# faults and context switches per block), then the GPU test suite, smoke and
# the 8-rank gloo rehearsal.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_d; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_$i.log 2>&1
  echo "bench i=$i rc=$?"
done
cat /proc/sys/kernel/numa_balancing /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > $O/host_mm.txt 2>&1
bash scripts/experiments/r3_session_c.sh
