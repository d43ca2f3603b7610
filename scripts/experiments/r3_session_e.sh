# Receive cost of one gRPC stream by component (reader_cost_probe.py), then
# a full bench with the ring's THP backing reported.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_e; mkdir -p $O
timeout -k 10 300 python3 scripts/experiments/reader_cost_probe.py --reps 3 > $O/reader_cost.jsonl 2> $O/reader_cost.err
echo "probe rc=$?"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
echo "bench rc=$?"
grep -E "AnonHugePages|HugePages_|Hugepagesize" /proc/meminfo > $O/meminfo.txt
cat /sys/kernel/mm/transparent_hugepage/khugepaged/defrag /proc/buddyinfo > $O/buddy.txt 2>&1
