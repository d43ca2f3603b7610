set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_stall; mkdir -p $O
timeout -k 10 200 python3 scripts/experiments/sync_stall_probe.py --reps 8 > $O/probe_default.jsonl 2> $O/probe_default.err
echo "default rc=$?"
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 scripts/experiments/sync_stall_probe.py --reps 8 > $O/probe_hwq8.jsonl 2> $O/probe_hwq8.err
echo "hwq8 rc=$?"
GCSB_STREAMS=4 timeout -k 10 200 python3 scripts/experiments/sync_stall_probe.py --reps 8 > $O/probe_pool4.jsonl 2> $O/probe_pool4.err
echo "pool4 rc=$?"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
echo "bench rc=$?"
timeout -k 10 300 rocprofv3 --hip-runtime-trace --memory-copy-trace --kernel-trace --output-format csv -d $O/trace -o b -- python3 scripts/experiments/sync_stall_probe.py --reps 4 --variants sync > $O/trace.log 2>&1
echo "trace rc=$?"
ls $O/trace
