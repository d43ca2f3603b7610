# Is the headline's receive slower inside bench.py than in a bare probe
# process?  Interleaved on one box: bench (RCCL), probe, bench (gloo control
# plane), probe, bench (RCCL).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_f; mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --blocks cpu_baseline,ceiling > $O/bench_rccl_1.log 2>&1; echo "b1 rc=$?"
timeout -k 10 200 python3 scripts/experiments/reader_cost_probe.py --reps 1 > $O/probe_1.jsonl 2>&1; echo "p1 rc=$?"
GCSB_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --blocks cpu_baseline,ceiling > $O/bench_gloo.log 2>&1; echo "b2 rc=$?"
timeout -k 10 200 python3 scripts/experiments/reader_cost_probe.py --reps 1 > $O/probe_2.jsonl 2>&1; echo "p2 rc=$?"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --blocks cpu_baseline,ceiling > $O/bench_rccl_2.log 2>&1; echo "b3 rc=$?"
