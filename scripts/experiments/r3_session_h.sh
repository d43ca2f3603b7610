# 48 x 1 MiB HTTP first-rep stall: thread states every 2 ms, per-thread run
# delay and vmstat deltas per rep; warm-up length and a pause varied.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_h; mkdir -p $O
timeout -k 10 200 python3 scripts/experiments/w48_tail_probe.py --reps 3 > $O/w48_default.jsonl 2> $O/w48_default.err; echo "default rc=$?"
timeout -k 10 200 python3 scripts/experiments/w48_tail_probe.py --reps 2 --warm-reads 20 > $O/w48_warm20.jsonl 2> $O/w48_warm20.err; echo "warm20 rc=$?"
timeout -k 10 200 python3 scripts/experiments/w48_tail_probe.py --reps 2 --gap-s 3 > $O/w48_gap3.jsonl 2> $O/w48_gap3.err; echo "gap3 rc=$?"
