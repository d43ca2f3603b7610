# (1) 48 x 1 MiB HTTP first-rep stall: which syscall the D-state threads sit in.
# (2) config-3 list-read A/B: end-of-read event wait by hipEventSynchronize
#     (runtime spins before it sleeps) vs polling with 10 us sleeps.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_i; mkdir -p $O
timeout -k 10 200 python3 scripts/experiments/w48_tail_probe.py --reps 2 > $O/w48_default.jsonl 2> $O/w48_default.err; echo "w48 rc=$?"
for k in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --blocks list_read > $O/list_sync_$k.log 2>&1; echo "sync$k rc=$?"
  GCSB_WAIT_POLL_US=10 timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --blocks list_read > $O/list_poll_$k.log 2>&1; echo "poll$k rc=$?"
done
