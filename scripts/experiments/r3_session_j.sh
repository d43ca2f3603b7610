# (1) 48 x 1 MiB HTTP after the fd-table reservation: is the first-rep stall gone?
# (2) multiplexed gRPC: reader thread on a core of its own (isolate) vs shared,
#     48 x 1 MiB on one connection and config-3 list-read, interleaved.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_j; mkdir -p $O
timeout -k 10 200 python3 scripts/experiments/w48_tail_probe.py --reps 2 > $O/w48_http.jsonl 2> $O/w48_http.err; echo "w48 http rc=$?"
for k in 1 2; do
  timeout -k 10 200 python3 scripts/experiments/w48_tail_probe.py --protocol grpc --reps 2 --sample-ms 0 > $O/w48_grpc_shared_$k.jsonl 2>&1; echo "grpc shared$k rc=$?"
  timeout -k 10 200 python3 scripts/experiments/w48_tail_probe.py --protocol grpc --reps 2 --sample-ms 0 --isolate-reader > $O/w48_grpc_isolate_$k.jsonl 2>&1; echo "grpc isolate$k rc=$?"
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --blocks list_read,ref_default > $O/bench_shared_$k.log 2>&1; echo "bench shared$k rc=$?"
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --blocks list_read,ref_default --mux-reader isolate > $O/bench_isolate_$k.log 2>&1; echo "bench isolate$k rc=$?"
done
