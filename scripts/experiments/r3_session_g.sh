# 48 x 1 MiB HTTP / gRPC tail: every read recorded, slow ones listed by start time.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_g; mkdir -p $O
timeout -k 10 200 python3 scripts/experiments/w48_tail_probe.py --protocol http --reps 3 > $O/w48_http.jsonl 2> $O/w48_http.err; echo "http rc=$?"
timeout -k 10 200 python3 scripts/experiments/w48_tail_probe.py --protocol grpc --reps 2 --slow-ms 30 > $O/w48_grpc.jsonl 2> $O/w48_grpc.err; echo "grpc rc=$?"
