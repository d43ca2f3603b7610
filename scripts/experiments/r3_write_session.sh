# Config-5 upload A/B: endpoint WriteObject CRC on the reader thread (0) vs
# the connection's write worker (1), interleaved, write block per-thread CPU.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_write; mkdir -p $O
for i in 1 2; do
  for w in 0 1; do
    GCSB_SRV_WRITE_WORKER=$w timeout -k 10 200 python3 bench.py --workload write --steps 30 --warmup 3 > $O/write_w${w}_$i.log 2>&1
    echo "write w=$w i=$i rc=$?"
  done
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --list-objects 0 > $O/bench.log 2>&1
echo "bench rc=$?"
