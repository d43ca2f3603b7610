# Round-3 check after the receive-destination / handler-pool changes:
# the full bench once, then the multiplexed and upload blocks twice each.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_b; mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
echo "bench rc=$?"
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --side-steps 5 --blocks list_read,ref_default > $O/mux_$i.log 2>&1
  echo "mux i=$i rc=$?"
  for w in 0 1; do
    GCSB_SRV_WRITE_WORKER=$w timeout -k 10 200 python3 bench.py --workload write --steps 30 --warmup 3 > $O/write_w${w}_$i.log 2>&1
    echo "write w=$w i=$i rc=$?"
  done
done
