# Config-5 upload A/Bs on one box, interleaved (write headline, 30 uploads):
#   GCSB_UPLOAD_SPLICE      1: whole-object staging ring, content spliced to the socket; 0: copied (round 2)
#   GCSB_SRV_WRITE_WORKER   1: endpoint CRC on the connection's write worker; 0: on its reader thread
# Then a write trace (kernel + memory copy) to name the D2H staging copies.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_write2; mkdir -p $O
for i in 1 2; do
  for v in "1 1" "0 1" "1 0" "0 0"; do
    set -- $v
    GCSB_UPLOAD_SPLICE=$1 GCSB_SRV_WRITE_WORKER=$2 timeout -k 10 200 python3 bench.py --workload write --steps 30 --warmup 3 \
      > $O/write_s$1_w$2_$i.log 2>&1
    echo "write splice=$1 worker=$2 i=$i rc=$?"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace -o w -- \
  python3 bench.py --workload write --steps 10 --warmup 2 > $O/trace.log 2>&1
echo "trace rc=$?"
