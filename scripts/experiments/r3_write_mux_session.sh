# Config-5 upload A/Bs on one box, interleaved (write headline, 30 uploads):
#   GCSB_UPLOAD_SPLICE      1: whole-object staging ring, content spliced to the socket; 0: copied (round 2)
#   GCSB_SRV_WRITE_WORKER   1: endpoint CRC on the connection's write worker (GCSB_SRV_WRITE_BUFS
#                           buffers in rotation); 0: inline on its reader thread
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_write3; mkdir -p $O
for i in 1 2; do
  for v in "1 0 2" "1 1 2" "1 1 1" "0 0 2"; do
    set -- $v
    GCSB_UPLOAD_SPLICE=$1 GCSB_SRV_WRITE_WORKER=$2 GCSB_SRV_WRITE_BUFS=$3 timeout -k 10 200 \
      python3 bench.py --workload write --steps 30 --warmup 3 > $O/write_s$1_w$2_b$3_$i.log 2>&1
    echo "write splice=$1 worker=$2 bufs=$3 i=$i rc=$?"
  done
done
# Many streams on one connection (config 3 list+read over gRPC pool 1, the
# reference's 48 x 1 MiB default): ring geometry A/B, reader-thread profile.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_mux; mkdir -p $O
for i in 1 2; do
  for ring in 8x2MiB 2x1MiB 4x512KiB; do
    timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --side-steps 5 --blocks list_read,ref_default \
      --list-ring $ring > $O/mux_${ring}_$i.log 2>&1
    echo "mux ring=$ring i=$i rc=$?"
  done
done
