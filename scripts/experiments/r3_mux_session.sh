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
