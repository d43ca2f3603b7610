# N=8 rehearsal on one MI355X (verdict r2 item 3b): 8 rank processes share the
# GPU over a gloo control plane, every side block on, fan-out included.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_rehearsal8; mkdir -p $O
t0=$(date +%s.%N)
GCSB_DIST_BACKEND=gloo timeout -k 10 500 python3 bench.py --gpus 8 --object-size 64MiB --steps 5 --side-steps 3 \
  > $O/rehearsal8.log 2>&1
rc=$?
t1=$(date +%s.%N)
echo "rehearsal8 rc=$rc wall_s=$(python3 -c "print(round($t1-$t0,1))")" | tee $O/wall.txt
