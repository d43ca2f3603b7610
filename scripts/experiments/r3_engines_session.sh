set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_engines; mkdir -p $O
GCSB_WARM_ENGINES=0 timeout -k 10 120 python3 scripts/experiments/copy_engines_probe.py > $O/engines.jsonl 2> $O/engines.err
echo "engines rc=$?"
for i in 1 2; do
  for w in 0 1; do
    GCSB_WARM_ENGINES=$w timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --list-objects 0 > $O/bench_w${w}_$i.log 2>&1
    echo "bench w=$w i=$i rc=$?"
  done
done
