# Round-3 GPU check: the GPU test suite, smoke(), the N=8 gloo rehearsal on one
# MI355X (verdict r2 item 3b), and a rocprofv3 kernel profile of the bench.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O_C:-gpurun_out/r3_c}; mkdir -p $O
step() {  # step <name> <timeout> <cmd...>; a crash/abort/timeout ends the session
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  local t0=$(date +%s.%N)
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc wall_s=$(python3 -c "print(round($(date +%s.%N)-$t0,1))")"
  tail -n 3 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step rehearsal8 500 env GCSB_DIST_BACKEND=gloo python3 bench.py --gpus 8 --object-size 64MiB --steps 5 --side-steps 3
step write_trace 200 env GCSB_TRACE_SOURCE=1 python3 bench.py --workload write --steps 30 --warmup 3
step rocprof 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o bench -- \
  python3 bench.py --steps 10 --warmup 2
echo done
