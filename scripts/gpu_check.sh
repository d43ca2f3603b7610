#!/bin/bash
# One GPU-box session: GPU tests, smoke, a short bench and a rocprofv3 kernel
# profile.  Every GPU step has its own time limit; a crash/abort/timeout ends
# the script (test *failures* do not — their logs are what we came for).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0

step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "fatal rc=$rc in $name: stopping"; exit $rc
  fi
  return $rc
}

step import 300 python -c "import custom_go_client_benchmark_amd as p; print(p._native.__file__)" || exit 1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -X faulthandler bench.py --steps ${BENCH_STEPS:-20} --warmup 3 --json-out $OUT/bench.json
if [ "${PROFILE:-1}" = "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
    python bench.py --steps 10 --warmup 2
fi
echo "done"
