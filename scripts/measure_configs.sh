#!/bin/bash
# Measures the BASELINE.json configs on one MI355X box (1-GPU parts; the
# 8-GPU scaling curve is the driver's bench.py run).  Each run writes a
# -summary-json under $OUT; scripts/configs_table.py turns them into the
# BASELINE.md table.  Every GPU step has its own time limit and a crash /
# abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/configs}
mkdir -p "$OUT"
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
MIB=1048576

run() {  # run <name> <timeout> <gcsbench args...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" ./gcsbench -start-fake-server -latency-file "$OUT/$name.lat" \
    -summary-json "$OUT/$name.json" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 2 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
}

[ -f custom_go_client_benchmark_amd/_native*.so ] || timeout -k 10 900 make -j16 all > "$OUT/build.log" 2>&1 || exit 1

# config 1: single 1 MiB object, HTTP, CPU-only (discard sink + host CRC, the
# reference's io.Discard path); gRPC alongside for comparison
run c1_http_1m_cpu 300 -client-protocol http -worker 1 -read-call-per-worker 3000 -fake-object-size $MIB
run c1_grpc_1m_cpu 300 -client-protocol grpc -worker 1 -read-call-per-worker 3000 -fake-object-size $MIB
run c1_http_1m_cpu_w48 300 -client-protocol http -worker 48 -read-call-per-worker 200 -fake-object-size $MIB
run c1_grpc_1m_cpu_w48 300 -client-protocol grpc -worker 48 -read-call-per-worker 200 -fake-object-size $MIB

# config 2: 256 MiB sequential reads -> HBM (pinned ring + hipMemcpyAsync +
# CRC32C kernels); CPU-only reference-equivalent alongside
S256=$((256 * MIB))
run c2_grpc_256m_hbm 300 -client-protocol grpc -sink gpu -worker 1 -read-call-per-worker 40 -fake-object-size $S256
run c2_http_256m_hbm 300 -client-protocol http -sink gpu -worker 1 -read-call-per-worker 40 -fake-object-size $S256
run c2_grpc_256m_hbm_s8 300 -client-protocol grpc -sink gpu -worker 1 -read-call-per-worker 40 -fake-object-size $S256 \
  -slices 8 -ring-slot-bytes 4194304
run c2_http_256m_hbm_s8 300 -client-protocol http -sink gpu -worker 1 -read-call-per-worker 40 -fake-object-size $S256 \
  -slices 8 -ring-slot-bytes 4194304
run c2_grpc_256m_cpu 300 -client-protocol grpc -worker 1 -read-call-per-worker 40 -fake-object-size $S256
run c2_http_256m_cpu 300 -client-protocol http -worker 1 -read-call-per-worker 40 -fake-object-size $S256

# config 3: list 1000 x 1 MiB objects, read every one into HBM; HTTP vs gRPC
for p in http grpc; do
  run c3_${p}_list1000_hbm 300 -workload list-read -client-protocol $p -sink gpu -worker 8 \
    -read-call-per-worker 3 -fake-objects 1000 -fake-object-size $MIB
  run c3_${p}_list1000_cpu 300 -workload list-read -client-protocol $p -worker 8 \
    -read-call-per-worker 3 -fake-objects 1000 -fake-object-size $MIB
done

# config 5 (1-GPU part): 64 MiB uploads HBM -> pinned -> resumable / WriteObject.
# The synthetic server verifies size + CRC32C of every upload; the first run
# discards the bytes after that (server-side io.Discard), the second keeps them.
for p in grpc http; do
  run c5_${p}_write64m 300 -workload write -client-protocol $p -sink gpu -worker 1 -write-objects 20 \
    -fake-retain-uploads=false \
    -write-size $((64 * MIB)) -fake-objects 1 -fake-object-size $MIB
  run c5_${p}_write64m_pcu8 300 -workload write -client-protocol $p -sink gpu -worker 1 -write-objects 20 \
    -fake-retain-uploads=false -slices 8 -write-size $((64 * MIB)) -fake-objects 1 -fake-object-size $MIB
  run c5_${p}_write64m_retain 300 -workload write -client-protocol $p -sink gpu -worker 1 -write-objects 20 \
    -write-size $((64 * MIB)) -fake-objects 1 -fake-object-size $MIB
done
echo "done"
