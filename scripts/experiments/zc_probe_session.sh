#!/bin/bash
# TCP zero-copy receive on the GPU box's host (csrc/tools/zc_probe.cc): the
# copying recv() against TCP_ZEROCOPY_RECEIVE with a sendfile() sender (page-
# cache pages) and a send(MSG_ZEROCOPY) sender.  CPU only; no GPU call.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/zc
mkdir -p "$OUT"
read -r -a C < <(python3 -c "import os; print(' '.join(map(str, sorted(os.sched_getaffinity(0))[:6])))")
P=custom_go_client_benchmark_amd/bin/zc_probe
run() {
  local name=$1; shift
  timeout -k 5 60 "$P" -total 8589934592 -send-cpu "${C[0]}" -recv-cpu "${C[1]}" -worker-cpus "${C[2]},${C[3]},${C[4]}" "$@" \
    | tee -a "$OUT/zc.jsonl"
}
for rep in 1 2; do
  run recv -mode recv
  run zc_map_sendfile -mode zc_map -send sendfile
  run zc_map_mzc -mode zc_map -send msg_zerocopy
  run zc_workers_mzc -mode zc_workers -workers 3 -send msg_zerocopy
  run recv_mzc -mode recv -send msg_zerocopy
done
