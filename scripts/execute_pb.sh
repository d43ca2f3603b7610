#!/bin/bash
# Experiment driver (reference execute_pb.sh:1-9): runs the benchmark once over
# gRPC and once over HTTP, turning each latency line "<ms>ms" into a bare float
# with `tr 'ms' ' '` (so histogram.py / the README snippet can read it), and
# uploads each result file.
#
#   ./scripts/execute_pb.sh <exp_number>
#
# Extra benchmark flags come from $GCSB_ARGS (default: a node-local synthetic
# endpoint, since the benchmark boxes have no network); a %p in them becomes
# the run's protocol (e.g. -summary-json sum_%p.json).  Results go to
# $GCSB_RESULTS_URI with `gsutil cp` when gsutil exists (reference target
# gs://princer-working-dirs/), otherwise they are copied to $GCSB_RESULTS_DIR.
set -e
exp="${1:?usage: execute_pb.sh <exp_number>}"
here="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
args="${GCSB_ARGS:--start-fake-server -worker 8 -read-call-per-worker 20}"
uri="${GCSB_RESULTS_URI:-gs://princer-working-dirs/}"
dir="${GCSB_RESULTS_DIR:-$here/results}"

upload() {
  if command -v gsutil >/dev/null 2>&1; then
    gsutil cp "$1" "$uri"
  else
    mkdir -p "$dir" && cp "$1" "$dir/"
  fi
}

grpc_file="grpc_${exp}.txt"
# shellcheck disable=SC2086
"$here/gcsbench" -client-protocol grpc ${args//%p/grpc} | tr 'ms' ' ' > "$grpc_file"
upload "$grpc_file"

http_file="http_${exp}.txt"
# shellcheck disable=SC2086
"$here/gcsbench" -client-protocol http ${args//%p/http} | tr 'ms' ' ' > "$http_file"
upload "$http_file"
