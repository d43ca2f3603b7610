#!/bin/bash
# Slot CRC epilogue A/B: 64-bit XOR-atomic arrival words (default for
# one-segment batches) vs per-tile stores + two-level done counter + fold
# loads (GCSB_CRC_XOR=0).  GPU CRC tests under both, then per-launch us.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/crc_xor}
mkdir -p $OUT
for x in 1 0; do
  GCSB_CRC_XOR=$x timeout -k 10 300 python -u -m pytest tests/test_gpu_crc32c.py tests/test_gpu_sink.py -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_xor$x.log 2>&1 \
    || { tail -20 $OUT/pytest_xor$x.log; exit 1; }
  tail -1 $OUT/pytest_xor$x.log
done
for rep in 1 2 3; do
  for x in 1 0; do
    PROBES="${PROBES:-4 3 0}" GCSB_CRC_XOR=$x timeout -k 10 120 python scripts/experiments/crc_latency_probe.py 2>/dev/null \
      | grep '^{' | sed "s/^{/{\"xor\": $x, /" | tee -a $OUT/probe.jsonl | cut -c1-120 || exit 1
  done
done
python3 - $OUT/probe.jsonl <<'PY' | tee $OUT/summary.txt
import json, sys, collections
v = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l)
    v[(d["xor"], d["probe"], d["bytes"], d["seg_bytes"])].append(d["us_per_launch"])
for k in sorted(v):
    print("xor=%d probe=%d bytes=%d seg=%d  min %.2f us  all %s" % (*k, min(v[k]), v[k]))
PY
