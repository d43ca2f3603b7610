#!/bin/bash
# Slot CRC kernel A/B on one GPU: byte vs bank-replicated nibble tables x
# waves per workgroup (per-launch us on 1-4 MiB batches), correctness of
# each variant, and LDS bank-conflict counters (rocprofv3 --pmc, own pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/crc_ab}
mkdir -p $OUT
for nib in 0 1; do
  GCSB_CRC_NIB=$nib timeout -k 10 300 python -u -m pytest tests/test_gpu_crc32c.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $OUT/pytest_nib$nib.log 2>&1 || { tail -20 $OUT/pytest_nib$nib.log; exit 1; }
  tail -1 $OUT/pytest_nib$nib.log
done
for rep in 1 2; do
  for nib in 0 1; do
    for w in 1 2 4; do
      PROBES=0 GCSB_CRC_NIB=$nib GCSB_CRC_SLOT_WAVES=$w timeout -k 10 120 python scripts/experiments/crc_latency_probe.py \
        2>/dev/null | grep '^{' | sed "s/^{/{\"nib\": $nib, \"waves\": $w, /" | tee -a $OUT/probe.jsonl | cut -c1-120 \
        || exit 1
    done
  done
done
for nib in 0 1; do
  PROBES=0 GCSB_CRC_NIB=$nib timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
    SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d $OUT/pmc_nib$nib -o crc -- \
    python scripts/experiments/crc_latency_probe.py > $OUT/pmc_nib$nib.log 2>&1 || { tail -5 $OUT/pmc_nib$nib.log; exit 1; }
done
timeout -k 10 120 python3 - <<'PY'
import csv, glob, collections, json
for nib in (0, 1):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for p in glob.glob(f"gpurun_out/crc_ab/pmc_nib{nib}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            if "crc32c" not in k:
                continue
            k = k.split("(")[0][:60]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(k, r["Counter_Name"])] += 1
    for k, c in agg.items():
        lds = c.get("SQ_INSTS_LDS", 0.0)
        print(json.dumps({"nib": nib, "kernel": k, "counters": {q: round(v) for q, v in c.items()},
                          "bank_conflict_cycles_per_LDS_instr": round(c.get("SQ_LDS_BANK_CONFLICT", 0) / max(lds, 1), 3)}))
PY
echo done
