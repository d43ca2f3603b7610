set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
grep -io "SQ_[A-Z_]*MFMA[A-Z_0-9]*\|SQ_INSTS_VALU[A-Z_0-9]*\|SQ_VALU_MFMA[A-Z_0-9]*" gpurun_out/pmc/counters.txt | sort -u | head -30
for v in 1 0; do
  GCSB_CRC_MFMA=$v CRC_ITERS=3 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES --output-format csv -d gpurun_out/pmc/p$v -o crc -- python scripts/experiments/crc_bulk_once.py > gpurun_out/pmc/p$v.log 2>&1 || { tail -5 gpurun_out/pmc/p$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for v in (1, 0):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in glob.glob(f"gpurun_out/pmc/p{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if "crc32c" in r["Kernel_Name"] and "fold" not in r["Kernel_Name"]:
                agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, c in agg.items():
        print(v, k, {q: f"{x:.3g}" for q, x in c.items()})
PY
