set -u
mkdir -p gpurun_out/crc
timeout -k 10 300 python -u -m pytest tests/test_gpu_crc32c.py tests/test_gpu_sink.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/crc/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/crc/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/experiments/crc_latency_probe.py > gpurun_out/crc/probe_slot.jsonl 2>&1 || exit 1
PROBES=0 GCSB_CRC_SLOT_WAVES=1 timeout -k 10 200 python scripts/experiments/crc_latency_probe.py > gpurun_out/crc/probe_w1.jsonl 2>&1 || exit 1
PROBES=0 GCSB_CRC_SLOT_WAVES=4 timeout -k 10 200 python scripts/experiments/crc_latency_probe.py > gpurun_out/crc/probe_w4.jsonl 2>&1 || exit 1
PROBES=0 GCSB_CRC_SLOT_WAVES=8 timeout -k 10 200 python scripts/experiments/crc_latency_probe.py > gpurun_out/crc/probe_w8.jsonl 2>&1 || exit 1
PROBES=0 GCSB_CRC_SLOT=0 timeout -k 10 200 python scripts/experiments/crc_latency_probe.py > gpurun_out/crc/probe_fused.jsonl 2>&1 || exit 1
grep -h '^{' gpurun_out/crc/probe_slot.jsonl | cut -c1-90
for f in w1 w4 w8 fused; do echo $f; grep -h '^{' gpurun_out/crc/probe_$f.jsonl | cut -c1-90; done
