#!/usr/bin/env python3
"""Decomposes the per-launch time of the fused CRC32C kernel on a slot-sized
batch: GCSB_CRC_PROBE=2 exits at kernel entry (launch + dispatch of the
grid), =1 after the LDS table staging, unset = the full kernel.  Run once per
probe value (the probe is read per call)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import custom_go_client_benchmark_amd as pkg  # noqa: E402

n = pkg._native
t = torch.randint(0, 256, (8 << 20,), dtype=torch.uint8, device="cuda:0")
torch.cuda.synchronize()
for probe in os.environ.get("PROBES", "2 1 4 3 0").split():
    os.environ["GCSB_CRC_PROBE"] = probe
    for cover, seg in [(1 << 20, 1 << 20), (2 << 20, 1 << 20), (2 << 20, 2 << 20), (4 << 20, 4 << 20)]:
        best = None
        for _ in range(3):
            gbs, c0 = n.gpu_crc32c_throughput(0, t.data_ptr() + 7, cover, 400, seg, 12)
            us = cover / (gbs * 1e9) * 1e6
            best = us if best is None else min(best, us)
        print(json.dumps({"probe": int(probe), "bytes": cover, "seg_bytes": seg, "us_per_launch": round(best, 2),
                          "variant": os.environ.get("GCSB_CRC_VARIANT", "")}), flush=True)
