#!/usr/bin/env python3
"""CRC32C kernel (K1+K2) throughput on one MI355X, vs HBM bandwidth.

Prints one JSON line per configuration: bytes covered, segment size, GB/s.
Each run checks the first segment's CRC against the host CRC32C.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import custom_go_client_benchmark_amd as pkg  # noqa: E402

n = pkg._native


def main():
    total = int(os.environ.get("CRC_BYTES", 1 << 30))
    t = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    for seg in [2 << 20, 8 << 20, 32 << 20]:
        cover = min(total, seg * 32)
        gbs, c0 = n.gpu_crc32c_throughput(0, t.data_ptr(), cover, int(os.environ.get("CRC_ITERS", 20)), seg)
        want = n.crc32c(t[:seg].cpu().numpy().tobytes())
        print(json.dumps({"kernel": "crc32c_tiles+segments", "seg_bytes": seg, "bytes": cover,
                          "GB/s": round(gbs, 1), "crc_ok": c0 == want}), flush=True)
    # copy bandwidth reference for the same device (torch D2D)
    a = torch.empty_like(t)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.copy_(t)
    e0.record()
    for _ in range(10):
        a.copy_(t)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"reference": "torch D2D copy", "GB/s (read+write)": round(2 * total * 10 / (e0.elapsed_time(e1) / 1e3) / 1e9, 1)}))


if __name__ == "__main__":
    main()
