#!/usr/bin/env python3
"""CRC32C kernel throughput and per-launch time on one MI355X.

bulk : 1 GiB in 32 MiB segments (the kernel's streaming rate vs HBM);
slot : one ring-slot-sized batch per launch (1 / 2 / 4 MiB, one or two
       segments) back-to-back, reported as microseconds per launch: this is
       what sits on a read's latency path after its last byte lands.
Each configuration runs with 4 KiB and 16 KiB tiles (tile_log2 12 / 14) and
checks the first segment's CRC against the host CRC32C.  One JSON line each.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import custom_go_client_benchmark_amd as pkg  # noqa: E402

n = pkg._native


def main():
    if os.environ.get("CRC_OPTS"):  # e.g. '{"bank_private": true}' (CrcLaunchOptions)
        print(json.dumps({"crc_options": n.set_crc_options(json.loads(os.environ["CRC_OPTS"]))}), flush=True)
    total = int(os.environ.get("CRC_BYTES", 1 << 30))
    iters = int(os.environ.get("CRC_ITERS", 20))
    t = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    host = {}

    def host_crc(off, ln):
        k = (off, ln)
        if k not in host:
            host[k] = n.crc32c(t[off:off + ln].cpu().numpy().tobytes())
        return host[k]

    for tl in (12, 14):
        for seg in [32 << 20]:
            cover = min(total, seg * 32)
            gbs, c0 = n.gpu_crc32c_throughput(0, t.data_ptr(), cover, iters, seg, tl)
            print(json.dumps({"case": "bulk", "tile_kib": (1 << tl) >> 10, "seg_bytes": seg, "bytes": cover,
                              "GB/s": round(gbs, 1), "crc_ok": c0 == host_crc(0, seg)}), flush=True)
        for cover, seg in [(1 << 20, 1 << 20), (2 << 20, 2 << 20), (2 << 20, 1 << 20), (4 << 20, 4 << 20),
                           (2 << 20, (2 << 20) // 3)]:
            gbs, c0 = n.gpu_crc32c_throughput(0, t.data_ptr() + 7, cover, max(iters, 200), seg, tl)
            us = cover / (gbs * 1e9) * 1e6
            print(json.dumps({"case": "slot", "tile_kib": (1 << tl) >> 10, "seg_bytes": seg, "bytes": cover,
                              "us_per_launch": round(us, 2), "GB/s": round(gbs, 1),
                              "crc_ok": c0 == host_crc(7, min(seg, cover))}), flush=True)
    # copy bandwidth reference for the same device (torch D2D)
    a = torch.empty_like(t)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.copy_(t)
    e0.record()
    for _ in range(10):
        a.copy_(t)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"reference": "torch D2D copy",
                      "GB/s (read+write)": round(2 * total * 10 / (e0.elapsed_time(e1) / 1e3) / 1e9, 1)}))


if __name__ == "__main__":
    main()
