#!/usr/bin/env python3
"""One bulk CRC32C configuration (for rocprofv3 --pmc passes): 1 GiB in 32 MiB
segments, 4 KiB tiles, CRC_ITERS launches; GCSB_CRC_MFMA selects the tile kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import custom_go_client_benchmark_amd as pkg  # noqa: E402

t = torch.randint(0, 256, (1 << 30,), dtype=torch.uint8, device="cuda:0")
torch.cuda.synchronize()
gbs, _ = pkg._native.gpu_crc32c_throughput(0, t.data_ptr(), 1 << 30, int(os.environ.get("CRC_ITERS", 5)), 32 << 20,
                                           int(os.environ.get("CRC_TILE_LOG2", 12)))
print(f"GB/s {gbs:.1f}")
