"""Pinned host -> HBM copy ceiling on this box (the bound under bench.py's
HBM landing): one big copy, chunked copies on 1..4 streams, for the engine
that HIP picks (SDMA unless HSA_ENABLE_SDMA=0 selects blit kernels).
Prints one JSON line per configuration."""
import json
import os

import torch

MIB = 1 << 20


def run(total, chunk, nstreams, reps=10):
    src = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    src.fill_(7)
    dst = torch.empty(total, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    times = []
    for r in range(reps + 2):
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for s in streams:
            s.wait_event(t0)
        for i, off in enumerate(range(0, total, chunk)):
            s = streams[i % nstreams]
            with torch.cuda.stream(s):
                dst[off:off + chunk].copy_(src[off:off + chunk], non_blocking=True)
        for s in streams:
            torch.cuda.current_stream().wait_stream(s)
        t1.record()
        torch.cuda.synchronize()
        if r >= 2:
            times.append(t0.elapsed_time(t1))
    times.sort()
    ms = times[len(times) // 2]
    return {"sdma": os.environ.get("HSA_ENABLE_SDMA", "default"), "total_mib": total // MIB,
            "chunk_mib": chunk / MIB, "streams": nstreams, "p50_ms": round(ms, 3),
            "GB_s": round(total / ms / 1e6, 1), "GiB_s": round(total / ms * 1e3 / 2**30, 2)}


if __name__ == "__main__":
    total = 256 * MIB
    for chunk, ns in [(total, 1), (4 * MIB, 1), (4 * MIB, 2), (4 * MIB, 4), (2 * MIB, 4), (1 * MIB, 4),
                      (8 * MIB, 4)]:
        print(json.dumps(run(total, chunk, ns)), flush=True)
