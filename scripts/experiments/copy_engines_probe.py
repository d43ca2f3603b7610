"""SDMA copy engines and the pinned <-> HBM copy ceiling on one MI355X.

1. copy_engine_probe: engines per direction, per-engine first / second /
   after-hipDeviceSynchronize tiny-copy times (run with GCSB_WARM_ENGINES=0
   so nothing has warmed them yet).
2. copy_ceiling: 256 MiB as 2 MiB hipMemcpyAsync copies from an 8-slot
   pinned THP ring, over 1 / 2 / 4 / 8 pool streams, H2D and D2H.
One JSON line each."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402,F401

import custom_go_client_benchmark_amd as pkg  # noqa: E402

n = pkg._native
print(json.dumps({"probe": json.loads(n.copy_engine_probe(0))}), flush=True)
for d in ("h2d", "d2h"):
    for st in (1, 2, 4, 8):
        r = n.copy_ceiling(0, d, 256 << 20, 2 << 20, 8, st, 5)
        print(json.dumps({"dir": d, "streams": st, **{k: round(v, 3) for k, v in r.items()}}), flush=True)
print(json.dumps({"h2d_64MiB_chunks": n.copy_ceiling(0, "h2d", 256 << 20, 64 << 20, 2, 2, 5)}), flush=True)
