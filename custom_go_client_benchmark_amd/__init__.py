"""MI355X-native object-storage read benchmark (capabilities of
tritone/custom-go-client-benchmark, re-designed MI355X-first).

Layout:
  _native        C++/HIP core (transports, fake GCS server, GPU sink, kernels)
  models/        workloads: read, list+read, write (the "models" this benchmark runs)
  ops/           GPU ops: CRC32C kernels, pattern fill/verify, HBM landing
  parallel/      one-process-per-GPU launcher, RCCL barriers and stat reductions
  utils/         Go-compatible flags, metrics/trace exporters, latency files
  server/        synthetic GCS endpoint management
"""
from __future__ import annotations

import os as _os

# One HIP runtime per process: torch bundles libamdhip64.so.7 and loads it
# with RPATH; importing torch first makes our extension bind to that same copy
# (matching soname) instead of /opt/rocm's.
if _os.environ.get("GCSB_NO_TORCH", "0") != "1":
    try:  # pragma: no cover - import side effect only
        import torch as _torch  # noqa: F401
    except Exception:  # torch is optional for the CPU-only paths
        _torch = None

from . import _native  # noqa: E402

__version__ = "0.1.0"

StorageError = _native.StorageError

__all__ = ["_native", "StorageError", "__version__"]
