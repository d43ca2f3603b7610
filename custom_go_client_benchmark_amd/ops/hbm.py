"""HBM landing helpers on top of the native GPU sink.

The GPU sink (csrc/gpu/engine.hip) receives object bytes into a page-locked
ring, copies each full slot to HBM with hipMemcpyAsync on its own stream and
verifies CRC32C with the CDNA4 kernels (csrc/gpu/crc32c_kernels.hip).  These
helpers expose that path to PyTorch users: read an object straight into a
``torch.uint8`` CUDA tensor.
"""
from __future__ import annotations

from .. import _native


def available_protocols() -> list[str]:
    """Transports compiled into the native module."""
    protos = ["http"]
    if getattr(_native, "HAS_GRPC", False):
        protos.append("grpc")
    return protos


def gpu_required() -> None:
    """Fail loudly when the HIP path cannot run (no silent CPU fallback)."""
    if _native.gpu_device_count() <= 0:
        raise RuntimeError("no HIP device visible: the GPU data plane cannot run on this host")


def read_object_to_tensor(client, bucket: str, name: str, device: int = 0, sink=None,
                          slot_bytes: int = 8 << 20, slots: int = 4):
    """Reads ``bucket/name`` into a new uint8 tensor on ``cuda:device``.

    Returns (tensor, result_dict).  The tensor holds the object bytes exactly;
    ``result['verified']`` is True when every server checksum matched the
    GPU-computed CRC32C.
    """
    import torch

    gpu_required()
    meta = client.stat(bucket, name)
    out = torch.empty(int(meta["size"]), dtype=torch.uint8, device=f"cuda:{device}")
    if sink is None:
        sink = _native.GpuSink({"device": device, "ring_slot_bytes": slot_bytes, "ring_slots": slots})
    sink.set_external_destination(out.data_ptr(), out.numel())
    res = client.read_gpu(bucket, name, sink)
    return out, res


def crc32c(tensor) -> int:
    """CRC32C of a contiguous CUDA tensor's bytes, computed by the HIP kernels."""
    gpu_required()
    t = tensor.contiguous()
    return _native.gpu_crc32c(t.device.index or 0, t.data_ptr(), t.numel() * t.element_size())
