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


class HbmReader:
    """Reusable object -> HBM reader for PyTorch users.

    ``slices == 1``: one stream per object through a GpuSink (pinned ring ->
    hipMemcpyAsync -> HBM, CRC32C on the GPU), the reference's one NewReader
    per object.  ``slices > 1``: a sliced read (csrc/storage/sliced.h) -- N
    concurrent ranged streams, each on its own connection, landing at their
    offsets of the destination; the object CRC32C is combined from the slices
    and checked.  Pinned rings, streams and connections are created once and
    reused across reads.

        r = HbmReader("grpc", "http://127.0.0.1:8080", device=0, slices=8)
        t, res = r.read("bucket", "object")          # new uint8 tensor
        r.read("bucket", "object", out=t)            # into an existing tensor
    """

    def __init__(self, protocol: str, endpoint: str, device: int = 0, slices: int = 1, slot_bytes: int = 4 << 20,
                 slots: int = 4, **client_cfg):
        gpu_required()
        self.device = device
        self.slices = max(1, int(slices))
        cfg = {"protocol": protocol, "endpoint": endpoint, "device": device, "ring_slot_bytes": slot_bytes,
               "ring_slots": slots}
        cfg.update(client_cfg)
        self._client = _native.Client(cfg)
        self._sink = None
        self._sliced = None
        if self.slices > 1:
            self._sliced = _native.SlicedGpuReader({**cfg, "slices": self.slices})
        else:
            self._sink = _native.GpuSink(cfg)

    def read(self, bucket: str, name: str, out=None):
        import torch

        if out is None:
            size = int(self._client.stat(bucket, name)["size"])
            out = torch.empty(size, dtype=torch.uint8, device=f"cuda:{self.device}")
        if not (out.is_cuda and out.is_contiguous() and out.dtype == torch.uint8):
            raise ValueError("out must be a contiguous torch.uint8 CUDA tensor")
        if self._sliced is not None:
            res = self._sliced.read_into(bucket, name, out.data_ptr(), out.numel())
        else:
            self._sink.set_external_destination(out.data_ptr(), out.numel())
            res = self._client.read_gpu(bucket, name, self._sink)
        if res.get("crc_mismatch"):
            raise _native.StorageError(f"CRC32C mismatch reading {bucket}/{name}: {res.get('detail', '')}")
        return out, res
