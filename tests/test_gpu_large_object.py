"""Objects larger than 4 GiB streamed into HBM (object size is
this benchmark's "sequence length"; the reference streams arbitrarily large
objects with constant memory, /root/reference/main.go:140, and its FS matrix
goes to 1 GB objects, benchmark-script/read_operation/read_operations.sh:14).

A 5 GiB + 12345 B synthetic object crosses the 32-bit byte-offset boundary
(4 GiB) inside one read.  Both transports land it in a caller-owned HBM
tensor (landing = object): gRPC as one ReadObject stream (the reference's
path), HTTP as a sliced read of 4 ranged streams pulling 64 MiB pieces.
Checks: every ChecksummedData / whole-object CRC32C verified on the GPU, the
GPU CRC32C of the landed bytes equal to the server's stored CRC32C, a full
pattern check in HBM, and byte-exact host comparisons (D2H) of 64 MiB windows
at the start, across the 4 GiB boundary and at the end against the server's
own object bytes.
"""
import pytest

pytestmark = pytest.mark.gpu

B = "large-bucket"
P = "large_objects/file_"
SIZE = (5 << 30) + 12345
WIN = 64 << 20


@pytest.fixture(scope="module")
def big_server(native):
    srv = native.Server({"port": 0, "md5": False})
    srv.start()
    srv.add_synthetic(B, P, "", 0, 1, SIZE)
    yield srv
    srv.stop()


def _check_landed(native, srv, dst):
    import torch

    name = P + "0"
    torch.cuda.synchronize()
    assert native.gpu_crc32c(0, dst.data_ptr(), SIZE) == srv.object_info(B, name)["crc32c"]
    bad, first = native.gpu_verify_pattern(0, dst.data_ptr(), SIZE, name, 0)
    assert bad == 0, first
    for off in (0, (4 << 30) - WIN // 2, SIZE - WIN):
        got = dst[off:off + WIN].cpu().numpy().tobytes()
        assert got == srv.object_bytes(B, name, off, WIN), off


@pytest.mark.parametrize("slot", [2 << 20, 8 << 20])
def test_grpc_single_stream_5gib(native, big_server, gpu_available, slot):
    import torch

    dst = torch.empty(SIZE, dtype=torch.uint8, device="cuda:0")
    c = native.Client({"protocol": "grpc", "endpoint": big_server.url})
    sink = native.GpuSink({"device": 0, "ring_slot_bytes": slot, "ring_slots": 8, "async_submit": slot == 2 << 20})
    sink.set_external_destination(dst.data_ptr(), dst.numel())
    r = c.read_gpu(B, P + "0", sink)
    assert r["bytes"] == SIZE and r["verified"] and not r["crc_mismatch"], r
    st = sink.stats()
    assert st["objects_verified"] == 1 and st["chunks_verified_gpu"] + st["chunks_verified_host"] >= SIZE >> 21
    _check_landed(native, big_server, dst)
    del dst


def test_http_sliced_5gib(native, big_server, gpu_available):
    import torch

    dst = torch.empty(SIZE, dtype=torch.uint8, device="cuda:0")
    rd = native.SlicedGpuReader({"protocol": "http", "endpoint": big_server.url, "device": 0, "slices": 4,
                                 "slice_piece_bytes": 64 << 20, "ring_slot_bytes": 4 << 20, "ring_slots": 4})
    r = rd.read_into(B, P + "0", dst.data_ptr(), dst.numel())
    assert r["bytes"] == SIZE and r["verified"] and not r["crc_mismatch"], r
    _check_landed(native, big_server, dst)
    del dst
