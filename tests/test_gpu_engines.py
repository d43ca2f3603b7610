"""SDMA copy engines, the copy ceiling and the zero-copy upload path on MI355X
(profiles/r3_sdma_engines, profiles/r3_write)."""
import json

import pytest

pytestmark = pytest.mark.gpu

B = "princer-working-dirs"


def test_every_copy_engine_is_warm(native, gpu_available):
    """After the stream pool is up (it warms every SDMA engine once), no
    engine pays the ~7 ms first-use cost any more, in either direction, and
    a device-wide synchronize does not make one cold again."""
    native.warm_copy_engines(0)  # 0 if the pool already did it
    p = json.loads(native.copy_engine_probe(0))
    assert "error" not in p, p
    assert p["num_sdma"] >= 1
    for d in ("h2d", "d2h"):
        assert p[d], p
        for e in p[d]:
            if "error" in e:
                continue  # an engine this direction cannot use
            assert e["first_ms"] < 2.0 and e["second_ms"] < 2.0 and e["after_sync_ms"] < 2.0, (d, e)


def test_no_read_handoff_blocks(native, server, gpu_available):
    """Slot hand-offs of a read (H2D copy, CRC launch, event) never block the
    submitting thread for >= 1 ms once the engines are warm, also right
    after a torch.cuda.synchronize()."""
    import torch

    size = 64 << 20
    server.add_synthetic(B, "eng/file_", "", 0, 1, size)
    c = native.Client({"protocol": "grpc", "endpoint": server.url})
    t = torch.empty(size, dtype=torch.uint8, device="cuda:0")
    sink = native.GpuSink({"device": 0, "ring_slot_bytes": 2 << 20, "ring_slots": 8})
    sink.set_external_destination(t.data_ptr(), size)
    assert c.read_gpu(B, "eng/file_0", sink)["verified"]
    native.reset_slow_hip_calls()
    for _ in range(3):
        torch.cuda.synchronize()
        r = c.read_gpu(B, "eng/file_0", sink)
        assert r["verified"] and not r["crc_mismatch"], r
    s = native.slow_hip_calls()
    assert s["calls"] >= 3 * 32 and s["slow"] == 0, s


@pytest.mark.parametrize("direction", ["h2d", "d2h"])
def test_copy_ceiling(native, gpu_available, direction):
    r = native.copy_ceiling(0, direction, 64 << 20, 2 << 20, 8, 8, 3)
    # PCIe Gen5 x16: tens of GB/s; far below would mean the copies fell off SDMA / pinned memory
    assert 10.0 < r["gbps"] < 100.0, r


@pytest.mark.parametrize("async_stage", [True, False])
@pytest.mark.parametrize("slot", [(1 << 20), (2 << 20)])
@pytest.mark.parametrize("size", [(64 << 20), (5 << 20) + 4321])
def test_spliced_upload_from_hbm_is_byte_exact(native, server, gpu_available, size, slot, async_stage):
    """Uploads from HBM stage the whole object (no slot refilled mid-upload)
    and hand the staged pages to the socket by reference (vmsplice +
    splice); the endpoint's CRC32C of what it received must equal the GPU's,
    and a read-back must match the HBM bytes.  async_stage: slots past the
    first two are issued on the device submitter while the upload sends."""
    import torch

    srv = native.Server({"port": 0, "retain_uploads": True})
    srv.start()
    try:
        t = torch.empty(size, dtype=torch.uint8, device="cuda:0")
        native.gpu_fill_pattern(0, t.data_ptr(), size, "splice/src", 0)
        for proto in ("grpc",):
            c = native.Client({"protocol": proto, "endpoint": srv.url})
            for i in range(3):  # the pinned staging ring is recycled between uploads
                name = f"splice/{size}_{i}"
                m = c.write_from_device(B, name, t.data_ptr(), size, 0, True, 16 << 20, slot, 8, async_stage)
                assert m["size"] == size and m["crc32c"] == m["gpu_crc32c"], m
                assert m["staged_whole"] and m["d2h_copies"] == -(-size // slot), m
                back = c.read_bytes(B, name)
                assert native.crc32c(back) == m["crc32c"]
                assert back == native.gpu_read_bytes(0, t.data_ptr(), size)
    finally:
        srv.stop()


def test_upload_ceiling_sends_gpu_staged_pages(native, gpu_available):
    """The write block's bound: the probe's sender sends a GpuByteSource's
    staging pages (HBM copied D2H into pinned slots) by reference, one
    object per read, and releases them only after the receiver has them."""
    import torch

    size = 64 << 20
    t = torch.empty(size, dtype=torch.uint8, device="cuda:0")
    native.gpu_fill_pattern(0, t.data_ptr(), size, "ceil/src", 0)
    base = {"mode": "tcp", "object_bytes": size, "reads": 4, "ring_bytes": 4 << 20}
    staged = native.loopback_ceiling({**base, "gpu_source_ptr": t.data_ptr(), "gpu_source_device": 0,
                                      "gpu_source_slot_bytes": 2 << 20, "gpu_source_slots": 4})
    thp = native.loopback_ceiling(base)
    assert staged["gbps"] > 1.0 and thp["gbps"] > 1.0, (staged, thp)
    assert staged["recv_cpu_s_per_gib"] > 0 and staged["send_cpu_s_per_gib"] > 0, staged


@pytest.mark.parametrize("poll_us", [0, 10])
def test_end_of_read_wait_modes(native, server, gpu_available, poll_us):
    """Both slot-event waits land and verify every byte: the runtime's
    blocking hipEventSynchronize (wait_poll_us 0) and the default poll of
    hipEventQuery with short sleeps; 1 MiB objects make every read end on a
    short wait, 8 MiB ones wrap the 2-slot ring (waits on the transport
    thread)."""
    import torch

    for size in (1 << 20, 8 << 20):
        server.add_synthetic(B, f"wait{poll_us}/s{size}_", "", 0, 1, size)
        c = native.Client({"protocol": "grpc", "endpoint": server.url})
        t = torch.empty(size, dtype=torch.uint8, device="cuda:0")
        sink = native.GpuSink({"device": 0, "ring_slot_bytes": 1 << 20, "ring_slots": 2, "wait_poll_us": poll_us})
        sink.set_external_destination(t.data_ptr(), size)
        for _ in range(3):
            r = c.read_gpu(B, f"wait{poll_us}/s{size}_0", sink)
            assert r["verified"] and not r["crc_mismatch"] and r["bytes"] == size, r
        torch.cuda.synchronize()
        bad, first = native.gpu_verify_pattern(0, t.data_ptr(), size, f"wait{poll_us}/s{size}_0", 0)
        assert bad == 0, (bad, first)
