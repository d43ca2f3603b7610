"""Pinned ring -> hipMemcpyAsync -> HBM landing with GPU CRC32C verification."""
import pytest

pytestmark = pytest.mark.gpu

B = "princer-working-dirs"
P = "princer_100M_files/file_"


def _protocols(native):
    from custom_go_client_benchmark_amd.ops import hbm

    return hbm.available_protocols()


@pytest.mark.parametrize("slot", [1 << 20, 3 << 20, 8 << 20])
def test_read_into_tensor_byte_exact(native, server, gpu_available, slot):
    import torch

    size = (13 << 20) + 777
    server.add_synthetic(B, P, "", 0, 1, size)
    for proto in _protocols(native):
        c = native.Client({"protocol": proto, "endpoint": server.url})
        t = torch.empty(size, dtype=torch.uint8, device="cuda:0")
        sink = native.GpuSink({"device": 0, "ring_slot_bytes": slot, "ring_slots": 3})
        sink.set_external_destination(t.data_ptr(), t.numel())
        for _ in range(2):  # reuse the sink across reads
            r = c.read_gpu(B, P + "0", sink)
            assert r["verified"] and not r["crc_mismatch"] and r["bytes"] == size, r
            bad, first = native.gpu_verify_pattern(0, t.data_ptr(), size, P + "0", 0)
            assert bad == 0, (proto, first)
        assert t[:4096].cpu().numpy().tobytes() == native.object_bytes(P + "0", 0, 4096)


def test_ring_landing_mode(native, server, gpu_available):
    server.add_synthetic(B, P, "", 0, 1, 20 << 20)
    c = native.Client({"protocol": "http", "endpoint": server.url})
    sink = native.GpuSink({"device": 0, "ring_slot_bytes": 2 << 20, "ring_slots": 4, "landing": "ring"})
    r = c.read_gpu(B, P + "0", sink)
    assert r["verified"] and r["bytes"] == 20 << 20
    assert sink.stats()["slots_submitted"] >= 10


def test_gpu_detects_corruption(native, server, gpu_available):
    server.add_synthetic(B, P, "", 0, 1, 6 << 20)
    server.set_faults({"corrupt_at": (3 << 20) + 5, "corrupt_count": 1})
    c = native.Client({"protocol": "http", "endpoint": server.url})
    sink = native.GpuSink({"device": 0, "ring_slot_bytes": 1 << 20, "ring_slots": 2})
    r = c.read_gpu(B, P + "0", sink)
    assert r["crc_mismatch"] and not r["verified"]


def test_gpu_resume_after_disconnect(native, server, gpu_available):
    server.add_synthetic(B, P, "", 0, 1, 9 << 20)
    server.set_faults({"disconnect_at": (4 << 20) + 100, "disconnect_count": 1})
    c = native.Client({"protocol": "http", "endpoint": server.url, "retry_initial_s": 0.001})
    sink = native.GpuSink({"device": 0, "ring_slot_bytes": 1 << 20, "ring_slots": 3})
    r = c.read_gpu(B, P + "0", sink)
    assert r["attempts"] == 2 and r["verified"]
    bad, _ = native.gpu_verify_pattern(0, r["device_ptr"], 9 << 20, P + "0", 0)
    assert bad == 0


def test_runner_gpu_sink(native, server, gpu_available):
    server.add_synthetic(B, P, "", 0, 4, 4 << 20)
    run = native.Runner({"protocol": "http", "endpoint": server.url, "bucket": B, "workers": 4,
                         "reads_per_worker": 3, "sink": "gpu", "ring_slot_bytes": 1 << 20})
    run.start()
    run.wait()
    s = run.summary()
    assert s["reads"] == 12 and s["errors"] == 0 and s["verified"] == 12, s
    assert s["gpu"]["objects_verified"] == 12


def test_hbm_helper_roundtrip(native, server, gpu_available):
    from custom_go_client_benchmark_amd.ops import hbm

    server.add_synthetic(B, P, "", 0, 1, 3 << 20)
    c = native.Client({"protocol": "http", "endpoint": server.url})
    t, r = hbm.read_object_to_tensor(c, B, P + "0")
    assert r["verified"] and hbm.crc32c(t) == server.object_info(B, P + "0")["crc32c"]


def test_grpc_chunks_verified_by_gpu_epilogue(native, server, gpu_available):
    size = (20 << 20) + 4321
    server.add_synthetic(B, P, "", 0, 1, size)
    c = native.Client({"protocol": "grpc", "endpoint": server.url})
    # sink-owned landing buffer: gRPC learns the size after the first message
    sink = native.GpuSink({"device": 0, "ring_slot_bytes": 8 << 20, "ring_slots": 3})
    for _ in range(2):
        r = c.read_gpu(B, P + "0", sink)
        assert r["verified"] and r["bytes"] == size, r
    st = sink.stats()
    assert st["chunks_verified_gpu"] >= 2 * 10 and st["objects_verified"] == 2
    bad, _ = native.gpu_verify_pattern(0, sink.device_ptr, size, P + "0", 0)
    assert bad == 0


def test_grpc_chunk_spanning_slots_folded_on_host(native, server, gpu_available):
    # 1 MiB slots < 2 MiB messages: every chunk spans two slots
    server.add_synthetic(B, P, "", 0, 1, 6 << 20)
    c = native.Client({"protocol": "grpc", "endpoint": server.url})
    sink = native.GpuSink({"device": 0, "ring_slot_bytes": 1 << 20, "ring_slots": 2})
    r = c.read_gpu(B, P + "0", sink)
    assert r["verified"]
    assert sink.stats()["chunks_verified_host"] == 3


def test_grpc_gpu_detects_corrupt_message(native, server, gpu_available):
    server.add_synthetic(B, P, "", 0, 1, 6 << 20)
    server.set_faults({"corrupt_at": (2 << 20) + 99, "corrupt_count": 1})
    c = native.Client({"protocol": "grpc", "endpoint": server.url})
    sink = native.GpuSink({"device": 0, "ring_slot_bytes": 4 << 20, "ring_slots": 2})
    r = c.read_gpu(B, P + "0", sink)
    assert r["crc_mismatch"] and "chunk crc32c mismatch" in r["detail"]


@pytest.mark.parametrize("proto", ["http", "grpc"])
@pytest.mark.parametrize("resumable", [True, False])
def test_write_path_hbm_to_server(native, server, gpu_available, proto, resumable):
    """Config 5: object generated in HBM (K3), D2H-staged through the pinned
    ring, uploaded; the server verifies the GPU-computed CRC32C."""
    import torch

    size = (9 << 20) + 77
    name = "upload/obj_3"
    t = torch.empty(size, dtype=torch.uint8, device="cuda:0")
    native.gpu_fill_pattern(0, t.data_ptr(), size, name, 0)
    c = native.Client({"protocol": proto, "endpoint": server.url})
    m = c.write_from_device(B, name, t.data_ptr(), size, 0, resumable, 4 << 20, 1 << 20, 3)
    assert m["size"] == size and m["crc32c"] == m["gpu_crc32c"] == native.crc32c(native.object_bytes(name, 0, size))
    assert m["d2h_copies"] >= 10
    if proto == "grpc":
        # every WriteObject message's ChecksummedData CRC came from the GPU
        # chunk CRCs (the server rejects a wrong one with DATA_LOSS)
        assert m["gpu_message_crcs"] == 10
    assert server.object_bytes(B, name, 0, size) == native.object_bytes(name, 0, size)


def test_upload_above_whole_ring_cap_copies(native, server, gpu_available):
    """An object larger than the whole-object staging cap (64 MiB) is
    staged through the bounded refilling ring and sent by copy, byte-exact
    (pinned staging must not grow with the object)."""
    import torch

    size = (80 << 20) + 4099
    name = "upload/big_0"
    t = torch.empty(size, dtype=torch.uint8, device="cuda:0")
    native.gpu_fill_pattern(0, t.data_ptr(), size, name, 0)
    c = native.Client({"protocol": "grpc", "endpoint": server.url})
    m = c.write_from_device(B, name, t.data_ptr(), size, 0, True, 16 << 20, 2 << 20, 4)
    assert not m["staged_whole"]
    assert m["size"] == size and m["crc32c"] == m["gpu_crc32c"] == native.crc32c(native.object_bytes(name, 0, size))
    assert server.object_bytes(B, name, 0, size) == native.object_bytes(name, 0, size)
    m = c.write_from_device(B, "upload/small_0", t.data_ptr(), 8 << 20, 0, True, 16 << 20, 2 << 20, 4)
    assert m["staged_whole"]


def test_cli_gpu_sink(native, gpu_available):
    import subprocess
    import sys as _sys
    import os as _os

    root = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
    r = subprocess.run([_os.path.join(root, "gcsbench"), "-worker", "2", "-read-call-per-worker", "3",
                        "-start-fake-server", "-fake-object-size", str(3 << 20), "-sink", "gpu",
                        "-client-protocol", "grpc"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert len(r.stdout.strip().splitlines()) == 6


@pytest.mark.parametrize("proto", ["http", "grpc"])
@pytest.mark.parametrize("slices,piece,taper", [(2, 0, 0), (4, 0, 0), (4, 4 << 20, 0), (3, 6 << 20, 0),
                                                (4, 8 << 20, 2 << 20)])
def test_sliced_read_lands_byte_exact_in_hbm(native, server, gpu_available, proto, slices, piece, taper):
    """piece > 0: dynamic pieces pulled by the streams, two GPU sinks per
    stream (one piece's copy tail overlapping the next piece's receive).
    taper > 0: guided schedule, pieces shrink toward the end of the object."""
    size = (40 << 20) + 4097
    server.add_synthetic(B, P, "", 0, 1, size)
    r = native.Runner({"protocol": proto, "endpoint": server.url, "bucket": B, "object_prefix": P, "workers": 1,
                       "reads_per_worker": 2, "sink": "gpu", "slices": slices, "ring_slot_bytes": 4 << 20,
                       "ring_slots": 4, "keep_records": False, "slice_piece_bytes": piece,
                       "slice_piece_min_bytes": taper})
    r.start()
    r.wait()
    s = r.summary()
    assert s["errors"] == 0, s["first_error"]
    assert s["verified"] == 2 and s["bytes"] == 2 * size
    assert s["gpu"]["chunks_verified_gpu"] + s["gpu"]["chunks_verified_host"] > 0 or proto == "http"
    bad, first = native.gpu_verify_pattern(0, r.landing_ptr(0), size, P + "0", 0)
    assert bad == 0, first


def test_sliced_gpu_read_detects_corruption(native, server, gpu_available):
    size = 32 << 20
    server.add_synthetic(B, P, "", 0, 1, size)
    server.set_faults({"corrupt_at": (27 << 20) + 3, "corrupt_count": 1})
    r = native.Runner({"protocol": "http", "endpoint": server.url, "bucket": B, "object_prefix": P, "workers": 1,
                       "reads_per_worker": 1, "sink": "gpu", "slices": 4, "keep_records": False})
    r.start()
    r.wait()
    s = r.summary()
    assert s["errors"] == 1 and "bad CRC" in s["first_error"]


@pytest.mark.parametrize("async_submit,blocking", [(True, True), (True, False), (False, False)])
def test_submit_modes_byte_exact(native, server, gpu_available, async_submit, blocking):
    """Every hand-off mode (submitter thread / inline, blocking / spinning
    event waits) lands the same bytes and verifies every chunk."""
    size = (21 << 20) + 99
    server.add_synthetic(B, P, "", 0, 1, size)
    for proto in ("http", "grpc"):
        r = native.Runner({"protocol": proto, "endpoint": server.url, "bucket": B, "object_prefix": P, "workers": 1,
                           "reads_per_worker": 3, "sink": "gpu", "slices": 3, "ring_slot_bytes": 2 << 20,
                           "ring_slots": 3, "keep_records": False, "async_submit": async_submit,
                           "blocking_sync": blocking})
        r.start()
        r.wait()
        s = r.summary()
        assert s["errors"] == 0 and s["verified"] == 3, s["first_error"]
        bad, first = native.gpu_verify_pattern(0, r.landing_ptr(0), size, P + "0", 0)
        assert bad == 0, (proto, first)


def test_async_submit_detects_corruption(native, server, gpu_available):
    server.add_synthetic(B, P, "", 0, 1, 6 << 20)
    server.set_faults({"corrupt_at": (3 << 20) + 5, "corrupt_count": 1})
    c = native.Client({"protocol": "grpc", "endpoint": server.url})
    sink = native.GpuSink({"device": 0, "ring_slot_bytes": 1 << 20, "ring_slots": 2, "async_submit": True})
    r = c.read_gpu(B, P + "0", sink)
    assert r["crc_mismatch"] and not r["verified"]


@pytest.mark.parametrize("slices", [1, 4])
@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_hbm_reader_api(native, server, gpu_available, slices, proto):
    from custom_go_client_benchmark_amd.ops import hbm

    size = (19 << 20) + 321
    server.add_synthetic(B, P, "", 0, 2, size)
    r = hbm.HbmReader(proto, server.url, device=0, slices=slices, slot_bytes=2 << 20, slots=3,
                      slice_min_bytes=2 << 20)
    t, res = r.read(B, P + "0")
    assert res["verified"] and res["bytes"] == size and t.numel() == size
    bad, first = native.gpu_verify_pattern(0, t.data_ptr(), size, P + "0", 0)
    assert bad == 0, first
    t2, res2 = r.read(B, P + "1", out=t)  # reuse the destination
    assert t2.data_ptr() == t.data_ptr() and res2["verified"]
    bad, first = native.gpu_verify_pattern(0, t.data_ptr(), size, P + "1", 0)
    assert bad == 0, first
    assert hbm.crc32c(t) == server.object_info(B, P + "1")["crc32c"]


def test_hbm_reader_destination_too_small(native, server, gpu_available):
    import torch
    from custom_go_client_benchmark_amd.ops import hbm

    server.add_synthetic(B, P, "", 0, 1, 8 << 20)
    r = hbm.HbmReader("http", server.url, slices=4, slice_min_bytes=1 << 20)
    with pytest.raises(native.StorageError, match="larger than the destination"):
        r.read(B, P + "0", out=torch.empty(1 << 20, dtype=torch.uint8, device="cuda:0"))


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_parallel_composite_upload_from_hbm(native, server, gpu_available, proto):
    import torch

    size = (24 << 20) + 4097
    name = "upload/pcu"
    t = torch.empty(size, dtype=torch.uint8, device="cuda:0")
    native.gpu_fill_pattern(0, t.data_ptr(), size, name, 0)
    w = native.SlicedWriter({"protocol": proto, "endpoint": server.url, "slices": 6, "slice_min_bytes": 1 << 20})
    m = w.write_from_device(B, name, t.data_ptr(), size, 0, True, 4 << 20, 2 << 20, 3)
    assert m["size"] == size and m["crc32c"] == native.gpu_crc32c(0, t.data_ptr(), size)
    c = native.Client({"protocol": proto, "endpoint": server.url})
    assert c.read_bytes(B, name) == native.object_bytes(name, 0, size)
    assert [o["name"] for o in c.list_all(B, "upload/")] == [name]


def test_write_combined_ring_byte_exact(native, server, gpu_available):
    """ring_wc (the config-3 list-read rings): write-combined pinned slots land
    the same bytes and CRC checks as cached ones, over several reads that
    reuse the sink, and corruption is still caught."""
    import torch

    size = (5 << 20) + 4099
    server.add_synthetic(B, P, "", 0, 1, size)
    for proto in _protocols(native):
        c = native.Client({"protocol": proto, "endpoint": server.url})
        t = torch.empty(size, dtype=torch.uint8, device="cuda:0")
        sink = native.GpuSink({"device": 0, "ring_slot_bytes": 1 << 20, "ring_slots": 2, "ring_wc": True})
        sink.set_external_destination(t.data_ptr(), t.numel())
        for _ in range(3):
            r = c.read_gpu(B, P + "0", sink)
            assert r["verified"] and not r["crc_mismatch"] and r["bytes"] == size, r
            bad, first = native.gpu_verify_pattern(0, t.data_ptr(), size, P + "0", 0)
            assert bad == 0, (proto, first)
    server.set_faults({"corrupt_at": (2 << 20) + 5, "corrupt_count": 1})
    c = native.Client({"protocol": "grpc", "endpoint": server.url})
    sink = native.GpuSink({"device": 0, "ring_slot_bytes": 1 << 20, "ring_slots": 2, "ring_wc": True})
    r = c.read_gpu(B, P + "0", sink)
    assert r["crc_mismatch"] and not r["verified"]
