"""Connection ring (GpuSinkConfig::conn_ring, profiles/r4_bigring): every
worker's gRPC stream on ONE multiplexed connection lands through one shared
pinned ring -- segments of different streams side by side in a slot, one H2D
per segment to its own object's HBM, one CRC launch per slot part, results
collected per owner, chunks and objects folded on the host.  Compared
against the bytes the endpoint serves (gpu_verify_pattern) and the
endpoint's CRC32C values."""
import pytest

pytestmark = pytest.mark.gpu

B = "bkt"
P = "ring/obj_"


def _runner(native, server, workers, reads, slot_bytes, slots, proto="grpc", **kw):
    cfg = {"protocol": proto, "endpoint": server.url, "bucket": B, "object_prefix": P, "workers": workers,
           "reads_per_worker": reads, "sink": "gpu", "grpc_conn_pool_size": 1, "keep_records": False,
           "conn_ring_slot_bytes": slot_bytes, "conn_ring_slots": slots, "retry_initial_s": 0.01}
    cfg.update(kw)
    return native.Runner(cfg)


FRAMES = {"ref": {"h2_max_frame_size": 0, "h2_window": 16 << 20},
          "ref_nospan": {"h2_max_frame_size": 0, "h2_window": 16 << 20, "h2_span_max_frame": 0},
          "large": {"h2_max_frame_size": (1 << 24) - 1, "h2_window": 0x7FFFFFFF}}


@pytest.mark.parametrize("frames", ["ref", "ref_nospan", "large"])
@pytest.mark.parametrize("proto,slot_bytes,slots", [("grpc", 1 << 20, 4), ("grpc", 1 << 20, 2), ("grpc", 64 << 10, 3),
                                                    ("http2", 1 << 20, 4)])
def test_conn_ring_many_streams_byte_exact(native, server, gpu_available, proto, slot_bytes, slots, frames):
    """12 streams on one connection; frames: the HTTP/2 receive settings
    (the reference's 16 KiB frames with and without the multi-frame spanning
    receive, or 16 MiB frames).  With 16 KiB frames of 12 streams the ring
    wraps between two frames of one stream (the slot fill generation of
    GpuSink::ring_extends)."""
    workers = 12
    sizes = [(3 << 20) + 4099 * i + 77 for i in range(workers)]
    for i, n in enumerate(sizes):
        server.add_synthetic(B, P, "", i, 1, n)
    r = _runner(native, server, workers, 3, slot_bytes, slots, proto=proto, **FRAMES[frames])
    r.start()
    r.wait()
    s = r.summary()
    assert s["errors"] == 0 and s["verified"] == 3 * workers, s["first_error"]
    st = r.conn_ring_stats()
    assert st is not None and st["segments"] >= 3 * workers and st["submissions"] > 0
    for w, n in enumerate(sizes):
        bad, first = native.gpu_verify_pattern(0, r.landing_ptr(w), n, P + str(w), 0)
        assert bad == 0, (w, first)


def test_conn_ring_off_keeps_per_worker_rings(native, server, gpu_available):
    server.add_synthetic(B, P, "", 0, 4, (2 << 20) + 5)
    r = _runner(native, server, 4, 2, 1 << 20, 8, conn_ring=False)
    r.start()
    r.wait()
    s = r.summary()
    assert s["errors"] == 0 and s["verified"] == 8 and r.conn_ring_stats() is None


def test_conn_ring_detects_corruption(native, server, gpu_available):
    """One stream's corrupted byte fails that read's check (chunk and object
    CRC on the host fold); the other streams sharing its slots verify."""
    workers = 6
    server.add_synthetic(B, P, "", 0, workers, 5 << 20)
    r = _runner(native, server, workers, 1, 1 << 20, 4, stop_on_error=False)
    server.set_faults({"corrupt_at": (2 << 20) + 11, "corrupt_count": 1})
    r.start()
    r.wait()
    s = r.summary()
    assert s["errors"] == 1 and s["verified"] == workers - 1
    assert "crc" in s["first_error"].lower()


def test_conn_ring_resume_after_disconnect(native, server, gpu_available):
    """A connection cut mid-stream: every stream on it resumes at its
    delivered offset on a new connection; the bytes already in the ring's
    slots (from the old connection's reader) land, and every object lands
    byte-exact."""
    workers = 4
    size = (6 << 20) + 321
    server.add_synthetic(B, P, "", 0, workers, size)
    r = _runner(native, server, workers, 2, 1 << 20, 4)
    server.set_faults({"disconnect_at": (3 << 20) + 17, "disconnect_count": 1})
    r.start()
    r.wait()
    s = r.summary()
    assert s["errors"] == 0 and s["verified"] == 2 * workers, s["first_error"]
    for w in range(workers):
        bad, first = native.gpu_verify_pattern(0, r.landing_ptr(w), size, P + str(w), 0)
        assert bad == 0, (w, first)


@pytest.mark.parametrize("proto", ["grpc", "http2"])
def test_conn_ring_stalled_stream_resumes(native, server, gpu_available, proto):
    """One stream goes silent mid-body past the read timeout: it is cancelled
    alone (its segments already in the ring still land), resumes at its
    delivered offset, and every stream sharing the ring lands byte-exact."""
    workers = 6
    size = (3 << 20) + 999
    server.add_synthetic(B, P, "", 0, workers, size)
    server.set_faults({"stall_at": 1 << 20, "stall_ms": 800, "stall_count": 1})
    r = _runner(native, server, workers, 2, 1 << 20, 4, proto=proto, io_timeout_ms=100, retry_max_attempts=3)
    r.start()
    r.wait()
    s = r.summary()
    assert s["errors"] == 0 and s["verified"] == 2 * workers, s["first_error"]
    assert s["retries"] >= 1
    for w in range(workers):
        bad, first = native.gpu_verify_pattern(0, r.landing_ptr(w), size, P + str(w), 0)
        assert bad == 0, (w, first)
