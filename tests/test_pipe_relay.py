"""gRPC reads relayed through per-read pipes (csrc/storage/pipe_relay.h).

The connection's reader splice()s each payload into the read's pipe and the
read's own thread copies it into the sink: every read must land the same
bytes, checks and resume points as the direct path (tests/test_grpc_e2e.py).
"""
import pytest

B = "princer-working-dirs"
P = "princer_100M_files/file_"


def _c(native, server, **kw):
    cfg = {"protocol": "grpc", "endpoint": server.url, "retry_initial_s": 0.001, "splice_recv": 1}
    cfg.update(kw)
    return native.Client(cfg)


def _relayed(native, before):
    after = native.pipe_relay_stats()
    return after["relays"] - before["relays"], after


def test_relayed_read_is_verified_and_exact(native, server):
    size = 9 * (1 << 20) + 11
    server.add_synthetic(B, P, "", 0, 1, size)
    s0 = native.pipe_relay_stats()
    c = _c(native, server)
    r = c.read(B, P + "0")
    assert r["bytes"] == size and r["verified"] and not r["crc_mismatch"]
    assert c.read_bytes(B, P + "0") == native.object_bytes(P + "0", 0, size)
    n, s1 = _relayed(native, s0)
    assert n == 2 and s1["spliced_bytes"] > s0["spliced_bytes"]


@pytest.mark.parametrize("sink", ["discard", "deferred"])
def test_relayed_small_messages(native, sink):
    # 4 KiB + 3 messages: every payload piece is short and unaligned
    srv = native.Server({"port": 0, "grpc_chunk": 4096 + 3})
    srv.start()
    try:
        srv.add_synthetic(B, P, "", 0, 1, 100000)
        c = native.Client({"protocol": "grpc", "endpoint": srv.url, "splice_recv": 1})
        assert c.read_bytes(B, P + "0") == native.object_bytes(P + "0", 0, 100000)
        assert c.read(B, P + "0", sink)["verified"]
    finally:
        srv.stop()


def test_relayed_resume_after_disconnect(native, server):
    server.add_synthetic(B, P, "", 0, 1, 10 << 20)
    server.set_faults({"disconnect_at": (5 << 20) + 1, "disconnect_count": 1})
    c = _c(native, server)
    r = c.read(B, P + "0")
    assert r["attempts"] == 2 and r["bytes"] == 10 << 20 and r["verified"]
    assert c.read_bytes(B, P + "0") == native.object_bytes(P + "0", 0, 10 << 20)


@pytest.mark.parametrize("sink", ["discard", "deferred"])
def test_relayed_corruption_detected(native, server, sink):
    server.add_synthetic(B, P, "", 0, 1, 6 << 20)
    server.set_faults({"corrupt_at": (4 << 20) + 17, "corrupt_count": 1})
    r = _c(native, server).read(B, P + "0", sink)
    assert r["crc_mismatch"] and "mismatch" in r["detail"].lower()


@pytest.mark.parametrize("ranged", [True, False])
def test_relayed_stream_cut_after_last_byte(native, server, ranged):
    size = 10 << 20
    server.add_synthetic(B, P, "", 0, 1, size)
    server.set_faults({"drop_trailers_count": 1})
    c = _c(native, server)
    off, lim = ((3 << 20) + 5, (2 << 20) + 7) if ranged else (0, -1)
    r = c.read(B, P + "0", offset=off, limit=lim)
    want = lim if ranged else size
    assert r["bytes"] == want and r["attempts"] == 2, r
    assert c.read_bytes(B, P + "0", off, want) == native.object_bytes(P + "0", off, want)


def test_runner_relays_when_streams_share_a_connection(native, server):
    """16 workers on one connection relay every read; the pipes go back to
    the pool clean (the next reads reuse them)."""
    server.add_synthetic(B, P, "", 0, 16, 2 << 20)
    s0 = native.pipe_relay_stats()
    run = native.Runner({"protocol": "grpc", "endpoint": server.url, "bucket": B, "workers": 16,
                         "reads_per_worker": 4, "grpc_conn_pool_size": 1, "splice_recv": 1})
    run.start()
    run.wait()
    s = run.summary()
    assert s["reads"] == 64 and s["errors"] == 0 and s["verified"] == 64
    n, s1 = _relayed(native, s0)
    assert n == 64
    assert s1["pipes"] - s0["pipes"] <= 16  # reused, not one per read


@pytest.mark.parametrize("proto", ["grpc", "http2"])
def test_relayed_many_streams_one_connection(native, server, proto):
    server.add_synthetic(B, P, "", 0, 8, (3 << 20) + 5)
    s0 = native.pipe_relay_stats()
    run = native.Runner({"protocol": proto, "endpoint": server.url, "bucket": B, "workers": 8,
                         "reads_per_worker": 3, "grpc_conn_pool_size": 1, "splice_recv": 1})
    run.start()
    run.wait()
    s = run.summary()
    assert s["errors"] == 0 and s["verified"] == 24
    assert _relayed(native, s0)[0] == 24


def test_runner_default_keeps_direct_path(native, server):
    server.add_synthetic(B, P, "", 0, 8, 1 << 20)
    s0 = native.pipe_relay_stats()
    run = native.Runner({"protocol": "grpc", "endpoint": server.url, "bucket": B, "workers": 8,
                         "reads_per_worker": 2, "grpc_conn_pool_size": 1})
    run.start()
    run.wait()
    assert run.summary()["verified"] == 16
    assert _relayed(native, s0)[0] == 0


def test_relayed_concurrent_reads_with_read_timeout(native, server):
    """A stalled stream is cancelled alone; its relay is settled and the
    neighbours' relayed reads complete."""
    server.add_synthetic(B, P, "", 0, 8, 4 << 20)
    run = native.Runner({"protocol": "grpc", "endpoint": server.url, "bucket": B, "workers": 8,
                         "reads_per_worker": 3, "grpc_conn_pool_size": 1, "io_timeout_ms": 5000,
                         "splice_recv": 1})
    run.start()
    run.wait()
    s = run.summary()
    assert s["errors"] == 0 and s["verified"] == 24
