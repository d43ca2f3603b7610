"""-read-timeout: an attempt with no byte for the limit fails retryably and the
read resumes; slow-but-moving and idle multiplexed connections are left alone.

The reference has no request timeout (http.Client Timeout 0, main.go:94;
SURVEY.md §5 "Optional --read-timeout"): 0 stays the default.
"""
import time

import pytest

B = "princer-working-dirs"
P = "princer_100M_files/file_"
PROTOS = ["http", "http2", "grpc"]


def _client(native, server, proto, **kw):
    cfg = {"protocol": proto, "endpoint": server.url, "retry_initial_s": 0.001}
    cfg.update(kw)
    return native.Client(cfg)


@pytest.mark.parametrize("proto", PROTOS)
def test_stalled_response_times_out(native, server, proto):
    server.add_synthetic(B, P, "", 0, 1, 1 << 20)
    server.set_faults({"latency_ms": 600})
    c = _client(native, server, proto, io_timeout_ms=100, retry_max_attempts=2)
    t0 = time.perf_counter()
    with pytest.raises(Exception, match="timeout"):
        c.read(B, P + "0")
    # two attempts of 100-200 ms of silence each, not the server's 2 x 600 ms
    assert time.perf_counter() - t0 < 1.0


@pytest.mark.parametrize("proto", PROTOS)
def test_timeout_then_resume_succeeds(native, server, proto):
    server.add_synthetic(B, P, "", 0, 1, 3 << 20)
    server.set_faults({"latency_ms": 400})
    c = _client(native, server, proto, io_timeout_ms=100, retry_max_attempts=0)
    import threading

    # the endpoint recovers while the client is retrying
    threading.Timer(0.25, lambda: server.set_faults({"latency_ms": 0})).start()
    r = c.read(B, P + "0")
    assert r["bytes"] == 3 << 20 and r["verified"] and r["attempts"] >= 2


@pytest.mark.parametrize("proto", PROTOS)
def test_slow_but_moving_read_is_not_cut(native, proto):
    # gRPC throttles per ReadObjectResponse: 128 KiB messages keep the
    # silences (~8 ms) as short as the media pieces' (10 ms)
    srv = native.Server({"port": 0, "grpc_chunk": 128 << 10})
    srv.start()
    try:
        srv.add_synthetic(B, P, "", 0, 1, 2 << 20)
        srv.set_faults({"throttle_bps": 16 << 20})  # ~125 ms for the object
        c = _client(native, srv, proto, io_timeout_ms=60, retry_max_attempts=1)
        r = c.read(B, P + "0")
        assert r["bytes"] == 2 << 20 and r["verified"] and r["attempts"] == 1
    finally:
        srv.stop()


@pytest.mark.parametrize("proto", ["grpc", "http2"])
def test_idle_multiplexed_connection_survives(native, server, proto):
    # the limit is per stream: an idle shared connection (no stream open)
    # keeps its reader thread, so the next read needs no new dial
    server.add_synthetic(B, P, "", 0, 1, 1 << 20)
    c = _client(native, server, proto, io_timeout_ms=50, retry_max_attempts=1)
    assert c.read(B, P + "0")["verified"]
    time.sleep(0.3)
    r = c.read(B, P + "0")
    assert r["verified"] and r["attempts"] == 1
    if proto == "grpc":  # (http2 mode sends its metadata requests without keep-alive)
        assert server.stats()["connections"] == 1


def test_cli_flag_parses():
    from custom_go_client_benchmark_amd.cli import build_flags

    fs = build_flags().parse(["-read-timeout", "1.5s"])
    assert fs.get("read-timeout") == pytest.approx(1.5)
    assert build_flags().parse([]).get("read-timeout") == 0.0


@pytest.mark.parametrize("proto", PROTOS)
def test_stall_mid_body_resumes(native, server, proto):
    # the endpoint goes silent 1 MiB into the body (inside gRPC's first 2 MiB
    # message, before its object_checksums field): the attempt times out and
    # the read resumes at the delivered offset
    server.add_synthetic(B, P, "", 0, 1, 3 << 20)
    server.set_faults({"stall_at": 1 << 20, "stall_ms": 400, "stall_count": 1})
    c = _client(native, server, proto, io_timeout_ms=100, retry_max_attempts=3)
    r = c.read(B, P + "0")
    assert r["bytes"] == 3 << 20 and r["verified"] and r["attempts"] == 2
    assert server.stats()["faults_injected"] == 1


@pytest.mark.parametrize("proto", PROTOS)
def test_corruption_before_a_timeout_is_caught_after_resume(native, server, proto):
    # a byte corrupted in the part the first attempt delivered, then a stall:
    # the resumed read must still check the whole-object CRC32C (gRPC used to
    # drop it when the first attempt never saw its checksums field)
    server.add_synthetic(B, P, "", 0, 1, 3 << 20)
    server.set_faults({"corrupt_at": 4242, "corrupt_count": 1, "stall_at": 1 << 20, "stall_ms": 400,
                       "stall_count": 1})
    c = _client(native, server, proto, io_timeout_ms=100, retry_max_attempts=3)
    r = c.read(B, P + "0")
    assert r["attempts"] == 2
    assert r["crc_mismatch"] and not r["verified"]


@pytest.mark.parametrize("proto", ["grpc", "http2"])
def test_one_stalled_stream_does_not_fail_its_neighbours(native, server, proto):
    # gRPC pool 1 / HTTP/2 multiplex every read on one connection: when one
    # stream times out, only that stream is cancelled (RST_STREAM) -- the
    # reads sharing the connection keep going on it, none is retried
    import threading

    server.add_synthetic(B, P, "", 0, 1, 3 << 20)
    server.add_synthetic(B, "small/file_", "", 0, 1, 256 << 10)
    # (the neighbours keep the connection busy, which the stalled stream's
    # idle check tolerates for 3 windows: 100 ms x (1 + 3) < the 800 ms stall)
    server.set_faults({"stall_at": 1 << 20, "stall_ms": 800, "stall_count": 1})
    c = _client(native, server, proto, io_timeout_ms=100, retry_max_attempts=3)
    assert c.read(B, "small/file_0")["verified"]  # the connection is up
    stalled = []
    t = threading.Thread(target=lambda: stalled.append(c.read(B, P + "0")))
    t.start()
    neighbours = []
    t_end = time.perf_counter() + 1.0
    while time.perf_counter() < t_end:
        neighbours.append(c.read(B, "small/file_0"))
    t.join()
    r = stalled[0]
    assert r["bytes"] == 3 << 20 and r["verified"] and r["attempts"] == 2
    assert server.stats()["faults_injected"] == 1
    assert len(neighbours) > 5
    assert all(x["verified"] and x["attempts"] == 1 for x in neighbours), [x["attempts"] for x in neighbours]
    if proto == "grpc":
        assert server.stats()["connections"] == 1  # the shared connection was never closed


def test_grpc_upload_finalize_has_its_own_bound(native, server):
    """-read-timeout covers an upload's final response with a longer bound
    of its own (10x): a finalize slower than -read-timeout still succeeds;
    one past the bound fails at once, NOT retried (a re-sent upload could
    duplicate a committed generation)."""
    data = bytes(range(256)) * 4096
    c = _client(native, server, "grpc", io_timeout_ms=100, retry_max_attempts=3)
    server.set_faults({"finalize_delay_ms": 400})
    m = c.write_bytes(B, "upload/fin_ok", data)
    assert m["size"] == len(data)
    server.set_faults({"finalize_delay_ms": 2500})
    t0 = time.perf_counter()
    with pytest.raises(Exception, match="final response"):
        c.write_bytes(B, "upload/fin_slow", data)
    # one attempt cut at 1-2 s of silence (10 x 100 ms), no retries
    assert time.perf_counter() - t0 < 2.4
    server.set_faults({"finalize_delay_ms": 0})
