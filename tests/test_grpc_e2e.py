"""Native gRPC transport against the synthetic server: reads, faults, resume."""
import os

import pytest

B = "princer-working-dirs"
P = "princer_100M_files/file_"


def _c(native, server, **kw):
    cfg = {"protocol": "grpc", "endpoint": server.url, "retry_initial_s": 0.001}
    cfg.update(kw)
    return native.Client(cfg)


def test_read_verified_chunks(native, server):
    server.add_synthetic(B, P, "", 0, 1, 9 * (1 << 20) + 11)
    r = _c(native, server).read(B, P + "0")
    assert r["bytes"] == 9 * (1 << 20) + 11 and r["verified"] and not r["crc_mismatch"]
    assert r["size"] == 9 * (1 << 20) + 11 and r["has_crc32c"]


def test_small_messages_many_frames(native):
    srv = native.Server({"port": 0, "grpc_chunk": 4096 + 3})
    srv.start()
    try:
        srv.add_synthetic(B, P, "", 0, 1, 100000)
        c = native.Client({"protocol": "grpc", "endpoint": srv.url})
        assert c.read_bytes(B, P + "0") == native.object_bytes(P + "0", 0, 100000)
        assert c.read(B, P + "0")["verified"]
    finally:
        srv.stop()


def test_send_threads_on_their_own_cpus(native):
    """ServerConfig::send_cpus pins the gRPC send threads apart from the
    endpoint's other threads (bench --mux-send isolate); reads stay exact."""
    cpus = sorted(os.sched_getaffinity(0))
    srv = native.Server({"port": 0, "cpus": cpus[:1], "send_cpus": cpus[-1:]})
    srv.start()
    try:
        srv.add_synthetic(B, P, "", 0, 1, 3 * (1 << 20) + 5)
        c = native.Client({"protocol": "grpc", "endpoint": srv.url})
        assert c.read_bytes(B, P + "0") == native.object_bytes(P + "0", 0, 3 * (1 << 20) + 5)
        assert c.read(B, P + "0")["verified"]
    finally:
        srv.stop()


@pytest.mark.parametrize("fill", [64, 512, 16384])
@pytest.mark.parametrize("frame", [0, (1 << 24) - 1])
def test_small_buffer_fills_stay_exact(native, server, fill, frame):
    """SocketOptions::fill_bytes caps what a frame-header fill takes of the
    payload behind it (16 KiB frames with the spanning receive, 16 MiB frames)."""
    server.add_synthetic(B, "fill/file_", "", 0, 3, 5 * (1 << 20) + 7)
    c = _c(native, server, fill_bytes=fill, h2_max_frame_size=frame)
    for i in range(3):
        assert c.read_bytes(B, f"fill/file_{i}") == native.object_bytes(f"fill/file_{i}", 0, 5 * (1 << 20) + 7)
        assert c.read(B, f"fill/file_{i}")["verified"]


def test_unavailable_is_retried(native, server):
    server.add_synthetic(B, P, "", 0, 1, 1 << 20)
    server.set_faults({"fail_next": 2, "fail_status": 503})
    r = _c(native, server).read(B, P + "0")
    assert r["attempts"] == 3 and r["verified"]


def test_resume_at_read_offset_after_disconnect(native, server):
    server.add_synthetic(B, P, "", 0, 1, 10 << 20)
    server.set_faults({"disconnect_at": (5 << 20) + 1, "disconnect_count": 1})
    c = _c(native, server)
    r = c.read(B, P + "0")
    assert r["attempts"] == 2 and r["bytes"] == 10 << 20 and r["verified"]
    assert c.read_bytes(B, P + "0") == native.object_bytes(P + "0", 0, 10 << 20)


def test_corruption_detected_per_message(native, server):
    server.add_synthetic(B, P, "", 0, 1, 6 << 20)
    server.set_faults({"corrupt_at": (4 << 20) + 17, "corrupt_count": 1})
    r = _c(native, server).read(B, P + "0")
    assert r["crc_mismatch"] and "mismatch" in r["detail"]


def test_not_found(native, server):
    with pytest.raises(native.StorageError, match="doesn't exist"):
        _c(native, server).read(B, "nope")


def test_many_workers_one_connection(native, server):
    server.add_synthetic(B, P, "", 0, 16, 2 << 20)
    run = native.Runner({"protocol": "grpc", "endpoint": server.url, "bucket": B, "workers": 16,
                         "reads_per_worker": 4, "grpc_conn_pool_size": 1})
    run.start()
    run.wait()
    s = run.summary()
    assert s["reads"] == 64 and s["errors"] == 0 and s["verified"] == 64
    assert server.stats()["connections"] == 1


def test_resumable_write_and_list(native, server):
    c = _c(native, server)
    data = os.urandom(5 * (1 << 20) + 3)
    m = c.write_bytes(B, "w/res", data, True)
    assert m["size"] == len(data) and m["crc32c"] == native.crc32c(data)
    assert c.read_bytes(B, "w/res") == data
    server.add_synthetic(B, "w/syn", "", 0, 3, 10)
    names = [o["name"] for o in c.list_all(B, "w/", 2)]
    assert names == ["w/res", "w/syn0", "w/syn1", "w/syn2"]


def test_auth_required(native):
    srv = native.Server({"port": 0, "require_auth": True})
    srv.start()
    try:
        srv.add_synthetic(B, P, "", 0, 1, 4096)
        c = native.Client({"protocol": "grpc", "endpoint": srv.url, "retry_max_attempts": 1})
        with pytest.raises(native.StorageError, match="code = 16"):
            c.read(B, P + "0")
        c = native.Client({"protocol": "grpc", "endpoint": srv.url, "auth": "static", "token": srv.issue_token()})
        assert c.read(B, P + "0")["verified"]
    finally:
        srv.stop()


def test_directpath_request_falls_back_to_cloudpath(native, server, monkeypatch):
    """Reference CreateGrpcClient (main.go:106-117) sets
    GOOGLE_CLOUD_ENABLE_DIRECT_PATH_XDS=true around client creation; without
    xDS/ALTS the library uses CloudPath.  The native client records the
    request and uses the configured endpoint."""
    monkeypatch.setenv("GOOGLE_CLOUD_ENABLE_DIRECT_PATH_XDS", "true")
    c = native.Client({"protocol": "grpc", "endpoint": server.url})
    assert c.stats()["path"].startswith("cloudpath (DirectPath requested")
    monkeypatch.delenv("GOOGLE_CLOUD_ENABLE_DIRECT_PATH_XDS")
    assert native.Client({"protocol": "grpc", "endpoint": server.url}).stats()["path"] == "cloudpath"


def test_cli_sets_directpath_env_only_during_client_creation(native):
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "custom_go_client_benchmark_amd", "-start-fake-server",
                        "-client-protocol", "grpc", "-worker", "1", "-read-call-per-worker", "1",
                        "-fake-object-size", "4096"], capture_output=True, text=True, timeout=120, cwd=root)
    assert r.returncode == 0, r.stderr
    assert "gRPC transport: cloudpath (DirectPath requested" in r.stderr
    assert os.environ.get("GOOGLE_CLOUD_ENABLE_DIRECT_PATH_XDS") is None


def test_connection_refused_is_a_clean_error(native):
    # dial failures must surface as StorageError (a failed dial once crashed
    # the connection's destructor, tests/test_tls.py found it)
    c = native.Client({"protocol": "grpc", "endpoint": "http://127.0.0.1:1", "retry_max_attempts": 2,
                       "retry_initial_s": 0.001})
    with pytest.raises(native.StorageError, match="refused"):
        c.read("b", "o")


@pytest.mark.parametrize("ranged", [True, False])
def test_stream_cut_after_last_byte_completes_without_refetch(native, server, ranged):
    """All requested bytes arrived but the connection died before the
    trailers: the retry must not ask again (read_limit=0 would mean "to the
    end of the object" and overrun a ranged/piece sink).  ADVICE r1."""
    size = 10 << 20
    server.add_synthetic(B, P, "", 0, 1, size)
    server.set_faults({"drop_trailers_count": 1})
    c = _c(native, server)
    off, lim = ((3 << 20) + 5, (2 << 20) + 7) if ranged else (0, -1)
    r = c.read(B, P + "0", offset=off, limit=lim)
    want = lim if ranged else size
    assert r["bytes"] == want and r["attempts"] == 2, r
    assert server.stats()["faults_injected"] == 1
    if not ranged:
        assert r["verified"]
    assert c.read_bytes(B, P + "0", off, want) == native.object_bytes(P + "0", off, want)


@pytest.mark.parametrize("proto", ["grpc", "http2"])
def test_deferred_host_crc_ring_wraps(native, server, proto):
    # a 64 KiB read chunk -> 256 KiB ring: a 3 MiB + 5 object wraps it many
    # times, so the reader thread has to help replay whenever it is full
    server.add_synthetic(B, P, "", 0, 1, (3 << 20) + 5)
    c = native.Client({"protocol": proto, "endpoint": server.url, "read_chunk": 64 << 10})
    r = c.read(B, P + "0", "deferred")
    assert r["bytes"] == (3 << 20) + 5 and r["verified"] and not r["crc_mismatch"]


@pytest.mark.parametrize("proto", ["grpc", "http2"])
def test_deferred_host_crc_detects_corruption(native, server, proto):
    server.add_synthetic(B, P, "", 0, 1, 6 << 20)
    server.set_faults({"corrupt_at": (4 << 20) + 17, "corrupt_count": 1})
    c = native.Client({"protocol": proto, "endpoint": server.url, "read_chunk": 256 << 10})
    r = c.read(B, P + "0", "deferred")
    assert r["crc_mismatch"] and "crc" in r["detail"].lower()


def test_deferred_host_crc_resume_after_disconnect(native, server):
    server.add_synthetic(B, P, "", 0, 1, 10 << 20)
    server.set_faults({"disconnect_at": (5 << 20) + 1, "disconnect_count": 1})
    r = _c(native, server).read(B, P + "0", "deferred")
    assert r["attempts"] == 2 and r["bytes"] == 10 << 20 and r["verified"] and not r["crc_mismatch"]
