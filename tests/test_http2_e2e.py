"""`-client-protocol http2`: media GETs as HTTP/2 streams (h2c with prior
knowledge, all GETs of a client multiplexed on one connection), the
reference's HTTP/2 transport mode (/root/reference/main.go:74-81), against the
synthetic server's HTTP/2 front end (plain GET/HEAD on the gRPC port)."""
import threading

import pytest

B = "princer-working-dirs"
P = "princer_100M_files/file_"


def h2client(native, server, **kw):
    return native.Client({"protocol": "http2", "endpoint": server.url, "retry_initial_s": 0.001, **kw})


@pytest.mark.parametrize("api", ["xml", "json"])
def test_h2_full_read_verified(native, server, api):
    server.add_synthetic(B, P, "", 0, 2, 3 * (1 << 20) + 17)
    before = server.stats()
    c = h2client(native, server, http_api=api)
    r = c.read(B, P + "1")
    assert r["bytes"] == 3 * (1 << 20) + 17
    assert r["verified"] and not r["crc_mismatch"]
    assert r["crc32c"] == server.object_info(B, P + "1")["crc32c"]
    st = c.stats()
    assert st["transport"] == "http2" and st["dials"] == 1
    after = server.stats()
    # served by the HTTP/2 front end: an HTTP request, no gRPC call
    assert after["http_requests"] == before["http_requests"] + 1
    assert after["grpc_calls"] == before["grpc_calls"]


def test_h2_range_bytes_exact(native, server):
    server.add_synthetic(B, P, "", 0, 1, 1 << 20)
    c = h2client(native, server)
    assert c.read_bytes(B, P + "0", 12345, 1000) == server.object_bytes(B, P + "0", 12345, 1000)
    assert c.read_bytes(B, P + "0") == server.object_bytes(B, P + "0", 0, 1 << 20)


def test_h2_streams_share_one_connection(native, server):
    server.add_synthetic(B, P, "", 0, 8, 1 << 20)
    c = h2client(native, server)
    out, errs = [], []

    def rd(i):
        try:
            out.append(c.read(B, P + str(i)))
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=rd, args=(i,)) for i in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs and len(out) == 8 and all(r["verified"] for r in out)
    assert c.stats()["dials"] == 1


def test_h2_not_found_and_retry_on_503(native, server):
    c = h2client(native, server)
    with pytest.raises(native.StorageError, match="doesn't exist"):
        c.read(B, "nope")
    server.add_synthetic(B, P, "", 0, 1, 1 << 20)
    server.set_faults({"fail_next": 2, "fail_status": 503})
    r = c.read(B, P + "0")
    assert r["attempts"] == 3 and r["verified"]


def test_h2_resume_after_disconnect(native, server):
    server.add_synthetic(B, P, "", 0, 1, 24 << 20)
    server.set_faults({"disconnect_at": 9 << 20, "disconnect_count": 1})
    c = h2client(native, server)
    r = c.read(B, P + "0")
    assert r["attempts"] == 2 and r["bytes"] == 24 << 20 and r["verified"]
    assert c.stats()["dials"] == 2  # the cut connection is replaced


def test_h2_corruption_detected(native, server):
    server.add_synthetic(B, P, "", 0, 1, 1 << 20)
    server.set_faults({"corrupt_at": 4242, "corrupt_count": 1})
    r = h2client(native, server).read(B, P + "0")
    assert r["crc_mismatch"] and "bad CRC" in r["detail"]


def test_h2_auth_required(native):
    srv = native.Server({"port": 0, "require_auth": True})
    srv.start()
    try:
        srv.add_synthetic(B, P, "", 0, 1, 4096)
        c = native.Client({"protocol": "http2", "endpoint": srv.url, "retry_max_attempts": 1})
        with pytest.raises(native.StorageError, match="401"):
            c.read(B, P + "0")
        c = native.Client({"protocol": "http2", "endpoint": srv.url, "auth": "static", "token": srv.issue_token()})
        assert c.read(B, P + "0")["verified"]
    finally:
        srv.stop()


def test_h2_sliced_read(native, server):
    server.add_synthetic(B, P, "", 0, 1, 9 * (1 << 20) + 5)
    run = native.Runner({"protocol": "http2", "endpoint": server.url, "bucket": B, "object_prefix": P, "workers": 1,
                         "reads_per_worker": 2, "sink": "discard", "slices": 4, "slice_min_bytes": 1 << 20,
                         "keep_records": False})
    run.start()
    run.wait()
    s = run.summary()
    assert s["errors"] == 0 and s["reads"] == 2 and s["verified"] == 2


def test_cli_http2_latency_lines(native, server, tmp_path):
    import subprocess
    import sys
    server.add_synthetic(B, P, "", 0, 2, 1 << 20)
    r = subprocess.run([sys.executable, "-m", "custom_go_client_benchmark_amd.cli", "-client-protocol", "http2",
                        "-endpoint", server.url, "-worker", "2", "-read-call-per-worker", "3"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.endswith("ms")]
    assert len(lines) == 6
