"""HTTP transport against the synthetic GCS server (XML + JSON APIs)."""
import os

import pytest

B = "princer-working-dirs"
P = "princer_100M_files/file_"


@pytest.mark.parametrize("api", ["xml", "json"])
def test_full_read_verified(native, server, api):
    server.add_synthetic(B, P, "", 0, 2, 3 * (1 << 20) + 17)
    c = native.Client({"protocol": "http", "endpoint": server.url, "http_api": api})
    r = c.read(B, P + "1")
    assert r["bytes"] == 3 * (1 << 20) + 17
    assert r["verified"] and not r["crc_mismatch"]
    assert r["crc32c"] == server.object_info(B, P + "1")["crc32c"]


def test_range_read_bytes(native, server):
    server.add_synthetic(B, P, "", 0, 1, 1 << 20)
    c = native.Client({"protocol": "http", "endpoint": server.url})
    got = c.read_bytes(B, P + "0", 12345, 1000)
    assert got == native.object_bytes(P + "0", 12345, 1000)
    assert got == server.object_bytes(B, P + "0", 12345, 1000)


def test_not_found_is_not_retried(native, server):
    c = native.Client({"protocol": "http", "endpoint": server.url, "retry_initial_s": 0.01})
    with pytest.raises(native.StorageError, match="doesn't exist"):
        c.read(B, "nope")


def test_retry_on_503_then_success(native, server):
    server.add_synthetic(B, P, "", 0, 1, 1 << 20)
    server.set_faults({"fail_next": 3, "fail_status": 503})
    c = native.Client({"protocol": "http", "endpoint": server.url, "retry_initial_s": 0.001})
    r = c.read(B, P + "0")
    assert r["attempts"] == 4 and r["verified"]


def test_resume_after_disconnect(native, server):
    server.add_synthetic(B, P, "", 0, 1, 8 << 20)
    server.set_faults({"disconnect_at": 3 << 20, "disconnect_count": 2})
    c = native.Client({"protocol": "http", "endpoint": server.url, "retry_initial_s": 0.001})
    r = c.read(B, P + "0")
    # the first attempt is cut at 3 MiB; the resumed Range request starts at
    # exactly that offset and is cut again (count 2); the third one finishes
    assert r["attempts"] == 3
    assert r["bytes"] == 8 << 20 and r["verified"]


def test_corruption_detected(native, server):
    server.add_synthetic(B, P, "", 0, 1, 1 << 20)
    server.set_faults({"corrupt_at": 4242, "corrupt_count": 1})
    c = native.Client({"protocol": "http", "endpoint": server.url})
    r = c.read(B, P + "0")
    assert r["crc_mismatch"] and "bad CRC" in r["detail"]


def test_list_stat_and_pagination(native, server):
    server.add_synthetic(B, "dir/obj_", "", 0, 25, 1024)
    c = native.Client({"protocol": "http", "endpoint": server.url})
    page = c.list(B, "dir/", 10)
    assert len(page["objects"]) == 10 and page["next_page_token"]
    names = [o["name"] for o in c.list_all(B, "dir/", 7)]
    assert names == sorted(f"dir/obj_{i}" for i in range(25))
    m = c.stat(B, "dir/obj_3")
    assert m["size"] == 1024 and m["has_crc32c"] and len(m["md5"]) == 16


def test_list_delimiter(native, server):
    for n in ["a/1", "a/2", "b/1", "top"]:
        server.add_object(B, n, b"x")
    c = native.Client({"protocol": "http", "endpoint": server.url})
    r = c.list(B, "", 100, "", "/")
    assert sorted(r["prefixes"]) == ["a/", "b/"]
    assert [o["name"] for o in r["objects"]] == ["top"]


@pytest.mark.parametrize("resumable", [True, False])
def test_upload_roundtrip(native, server, resumable):
    data = os.urandom(3 * (256 << 10) + 99)
    c = native.Client({"protocol": "http", "endpoint": server.url})
    m = c.write_bytes(B, "up/obj", data, resumable, 256 << 10)
    assert m["size"] == len(data) and m["crc32c"] == native.crc32c(data)
    assert c.read_bytes(B, "up/obj") == data


def test_user_agent_and_auth_required(native):
    srv = native.Server({"port": 0, "require_auth": True})
    srv.start()
    try:
        srv.add_synthetic(B, P, "", 0, 1, 4096)
        c = native.Client({"protocol": "http", "endpoint": srv.url, "retry_max_attempts": 1})
        with pytest.raises(native.StorageError, match="401"):
            c.read(B, P + "0")
        tok = srv.issue_token()
        c = native.Client({"protocol": "http", "endpoint": srv.url, "auth": "static", "token": tok})
        assert c.read(B, P + "0")["verified"]
    finally:
        srv.stop()


def test_generation_pinned_media_reads(native, server):
    """Resumed and sliced reads pin the object generation (?generation=N /
    ReadObjectRequest.generation); a stale generation is a 404, not bytes of
    another object version."""
    import http.client

    server.add_synthetic(B, P, "", 0, 1, 4096)
    gen = server.object_info(B, P + "0")["generation"]
    host, port = server.url.replace("http://", "").split(":")
    for q, want in ((f"?generation={gen}", 200), (f"?generation={gen + 1}", 404)):
        conn = http.client.HTTPConnection(host, int(port))
        conn.request("GET", f"/{B}/{P}0{q}")
        r = conn.getresponse()
        r.read()
        assert r.status == want, q
