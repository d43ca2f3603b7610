"""Synthetic server upload semantics: streamed resumable chunks, lazy MD5,
running CRC32C, and the non-retaining (verify + discard) benchmark mode."""
import hashlib
import os

import pytest

B = "princer-working-dirs"


@pytest.mark.parametrize("proto", ["http", "grpc"])
@pytest.mark.parametrize("resumable", [True, False])
def test_upload_md5_is_lazy_but_correct(native, server, proto, resumable):
    data = os.urandom(5 * (256 << 10) + 17)
    c = native.Client({"protocol": proto, "endpoint": server.url})
    m = c.write_bytes(B, "lazy/obj", data, resumable, 256 << 10)
    assert m["size"] == len(data) and m["crc32c"] == native.crc32c(data)
    # the upload response may omit MD5; metadata reads compute it
    assert c.stat(B, "lazy/obj")["md5"] == hashlib.md5(data).digest()
    assert c.read_bytes(B, "lazy/obj") == data


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_non_retaining_server_verifies_then_discards(native, proto):
    srv = native.Server({"port": 0, "retain_uploads": False})
    srv.start()
    try:
        data = os.urandom(3 * (256 << 10) + 5)
        c = native.Client({"protocol": proto, "endpoint": srv.url, "retry_max_attempts": 1})
        m = c.write_bytes(B, "gone/obj", data, True, 256 << 10)
        assert m["size"] == len(data) and m["crc32c"] == native.crc32c(data)
        st = c.stat(B, "gone/obj")
        assert st["size"] == len(data) and st["crc32c"] == native.crc32c(data)
        with pytest.raises(native.StorageError, match="not retained|412|code = 9"):
            c.read(B, "gone/obj")
    finally:
        srv.stop()


def test_resumable_chunk_with_overlap_is_deduplicated(native, server):
    """A client that resends already-persisted bytes (after a lost 308) must
    not duplicate them: the streamed chunk skips the overlap."""
    import http.client

    data = os.urandom(512 << 10)
    host, port = server.url.replace("http://", "").split(":")
    conn = http.client.HTTPConnection(host, int(port))
    conn.request("POST", f"/upload/storage/v1/b/{B}/o?uploadType=resumable&name=ovl",
                 body=b"{}", headers={"Content-Type": "application/json"})
    r = conn.getresponse()
    r.read()
    loc = r.getheader("Location")
    path = loc[loc.index("/upload/"):]
    half = 256 << 10
    conn.request("PUT", path, body=data[:half], headers={"Content-Range": f"bytes 0-{half - 1}/*"})
    r = conn.getresponse()
    r.read()
    assert r.status == 308 and r.getheader("Range") == f"bytes=0-{half - 1}"
    # resend from 128 KiB (overlapping 128 KiB) through the end
    start = 128 << 10
    conn.request("PUT", path, body=data[start:], headers={"Content-Range": f"bytes {start}-{len(data) - 1}/{len(data)}"})
    r = conn.getresponse()
    r.read()
    assert r.status == 200
    c = native.Client({"protocol": "http", "endpoint": server.url})
    assert c.read_bytes(B, "ovl") == data


def test_write_crc_worker_on_its_own_cpus(native):
    """ServerConfig::crc_cpus: the WriteObject CRC
    worker pinned apart from the connection thread still checks every
    message and the object lands exact."""
    cpus = sorted(os.sched_getaffinity(0))
    srv = native.Server({"port": 0, "cpus": cpus[:1], "crc_cpus": cpus[-1:], "send_cpus": cpus[-1:]})
    srv.start()
    try:
        data = os.urandom(6 * (1 << 20) + 3)
        c = native.Client({"protocol": "grpc", "endpoint": srv.url})
        m = c.write_bytes(B, "split/obj", data, True, 2 << 20)
        assert m["size"] == len(data) and m["crc32c"] == native.crc32c(data)
        assert c.read_bytes(B, "split/obj") == data
    finally:
        srv.stop()


def test_upload_phases_are_ordered(native, server):
    """UploadPhases (the write block's phases_ms): a resumable gRPC upload's
    start RPC answers before the first content byte is sent, the last byte
    after the first, and the final response after the last byte."""
    c = native.Client({"protocol": "grpc", "endpoint": server.url})
    data = bytes(range(256)) * ((6 << 20) // 256)
    m = c.write_bytes(B, "phases/obj", data, True, 16 << 20)
    assert m["size"] == len(data)
    p = c.last_upload()
    assert 0 < p["start_rpc_ms"] <= p["first_send_ms"] <= p["last_send_ms"] <= p["response_ms"], p
