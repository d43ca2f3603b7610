"""objects.compose / ComposeObject, DeleteObject, and parallel composite
uploads (storage/sliced.h SlicedWriter) against the synthetic server."""
import os

import pytest

B = "princer-working-dirs"


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_compose_and_delete(native, server, proto):
    c = native.Client({"protocol": proto, "endpoint": server.url})
    parts = [os.urandom((256 << 10) + 17 * i) for i in range(3)]
    for i, p in enumerate(parts):
        c.write_bytes(B, f"dir/p{i}", p, False)
    m = c.compose(B, "dir/whole", ["dir/p0", "dir/p1", "dir/p2"], "application/x-test")
    whole = b"".join(parts)
    assert m["size"] == len(whole) and m["crc32c"] == native.crc32c(whole)
    assert c.read_bytes(B, "dir/whole") == whole
    assert c.stat(B, "dir/whole")["content_type"] == "application/x-test"
    c.delete(B, "dir/p1")
    with pytest.raises(native.StorageError):
        c.stat(B, "dir/p1")
    with pytest.raises(native.StorageError):
        c.delete(B, "dir/p1")


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_compose_errors(native, server, proto):
    c = native.Client({"protocol": proto, "endpoint": server.url, "retry_max_attempts": 1})
    c.write_bytes(B, "x", b"abc", False)
    with pytest.raises(native.StorageError, match="not found|doesn.t exist"):
        c.compose(B, "y", ["x", "missing"])
    with pytest.raises(native.StorageError, match="between 1 and 32|400"):
        c.compose(B, "y", ["x"] * 33)


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_compose_of_synthetic_sources(native, server, proto):
    server.add_synthetic(B, "syn_", "", 0, 2, (1 << 20) + 5)
    c = native.Client({"protocol": proto, "endpoint": server.url})
    m = c.compose(B, "syn_both", ["syn_0", "syn_1"])
    want = native.object_bytes("syn_0", 0, (1 << 20) + 5) + native.object_bytes("syn_1", 0, (1 << 20) + 5)
    assert m["crc32c"] == native.crc32c(want)
    assert c.read_bytes(B, "syn_both") == want


@pytest.mark.parametrize("proto", ["http", "grpc"])
@pytest.mark.parametrize("slices", [2, 5, 8])
def test_parallel_composite_upload(native, server, proto, slices):
    data = os.urandom((9 << 20) + 333)
    w = native.SlicedWriter({"protocol": proto, "endpoint": server.url, "slices": slices,
                             "slice_min_bytes": 1 << 20})
    m = w.write_bytes(B, "big/obj", data, True, 1 << 20)
    assert m["size"] == len(data) and m["crc32c"] == native.crc32c(data)
    c = native.Client({"protocol": proto, "endpoint": server.url})
    assert c.read_bytes(B, "big/obj") == data
    assert [o["name"] for o in c.list_all(B, "big/")] == ["big/obj"]  # temporary parts deleted


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_parallel_composite_upload_retries_part_failures(native, server, proto):
    data = os.urandom(6 << 20)
    server.set_faults({"fail_next": 3, "fail_status": 503})
    w = native.SlicedWriter({"protocol": proto, "endpoint": server.url, "slices": 4, "slice_min_bytes": 1 << 20,
                             "retry_initial_s": 0.001})
    m = w.write_bytes(B, "flaky", data, True, 1 << 20)
    assert m["crc32c"] == native.crc32c(data)


def test_parallel_composite_upload_to_non_retaining_server(native):
    srv = native.Server({"port": 0, "retain_uploads": False})
    srv.start()
    try:
        data = os.urandom(8 << 20)
        for proto in ("http", "grpc"):
            w = native.SlicedWriter({"protocol": proto, "endpoint": srv.url, "slices": 4, "slice_min_bytes": 1 << 20})
            m = w.write_bytes(B, f"gone_{proto}", data)
            assert m["size"] == len(data) and m["crc32c"] == native.crc32c(data)
    finally:
        srv.stop()


def test_small_object_is_a_plain_upload(native, server):
    w = native.SlicedWriter({"protocol": "http", "endpoint": server.url, "slices": 8})
    data = os.urandom(1000)
    m = w.write_bytes(B, "tiny", data)
    assert m["size"] == 1000 and m["crc32c"] == native.crc32c(data)
