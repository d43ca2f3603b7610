"""Sliced (parallel ranged) reads: storage/sliced.{h,cc} through the runner."""
import pytest

B = "princer-working-dirs"
P = "princer_100M_files/file_"


def _run(native, server, proto, slices, reads=2, **kw):
    cfg = {"protocol": proto, "endpoint": server.url, "bucket": B, "object_prefix": P, "workers": 1,
           "reads_per_worker": reads, "slices": slices, "keep_records": True, "retry_initial_s": 0.01,
           "slice_min_bytes": 4 << 20}
    cfg.update(kw)
    r = native.Runner(cfg)
    r.start()
    r.wait()
    return r.summary(), r.drain()


@pytest.mark.parametrize("proto", ["http", "grpc"])
@pytest.mark.parametrize("slices", [2, 3, 4])
def test_sliced_read_verifies_whole_object(native, server, proto, slices):
    size = (24 << 20) + 12345  # not a multiple of the 2 MiB slice alignment
    server.add_synthetic(B, P, "", 0, 1, size)
    s, recs = _run(native, server, proto, slices)
    assert s["errors"] == 0, s["first_error"]
    assert s["reads"] == 2 and s["verified"] == 2 and s["bytes"] == 2 * size
    assert all(r["bytes"] == size and r["verified"] for r in recs)
    # each slice used its own connection: `slices` ranged requests per read (+1 stat)
    st = server.stats()
    if proto == "grpc":
        assert st["grpc_calls"] == 2 * (slices + 1)
    else:
        assert st["http_requests"] == 2 * (slices + 1)


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_small_object_falls_back_to_fewer_slices(native, server, proto):
    server.add_synthetic(B, P, "", 0, 1, 3 << 20)  # < 2 x slice_min_bytes
    s, _ = _run(native, server, proto, 4)
    assert s["errors"] == 0 and s["verified"] == 2


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_sliced_read_detects_corruption(native, server, proto):
    size = 16 << 20
    server.add_synthetic(B, P, "", 0, 1, size)
    server.set_faults({"corrupt_at": (13 << 20) + 7, "corrupt_count": 1})  # inside the last slice
    s, _ = _run(native, server, proto, 4, reads=1)
    assert s["errors"] == 1
    assert "mismatch" in s["first_error"] or "bad CRC" in s["first_error"]


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_sliced_read_resumes_a_dropped_slice(native, server, proto):
    size = 16 << 20
    server.add_synthetic(B, P, "", 0, 1, size)
    server.set_faults({"disconnect_at": (9 << 20) + 100, "disconnect_count": 1})
    s, recs = _run(native, server, proto, 4, reads=1)
    assert s["errors"] == 0, s["first_error"]
    assert s["verified"] == 1 and s["retries"] >= 1
    assert recs[0]["attempts"] >= 2


@pytest.mark.parametrize("proto", ["http", "grpc"])
@pytest.mark.parametrize("piece_mib", [2, 4])
def test_piece_mode_balances_and_verifies(native, server, proto, piece_mib):
    """slice_piece_bytes > 0: the streams pull 2 MiB-aligned pieces from a
    shared cursor (one ranged request per piece, two sinks per stream); the
    object CRC32C is the in-order combine of the piece CRCs."""
    size = (24 << 20) + 12345
    server.add_synthetic(B, P, "", 0, 1, size)
    s, recs = _run(native, server, proto, 4, slice_piece_bytes=piece_mib << 20)
    assert s["errors"] == 0, s["first_error"]
    assert s["reads"] == 2 and s["verified"] == 2 and s["bytes"] == 2 * size
    assert all(r["bytes"] == size and r["verified"] for r in recs)
    pieces = -(-size // (piece_mib << 20))
    st = server.stats()
    calls = st["grpc_calls"] if proto == "grpc" else st["http_requests"]
    assert calls == 2 * (pieces + 1)  # one ranged request per piece (+1 stat) per read
    assert s["slice_skew_ms"] >= 0.0


def _tapered_pieces(size, piece, floor, streams, align=2 << 20):
    """Python model of SlicedReader::read's guided piece schedule."""
    out, off = [], 0
    while off < size:
        guided = -(-((size - off) // (2 * streams)) // align) * align
        n = min(max(min(piece, guided), min(max(align, floor // align * align), piece)), size - off)
        out.append(n)
        off += n
    return out


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_piece_mode_tapers_toward_the_end(native, server, proto):
    """slice_piece_min_bytes > 0: pieces shrink toward the end of the object
    (min(piece, remaining / 2 streams), 2 MiB aligned, floor 2 MiB) so the
    streams finish together; the object still verifies byte-exact."""
    size = (40 << 20) + 777
    server.add_synthetic(B, P, "", 0, 1, size)
    s, recs = _run(native, server, proto, 4, slice_piece_bytes=8 << 20, slice_piece_min_bytes=2 << 20)
    assert s["errors"] == 0, s["first_error"]
    assert s["reads"] == 2 and s["verified"] == 2 and s["bytes"] == 2 * size
    plan = _tapered_pieces(size, 8 << 20, 2 << 20, 4)
    assert sum(plan) == size and plan[0] > plan[-2] == 2 << 20
    assert plan == sorted(plan, reverse=True)
    st = server.stats()
    calls = st["grpc_calls"] if proto == "grpc" else st["http_requests"]
    assert calls == 2 * (len(plan) + 1)  # one ranged request per piece (+1 stat) per read


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_piece_mode_detects_corruption_and_resumes(native, server, proto):
    size = 16 << 20
    server.add_synthetic(B, P, "", 0, 1, size)
    server.set_faults({"corrupt_at": (13 << 20) + 7, "corrupt_count": 1})
    s, _ = _run(native, server, proto, 4, reads=1, slice_piece_bytes=2 << 20)
    assert s["errors"] == 1
    assert "mismatch" in s["first_error"] or "bad CRC" in s["first_error"]
    server.set_faults({"disconnect_at": (9 << 20) + 100, "disconnect_count": 1})
    s, recs = _run(native, server, proto, 4, reads=1, slice_piece_bytes=2 << 20)
    assert s["errors"] == 0, s["first_error"]
    assert s["verified"] == 1 and s["retries"] >= 1


def test_sliced_discard_without_host_crc_is_unverified(native, server):
    server.add_synthetic(B, P, "", 0, 1, 16 << 20)
    s, _ = _run(native, server, "http", 4, host_crc=False)
    assert s["errors"] == 0 and s["verified"] == 0 and s["bytes"] == 2 * (16 << 20)
