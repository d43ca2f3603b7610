"""HTTP/2 receive settings of the reference's gRPC client, and the multi-frame
receive that keeps them fast.

grpc-go (reference go.mod:20; the client is built with library defaults,
main.go:106-117) does not advertise SETTINGS_MAX_FRAME_SIZE, so its peer sends
DATA frames of at most the RFC 7540 default of 16,384 bytes, and its BDP
estimator grows the stream / connection windows to at most 16 MiB
[lib, parity-unpinned: no grpc-go offline].  `h2_max_frame_size: 0` (not
advertised) and `h2_window: 16 MiB` are that framing here; every read must be
byte-exact under it, including messages that straddle frames, resumes in the
middle of a message, and streams interleaved on one connection (where the
spanning receive's guess of the next frame is wrong and its bytes go back to
the parser: span_spills)."""
import pytest

B = "bkt"
REF = {"h2_max_frame_size": 0, "h2_window": 16 << 20}


def _client(native, srv, **kw):
    cfg = {"protocol": "grpc", "endpoint": srv.url, "retry_initial_s": 0.001}
    cfg.update(REF)
    cfg.update(kw)
    return native.Client(cfg)


def _delta(a, b):
    return {k: b[k] - a[k] for k in ("data_frames", "spanned_frames", "span_reads", "span_spills", "data_bytes")}


@pytest.mark.parametrize("size", [1, 16384 - 20, 16384, 16384 * 3 + 1, (2 << 20) - 1, (2 << 20) + 17, (9 << 20) + 11])
def test_reference_framing_byte_exact(native, server, size):
    server.add_synthetic(B, "f/o_", "", 0, 1, size)
    c = _client(native, server)
    s0 = native.h2_reader_stats()
    assert c.read_bytes(B, "f/o_0") == native.object_bytes("f/o_0", 0, size)
    r = c.read(B, "f/o_0")
    assert r["verified"] and not r["crc_mismatch"] and r["bytes"] == size
    d = _delta(s0, native.h2_reader_stats())
    # the endpoint never sent a frame above the 16 KiB we left it with (a
    # larger one is a connection error on the reader), so two reads of `size`
    # bytes took at least 2 * size / 16 KiB DATA frames
    assert d["data_frames"] >= 2 * (size // 16384)


def test_spanning_lands_many_frames_per_receive(native, server):
    size = 32 << 20
    server.add_synthetic(B, "s/o_", "", 0, 1, size)
    c = _client(native, server)
    c.read(B, "s/o_0")
    s0 = native.h2_reader_stats()
    for _ in range(2):
        assert c.read(B, "s/o_0")["verified"]
    d = _delta(s0, native.h2_reader_stats())
    assert d["data_frames"] >= 2 * size // 16384
    # most frames arrive inside a spanning receive, not one recv() each
    assert d["spanned_frames"] > d["data_frames"] // 2, d
    assert d["span_reads"] < d["data_frames"] // 2, d


def test_spanning_off_is_exact_too(native, server):
    server.add_synthetic(B, "n/o_", "", 0, 1, (3 << 20) + 5)
    c = _client(native, server, h2_span_max_frame=0)
    s0 = native.h2_reader_stats()
    assert c.read_bytes(B, "n/o_0") == native.object_bytes("n/o_0", 0, (3 << 20) + 5)
    assert _delta(s0, native.h2_reader_stats())["spanned_frames"] == 0


@pytest.mark.parametrize("chunk", [4096 + 3, 16384 + 1, 100000])
def test_messages_straddle_frames(native, chunk):
    """gRPC messages whose size is no multiple of the frame: a message's last
    frame is short, the next message starts a new frame (the spanning plan
    ends at the message's content and never guesses across it)."""
    srv = native.Server({"port": 0, "grpc_chunk": chunk})
    srv.start()
    try:
        n = 3 * chunk + 12345
        srv.add_synthetic(B, "m/o_", "", 0, 1, n)
        c = _client(native, srv)
        assert c.read_bytes(B, "m/o_0") == native.object_bytes("m/o_0", 0, n)
        assert c.read(B, "m/o_0")["verified"]
    finally:
        srv.stop()


def test_resume_mid_message_at_reference_framing(native, server):
    size = 10 << 20
    server.add_synthetic(B, "r/o_", "", 0, 1, size)
    # cut the connection inside a 2 MiB message, off any frame boundary
    server.set_faults({"disconnect_at": (5 << 20) + 16384 * 7 + 1234, "disconnect_count": 1})
    c = _client(native, server)
    r = c.read(B, "r/o_0")
    assert r["attempts"] == 2 and r["bytes"] == size and r["verified"]
    assert c.read_bytes(B, "r/o_0") == native.object_bytes("r/o_0", 0, size)


def test_corruption_detected_at_reference_framing(native, server):
    server.add_synthetic(B, "c/o_", "", 0, 1, 6 << 20)
    server.set_faults({"corrupt_at": (4 << 20) + 16384 * 3 + 17, "corrupt_count": 1})
    r = _client(native, server, retry_max_attempts=1).read(B, "c/o_0")
    assert r["crc_mismatch"] or not r["verified"]


@pytest.mark.parametrize("window", [65535, 100000, 1 << 20])
def test_small_windows_stay_exact(native, server, window):
    """Flow control below a message: the endpoint's trains stop at the
    window (rounded to whole frames) and WINDOW_UPDATEs at a quarter of it
    keep the read going."""
    n = (5 << 20) + 3
    server.add_synthetic(B, "w/o_", "", 0, 1, n)
    c = _client(native, server, h2_window=window)
    assert c.read_bytes(B, "w/o_0") == native.object_bytes("w/o_0", 0, n)


def test_interleaved_streams_spill_and_stay_exact(native, server):
    """8 workers multiplexed on ONE connection (pool 1, the reference's
    main.go:30,111): the endpoint interleaves their frames, so spanning
    plans meet another stream's frame and hand the bytes back."""
    workers = 8
    sizes = [(3 << 20) + 4099 * i + 77 for i in range(workers)]
    for i, n in enumerate(sizes):
        server.add_synthetic(B, "i/o_", "", i, 1, n)
    cfg = {"protocol": "grpc", "endpoint": server.url, "bucket": B, "object_prefix": "i/o_", "workers": workers,
           "reads_per_worker": 3, "sink": "discard", "grpc_conn_pool_size": 1, "keep_records": False}
    cfg.update(REF)
    s0 = native.h2_reader_stats()
    r = native.Runner(cfg)
    r.start()
    r.wait()
    s = r.summary()
    assert s["errors"] == 0 and s["verified"] == 3 * workers, s["first_error"]
    d = _delta(s0, native.h2_reader_stats())
    assert d["data_bytes"] >= 3 * sum(sizes)
    assert d["spanned_frames"] > 0


def test_http2_media_reference_framing(native, server):
    n = (7 << 20) + 99
    server.add_synthetic(B, "h/o_", "", 0, 1, n)
    c = native.Client({"protocol": "http2", "endpoint": server.url, **REF})
    s0 = native.h2_reader_stats()
    assert c.read_bytes(B, "h/o_0") == native.object_bytes("h/o_0", 0, n)
    d = _delta(s0, native.h2_reader_stats())
    assert d["data_frames"] >= n // 16384 and d["spanned_frames"] > 0


def test_bad_settings_rejected(native, server):
    with pytest.raises(Exception):
        native.Client({"protocol": "grpc", "endpoint": server.url, "h2_max_frame_size": 1000})
    with pytest.raises(Exception):
        native.Client({"protocol": "grpc", "endpoint": server.url, "h2_window": 100})
