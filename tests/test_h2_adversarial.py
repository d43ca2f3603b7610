"""The gRPC client's spanning receive (h2/h2_client.h H2DataCursor) against a
raw HTTP/2 peer written here frame by frame: frames shorter than the client's
plan assumed, control frames between DATA frames, padded frames and
END_STREAM on DATA -- every way the plan's guess of the next frame can be
wrong.  Each case must land the object byte-exact with every ChecksummedData
CRC checked, and the wrong guesses must show up as span_spills (the bytes went
back to the frame parser)."""
import random
import socket
import struct
import threading

import pytest

PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"


def frame(ftype, flags, sid, payload):
    n = len(payload)
    return struct.pack(">BHBBI", n >> 16, n & 0xFFFF, ftype, flags, sid & 0x7FFFFFFF) + payload


def hpack_literal(headers):
    out = b""
    for k, v in headers:  # literal header field without indexing, new name, no Huffman
        kb, vb = k.encode(), v.encode()
        assert len(kb) < 127 and len(vb) < 127
        out += b"\x00" + bytes([len(kb)]) + kb + bytes([len(vb)]) + vb
    return out


def varint(v):
    out = b""
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out += bytes([b | 0x80])
        else:
            return out + bytes([b])


def read_response_msg(native, content):
    crc = native.crc32c(content)
    cd = b"\x0a" + varint(len(content)) + content + b"\x15" + struct.pack("<I", crc)
    msg = b"\x0a" + varint(len(cd)) + cd
    return b"\x00" + struct.pack(">I", len(msg)) + msg


class RawPeer:
    """Accepts one connection, waits for `nreq` request streams and answers
    them with build(stream ids) (the frames to send)."""

    def __init__(self, build, nreq=1):
        self.build = build
        self.nreq = nreq
        self.ls = socket.socket()
        self.ls.bind(("127.0.0.1", 0))
        self.ls.listen(1)
        self.port = self.ls.getsockname()[1]
        self.t = threading.Thread(target=self.run, daemon=True)
        self.t.start()

    def recv_frame(self, c):
        hdr = b""
        while len(hdr) < 9:
            d = c.recv(9 - len(hdr))
            if not d:
                raise EOFError
            hdr += d
        n = (hdr[0] << 16) | (hdr[1] << 8) | hdr[2]
        p = b""
        while len(p) < n:
            d = c.recv(n - len(p))
            if not d:
                raise EOFError
            p += d
        return hdr[3], hdr[4], struct.unpack(">I", hdr[5:9])[0] & 0x7FFFFFFF, p

    def run(self):
        c, _ = self.ls.accept()
        try:
            got = b""
            while len(got) < 24:
                got += c.recv(24 - len(got))
            c.sendall(frame(4, 0, 0, b""))  # our SETTINGS (all defaults)
            sids = []
            while len(sids) < self.nreq:
                t, fl, s, p = self.recv_frame(c)
                if t == 4 and not (fl & 1):
                    c.sendall(frame(4, 1, 0, b""))
                if t == 0 and (fl & 1):
                    sids.append(s)
            c.sendall(b"".join(self.build(sids[0] if self.nreq == 1 else sids)))
            while True:
                self.recv_frame(c)
        except (EOFError, OSError):
            pass
        finally:
            c.close()

    @property
    def url(self):
        return f"http://127.0.0.1:{self.port}"


def resp_headers(sid):
    return frame(1, 4, sid, hpack_literal([(":status", "200"), ("content-type", "application/grpc")]))


def trailers(sid):
    return frame(1, 4 | 1, sid, hpack_literal([("grpc-status", "0")]))


def split(data, sizes):
    out, i, k = [], 0, 0
    while i < len(data):
        n = sizes[k % len(sizes)]
        out.append(data[i:i + n])
        i += n
        k += 1
    return out


def make_content(n, seed):
    r = random.Random(seed)
    return bytes(r.getrandbits(8) for _ in range(n))


def run_case(native, build_frames, contents):
    peer = RawPeer(build_frames)
    c = native.Client({"protocol": "grpc", "endpoint": peer.url, "h2_max_frame_size": 0, "h2_window": 16 << 20,
                       "retry_max_attempts": 1})
    s0 = native.h2_reader_stats()
    got = c.read_bytes("b", "o")
    s1 = native.h2_reader_stats()
    assert got == b"".join(contents)
    return {k: s1[k] - s0[k] for k in ("data_frames", "spanned_frames", "span_reads", "span_spills")}


def stream_of(native, contents):
    return b"".join(read_response_msg(native, x) for x in contents)


@pytest.fixture(scope="module")
def contents():
    return [make_content(300000, 1), make_content(70001, 2), make_content(16384 * 5, 3)]


def test_full_frames_span(native, contents):
    def build(sid):
        data = stream_of(native, contents)
        return [resp_headers(sid)] + [frame(0, 0, sid, p) for p in split(data, [16384])] + [trailers(sid)]
    d = run_case(native, build, contents)
    assert d["spanned_frames"] > 0


def test_short_frames_spill(native, contents):
    """Frames shorter than the 16 KiB the plan predicts."""
    def build(sid):
        data = stream_of(native, contents)
        return [resp_headers(sid)] + [frame(0, 0, sid, p) for p in split(data, [16384, 16384, 5000, 16384, 1, 9])] \
            + [trailers(sid)]
    d = run_case(native, build, contents)
    assert d["span_spills"] > 0 and d["spanned_frames"] > 0, d


def test_control_frames_between_data_spill(native, contents):
    """PING and WINDOW_UPDATE frames where the plan expects DATA."""
    def build(sid):
        data = stream_of(native, contents)
        out = [resp_headers(sid)]
        for i, p in enumerate(split(data, [16384])):
            out.append(frame(0, 0, sid, p))
            if i % 4 == 3:
                out.append(frame(6, 0, 0, b"12345678"))
            if i % 7 == 5:
                out.append(frame(8, 0, 0, struct.pack(">I", 1000)))
        return out + [trailers(sid)]
    d = run_case(native, build, contents)
    assert d["span_spills"] > 0, d


def test_padded_frames_spill(native, contents):
    def build(sid):
        data = stream_of(native, contents)
        out = [resp_headers(sid)]
        for i, p in enumerate(split(data, [16384 - 20])):
            if i % 3 == 1:
                out.append(frame(0, 0x8, sid, bytes([19]) + p + b"\0" * 19))  # PADDED
            else:
                out.append(frame(0, 0, sid, p))
        return out + [trailers(sid)]
    d = run_case(native, build, contents)
    assert d["span_spills"] > 0, d


def test_random_frame_sizes(native, contents):
    r = random.Random(7)
    sizes = [r.choice([1, 9, 100, 4096, 16383, 16384, 16384, 16384]) for _ in range(200)]

    def build(sid):
        data = stream_of(native, contents)
        return [resp_headers(sid)] + [frame(0, 0, sid, p) for p in split(data, sizes)] + [trailers(sid)]
    run_case(native, build, contents)


def test_end_stream_on_last_data(native, contents):
    """A trailers-less stream: END_STREAM on the last DATA frame is an error
    (no grpc-status); the plan must not read past it either way."""
    def build(sid):
        data = stream_of(native, contents)
        fr = split(data, [16384])
        return [resp_headers(sid)] + [frame(0, 0, sid, p) for p in fr[:-1]] + [frame(0, 1, sid, fr[-1])]
    peer = RawPeer(build)
    c = native.Client({"protocol": "grpc", "endpoint": peer.url, "h2_max_frame_size": 0, "retry_max_attempts": 1})
    with pytest.raises(Exception, match="without trailers|grpc-status|code"):
        c.read_bytes("b", "o")


def test_two_streams_interleaved_frame_by_frame(native, contents):
    """Two reads multiplexed on one connection (gRPC pool 1), their DATA
    frames alternating in runs of 1..3: every spanning plan meets the other
    stream's frame.  Both land byte-exact (discard sink, host CRC32C)."""
    other = [make_content(200001, 9), make_content(16384 * 2 + 5, 10)]

    def build(sids):
        a = split(stream_of(native, contents), [16384])
        b = split(stream_of(native, other), [16384])
        out = [resp_headers(sids[0]), resp_headers(sids[1])]
        i = j = k = 0
        while i < len(a) or j < len(b):
            for _ in range(1 + k % 3):
                if i < len(a):
                    out.append(frame(0, 0, sids[0], a[i]))
                    i += 1
            for _ in range(1 + (k + 1) % 3):
                if j < len(b):
                    out.append(frame(0, 0, sids[1], b[j]))
                    j += 1
            k += 1
        return out + [trailers(sids[0]), trailers(sids[1])]

    peer = RawPeer(build, nreq=2)
    s0 = native.h2_reader_stats()
    r = native.Runner({"protocol": "grpc", "endpoint": peer.url, "bucket": "b", "object_names": ["o"], "workers": 2,
                       "reads_per_worker": 1, "sink": "discard", "grpc_conn_pool_size": 1, "keep_records": True,
                       "retry_max_attempts": 1, "h2_max_frame_size": 0})
    r.start()
    r.wait()
    s = r.summary()
    d = native.h2_reader_stats()
    assert s["errors"] == 0 and s["verified"] == 2, s["first_error"]
    got = sorted(x["bytes"] for x in r.drain())
    assert got == sorted([sum(map(len, contents)), sum(map(len, other))])
    assert d["span_spills"] > s0["span_spills"]
