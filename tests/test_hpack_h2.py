"""HPACK (RFC 7541) conformance: Huffman + header blocks from Appendix C."""
import os

import pytest


@pytest.mark.parametrize("text,hexenc", [
    (b"www.example.com", "f1e3c2e5f23a6ba0ab90f4ff"),
    (b"no-cache", "a8eb10649cbf"),
    (b"custom-key", "25a849e95ba97d7f"),
    (b"custom-value", "25a849e95bb8e8b4bf"),
    (b"302", "6402"),
    (b"private", "aec3771a4b"),
    (b"Mon, 21 Oct 2013 20:13:21 GMT", "d07abe941054d444a8200595040b8166e082a62d1bff"),
    (b"https://www.example.com", "9d29ad171863c78f0b97c8e9ae82ae43d3"),
])
def test_huffman_rfc_vectors(native, text, hexenc):
    assert native.huffman_encode(text).hex() == hexenc
    assert native.huffman_decode(bytes.fromhex(hexenc)) == text


def test_huffman_roundtrip_all_bytes(native):
    for _ in range(50):
        s = os.urandom(200)
        assert native.huffman_decode(native.huffman_encode(s)) == s
    s = bytes(range(256))
    assert native.huffman_decode(native.huffman_encode(s)) == s


def test_huffman_rejects_bad_padding(native):
    enc = native.huffman_encode(b"a")  # 5 bits + 3 bits of 1s padding
    bad = bytes([enc[0] & 0xF8])  # padding bits zeroed
    with pytest.raises(RuntimeError):
        native.huffman_decode(bad)


def test_rfc_c3_requests_without_huffman(native):
    # RFC 7541 C.3: three requests sharing one decoder (dynamic table)
    b1 = bytes.fromhex("828684410f7777772e6578616d706c652e636f6d")
    b2 = bytes.fromhex("828684be58086e6f2d6361636865")
    b3 = bytes.fromhex("828785bf400a637573746f6d2d6b65790c637573746f6d2d76616c7565")
    out = native.hpack_decode_blocks([b1, b2, b3])
    assert out[0] == [(":method", "GET"), (":scheme", "http"), (":path", "/"), (":authority", "www.example.com")]
    assert out[1][-1] == ("cache-control", "no-cache") and out[1][3] == (":authority", "www.example.com")
    assert out[2] == [(":method", "GET"), (":scheme", "https"), (":path", "/index.html"),
                      (":authority", "www.example.com"), ("custom-key", "custom-value")]


def test_rfc_c4_requests_with_huffman(native):
    b1 = bytes.fromhex("828684418cf1e3c2e5f23a6ba0ab90f4ff")
    b2 = bytes.fromhex("828684be5886a8eb10649cbf")
    b3 = bytes.fromhex("828785bf408825a849e95ba97d7f8925a849e95bb8e8b4bf")
    out = native.hpack_decode_blocks([b1, b2, b3])
    assert out[0][3] == (":authority", "www.example.com")
    assert out[1][4] == ("cache-control", "no-cache")
    assert out[2][4] == ("custom-key", "custom-value")


@pytest.mark.parametrize("huffman", [False, True])
def test_encoder_roundtrip(native, huffman):
    h = [(":method", "POST"), (":scheme", "http"), (":path", "/google.storage.v2.Storage/ReadObject"),
         (":authority", "127.0.0.1:1234"), ("content-type", "application/grpc"), ("te", "trailers"),
         ("x-goog-request-params", "bucket=projects%2F_%2Fbuckets%2Fb"), ("authorization", "Bearer x" * 50)]
    blk = native.hpack_encode(h, huffman)
    assert native.hpack_decode_blocks([blk])[0] == h


def test_protobuf_codec_matches_python_protobuf(native):
    from custom_go_client_benchmark_amd.server import storage_v2_pb as pb

    r = pb.ReadObjectRequest.FromString(native.pb_read_request("bkt", "a/b", 12345, 678))
    assert (r.bucket, r.object, r.read_offset, r.read_limit) == ("projects/_/buckets/bkt", "a/b", 12345, 678)
    content = os.urandom(3000)
    m = pb.ReadObjectResponse.FromString(native.pb_read_response(content, 0xDEADBEEF, 0x1234, 99, "obj"))
    assert m.checksummed_data.content == content and m.checksummed_data.crc32c == 0xDEADBEEF
    assert m.object_checksums.crc32c == 0x1234 and m.metadata.size == 99 and m.content_range.complete_length == 99
    w = pb.WriteObjectRequest.FromString(native.pb_write_request("", "bkt", "x", 0, b"abc", True, 7))
    assert w.write_object_spec.resource.name == "x" and w.checksummed_data.content == b"abc"
    assert w.finish_write and w.object_checksums.crc32c == 7
    assert w.checksummed_data.crc32c == native.crc32c(b"abc")
    w2 = pb.WriteObjectRequest.FromString(native.pb_write_request("up1", "bkt", "x", 5, b"", False, 0))
    assert w2.upload_id == "up1" and w2.write_offset == 5 and not w2.finish_write
    o = pb.Object(name="n", bucket="projects/_/buckets/b", size=5, generation=9)
    o.checksums.crc32c = 42
    d = native.pb_decode_object(o.SerializeToString())
    assert d["name"] == "n" and d["size"] == 5 and d["generation"] == 9 and d["crc32c"] == 42
