"""Native HTTP/2 + gRPC stack vs grpcio (gRPC C-core) in both directions.

grpcio is the independent implementation here: it Huffman-codes headers,
uses dynamic HPACK tables and BDP-driven flow-control windows, so it checks
the native HPACK decoder, framing and flow control; messages are coded with
Python protobuf classes built from an independent descriptor.
"""
import os
import threading
from concurrent import futures

import grpc
import pytest

from custom_go_client_benchmark_amd.server import storage_v2_pb as pb

B = "princer-working-dirs"
P = "princer_100M_files/file_"
SVC = "google.storage.v2.Storage"


def _ident(x):
    return x


@pytest.fixture()
def chan(server):
    ch = grpc.insecure_channel(server.url.replace("http://", ""))
    yield ch
    ch.close()


def test_grpcio_client_reads_native_server(native, server, chan):
    size = 5 * (1 << 20) + 321
    server.add_synthetic(B, P, "", 0, 1, size)
    read = chan.unary_stream(f"/{SVC}/ReadObject", request_serializer=_ident,
                             response_deserializer=pb.ReadObjectResponse.FromString)
    req = pb.ReadObjectRequest(bucket=f"projects/_/buckets/{B}", object=P + "0").SerializeToString()
    data = b""
    first = True
    for msg in read(req, metadata=[("x-goog-request-params", f"bucket=projects/_/buckets/{B}")]):
        cd = msg.checksummed_data
        assert cd.HasField("crc32c") and cd.crc32c == native.crc32c(cd.content)
        if first:
            assert msg.metadata.size == size and msg.object_checksums.crc32c == server.object_info(B, P + "0")["crc32c"]
            first = False
        data += cd.content
    assert data == native.object_bytes(P + "0", 0, size)


def test_grpcio_client_ranged_read_and_not_found(native, server, chan):
    server.add_synthetic(B, P, "", 0, 1, 3 << 20)
    read = chan.unary_stream(f"/{SVC}/ReadObject", request_serializer=_ident,
                             response_deserializer=pb.ReadObjectResponse.FromString)
    req = pb.ReadObjectRequest(bucket=f"projects/_/buckets/{B}", object=P + "0", read_offset=1000,
                               read_limit=70000).SerializeToString()
    data = b"".join(m.checksummed_data.content for m in read(req))
    assert data == native.object_bytes(P + "0", 1000, 70000)
    with pytest.raises(grpc.RpcError) as ei:
        list(read(pb.ReadObjectRequest(bucket=f"projects/_/buckets/{B}", object="missing").SerializeToString()))
    assert ei.value.code() == grpc.StatusCode.NOT_FOUND


def test_grpcio_client_list_get_write(native, server, chan):
    server.add_synthetic(B, "ls/o", "", 0, 7, 100)
    lst = chan.unary_unary(f"/{SVC}/ListObjects", request_serializer=_ident,
                           response_deserializer=pb.ListObjectsResponse.FromString)
    r = lst(pb.ListObjectsRequest(parent=f"projects/_/buckets/{B}", prefix="ls/", page_size=5).SerializeToString())
    assert len(r.objects) == 5 and r.next_page_token
    get = chan.unary_unary(f"/{SVC}/GetObject", request_serializer=_ident, response_deserializer=pb.Object.FromString)
    o = get(pb.GetObjectRequest(bucket=f"projects/_/buckets/{B}", object="ls/o3").SerializeToString())
    assert o.size == 100 and o.checksums.crc32c == server.object_info(B, "ls/o3")["crc32c"]

    payload = os.urandom(5 * (1 << 20) + 7)
    write = chan.stream_unary(f"/{SVC}/WriteObject", request_serializer=_ident,
                              response_deserializer=pb.WriteObjectResponse.FromString)

    def msgs():
        step = 2 << 20
        for off in range(0, len(payload), step):
            chunk = payload[off : off + step]
            m = pb.WriteObjectRequest(write_offset=off,
                                      checksummed_data=pb.ChecksummedData(content=chunk, crc32c=native.crc32c(chunk)))
            if off == 0:
                m.write_object_spec.resource.name = "up/grpcio"
                m.write_object_spec.resource.bucket = f"projects/_/buckets/{B}"
            if off + step >= len(payload):
                m.finish_write = True
                m.object_checksums.crc32c = native.crc32c(payload)
            yield m.SerializeToString()

    resp = write(msgs())
    assert resp.resource.size == len(payload) and resp.resource.checksums.crc32c == native.crc32c(payload)
    c = native.Client({"protocol": "grpc", "endpoint": server.url})
    assert c.read_bytes(B, "up/grpcio") == payload


class _GrpcioStorage:
    """Minimal google.storage.v2 service on grpcio, for the native client."""

    def __init__(self, native, objects):
        self.native = native
        self.objects = dict(objects)
        self.writes = {}

    def ReadObject(self, req_bytes, ctx):
        req = pb.ReadObjectRequest.FromString(req_bytes)
        data = self.objects.get(req.object)
        if data is None:
            ctx.abort(grpc.StatusCode.NOT_FOUND, "no such object")
        start = req.read_offset
        end = len(data) if req.read_limit <= 0 else min(len(data), start + req.read_limit)
        first = True
        step = 2 << 20
        off = start
        while off < end or first:
            chunk = data[off : min(end, off + step)]
            m = pb.ReadObjectResponse(checksummed_data=pb.ChecksummedData(content=chunk,
                                                                           crc32c=self.native.crc32c(chunk)))
            if first:
                m.object_checksums.crc32c = self.native.crc32c(data)
                m.metadata.name = req.object
                m.metadata.size = len(data)
                m.metadata.generation = 7
                first = False
            yield m.SerializeToString()
            off += len(chunk)
            if not chunk:
                break

    def GetObject(self, req_bytes, ctx):
        req = pb.GetObjectRequest.FromString(req_bytes)
        data = self.objects[req.object]
        o = pb.Object(name=req.object, bucket=req.bucket, size=len(data), generation=7)
        o.checksums.crc32c = self.native.crc32c(data)
        return o.SerializeToString()

    def ListObjects(self, req_bytes, ctx):
        req = pb.ListObjectsRequest.FromString(req_bytes)
        r = pb.ListObjectsResponse()
        for name in sorted(self.objects):
            if name.startswith(req.prefix):
                r.objects.add(name=name, size=len(self.objects[name]))
        return r.SerializeToString()

    def WriteObject(self, it, ctx):
        buf = bytearray()
        name = None
        for raw in it:
            m = pb.WriteObjectRequest.FromString(raw)
            if m.HasField("write_object_spec"):
                name = m.write_object_spec.resource.name
            assert m.write_offset == len(buf)
            assert self.native.crc32c(m.checksummed_data.content) == m.checksummed_data.crc32c
            buf += m.checksummed_data.content
            if m.finish_write:
                assert m.object_checksums.crc32c == self.native.crc32c(bytes(buf))
        self.objects[name] = bytes(buf)
        r = pb.WriteObjectResponse()
        r.resource.name = name
        r.resource.size = len(buf)
        r.resource.checksums.crc32c = self.native.crc32c(bytes(buf))
        return r.SerializeToString()


@pytest.fixture()
def grpcio_server(native):
    objs = {P + "0": native.object_bytes(P + "0", 0, 7 * (1 << 20) + 99), "small": b"tiny"}
    impl = _GrpcioStorage(native, objs)
    handlers = {
        "ReadObject": grpc.unary_stream_rpc_method_handler(impl.ReadObject, request_deserializer=_ident,
                                                           response_serializer=_ident),
        "GetObject": grpc.unary_unary_rpc_method_handler(impl.GetObject, request_deserializer=_ident,
                                                         response_serializer=_ident),
        "ListObjects": grpc.unary_unary_rpc_method_handler(impl.ListObjects, request_deserializer=_ident,
                                                           response_serializer=_ident),
        "WriteObject": grpc.stream_unary_rpc_method_handler(impl.WriteObject, request_deserializer=_ident,
                                                            response_serializer=_ident),
    }
    srv = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
    srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SVC, handlers),))
    port = srv.add_insecure_port("127.0.0.1:0")
    srv.start()
    yield impl, f"http://127.0.0.1:{port}"
    srv.stop(0)


def test_native_client_against_grpcio_server(native, grpcio_server):
    impl, url = grpcio_server
    c = native.Client({"protocol": "grpc", "endpoint": url, "retry_max_attempts": 1})
    r = c.read(B, P + "0")
    assert r["bytes"] == len(impl.objects[P + "0"]) and r["verified"] and not r["crc_mismatch"]
    assert c.read_bytes(B, P + "0") == impl.objects[P + "0"]
    assert c.read_bytes(B, P + "0", 4096, 100) == impl.objects[P + "0"][4096:4196]
    assert c.stat(B, "small")["size"] == 4
    assert [o["name"] for o in c.list_all(B, "")] == sorted(impl.objects)
    with pytest.raises(native.StorageError, match="doesn't exist"):
        c.read(B, "missing")


def test_native_client_concurrent_streams_on_one_grpcio_connection(native, grpcio_server):
    impl, url = grpcio_server
    c = native.Client({"protocol": "grpc", "endpoint": url, "grpc_conn_pool_size": 1})
    errs = []

    def one():
        try:
            for _ in range(3):
                assert c.read(B, P + "0")["verified"]
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=one) for _ in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs


def test_native_client_writes_to_grpcio_server(native, grpcio_server):
    impl, url = grpcio_server
    c = native.Client({"protocol": "grpc", "endpoint": url})
    data = os.urandom(6 * (1 << 20) + 5)
    m = c.write_bytes(B, "from-native", data, False)
    assert m["size"] == len(data) and impl.objects["from-native"] == data
