"""google.storage.v2 message subset as *Python protobuf* classes, built from a
hand-written FileDescriptorProto (no protoc/grpc_tools in the image).

This is an independent encoding of the same schema the C++ codec hand-codes
(csrc/proto/storage_v2.h); tests use it to cross-check the native wire codec
and to drive grpcio (C-core) peers against the native HTTP/2 stack.  Field
numbers follow the public google/storage/v2/storage.proto; they cannot be
pinned against the real service offline ("parity unpinned").
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto

_MESSAGES = {
    "Timestamp": [("seconds", 1, _F.TYPE_INT64, None, False), ("nanos", 2, _F.TYPE_INT32, None, False)],
    "ObjectChecksums": [("crc32c", 1, _F.TYPE_FIXED32, None, True), ("md5_hash", 2, _F.TYPE_BYTES, None, False)],
    "ChecksummedData": [("content", 1, _F.TYPE_BYTES, None, False), ("crc32c", 2, _F.TYPE_FIXED32, None, True)],
    "ContentRange": [("start", 1, _F.TYPE_INT64, None, False), ("end", 2, _F.TYPE_INT64, None, False),
                     ("complete_length", 3, _F.TYPE_INT64, None, False)],
    "Object": [("name", 1, _F.TYPE_STRING, None, False), ("bucket", 2, _F.TYPE_STRING, None, False),
               ("generation", 3, _F.TYPE_INT64, None, False), ("metageneration", 4, _F.TYPE_INT64, None, False),
               ("storage_class", 5, _F.TYPE_STRING, None, False), ("size", 6, _F.TYPE_INT64, None, False),
               ("content_type", 13, _F.TYPE_STRING, None, False), ("create_time", 14, _F.TYPE_MESSAGE, "Timestamp", False),
               ("checksums", 16, _F.TYPE_MESSAGE, "ObjectChecksums", False),
               ("update_time", 17, _F.TYPE_MESSAGE, "Timestamp", False), ("etag", 27, _F.TYPE_STRING, None, False)],
    "ReadObjectRequest": [("bucket", 1, _F.TYPE_STRING, None, False), ("object", 2, _F.TYPE_STRING, None, False),
                          ("generation", 3, _F.TYPE_INT64, None, False), ("read_offset", 4, _F.TYPE_INT64, None, False),
                          ("read_limit", 5, _F.TYPE_INT64, None, False)],
    "ReadObjectResponse": [("checksummed_data", 1, _F.TYPE_MESSAGE, "ChecksummedData", False),
                           ("object_checksums", 2, _F.TYPE_MESSAGE, "ObjectChecksums", False),
                           ("content_range", 3, _F.TYPE_MESSAGE, "ContentRange", False),
                           ("metadata", 4, _F.TYPE_MESSAGE, "Object", False)],
    "GetObjectRequest": [("bucket", 1, _F.TYPE_STRING, None, False), ("object", 2, _F.TYPE_STRING, None, False),
                         ("generation", 3, _F.TYPE_INT64, None, False)],
    "ListObjectsRequest": [("parent", 1, _F.TYPE_STRING, None, False), ("page_size", 2, _F.TYPE_INT32, None, False),
                           ("page_token", 3, _F.TYPE_STRING, None, False), ("delimiter", 4, _F.TYPE_STRING, None, False),
                           ("prefix", 6, _F.TYPE_STRING, None, False)],
    "ListObjectsResponse": [("objects", 1, _F.TYPE_MESSAGE, "Object", "repeated"),
                            ("prefixes", 2, _F.TYPE_STRING, None, "repeated"),
                            ("next_page_token", 3, _F.TYPE_STRING, None, False)],
    "WriteObjectSpec": [("resource", 1, _F.TYPE_MESSAGE, "Object", False), ("object_size", 8, _F.TYPE_INT64, None, True)],
    "WriteObjectRequest": [("upload_id", 1, _F.TYPE_STRING, None, False),
                           ("write_object_spec", 2, _F.TYPE_MESSAGE, "WriteObjectSpec", False),
                           ("write_offset", 3, _F.TYPE_INT64, None, False),
                           ("checksummed_data", 4, _F.TYPE_MESSAGE, "ChecksummedData", False),
                           ("object_checksums", 6, _F.TYPE_MESSAGE, "ObjectChecksums", False),
                           ("finish_write", 7, _F.TYPE_BOOL, None, False)],
    "WriteObjectResponse": [("persisted_size", 1, _F.TYPE_INT64, None, False),
                            ("resource", 2, _F.TYPE_MESSAGE, "Object", False)],
    "StartResumableWriteRequest": [("write_object_spec", 1, _F.TYPE_MESSAGE, "WriteObjectSpec", False),
                                   ("object_checksums", 5, _F.TYPE_MESSAGE, "ObjectChecksums", False)],
    "StartResumableWriteResponse": [("upload_id", 1, _F.TYPE_STRING, None, False)],
    "QueryWriteStatusRequest": [("upload_id", 1, _F.TYPE_STRING, None, False)],
    "QueryWriteStatusResponse": [("persisted_size", 1, _F.TYPE_INT64, None, False),
                                 ("resource", 2, _F.TYPE_MESSAGE, "Object", False)],
}

_ONEOFS = {"WriteObjectRequest": {"first_message": ["upload_id", "write_object_spec"], "data": ["checksummed_data"]},
           "WriteObjectResponse": {"write_status": ["persisted_size", "resource"]},
           "QueryWriteStatusResponse": {"write_status": ["persisted_size", "resource"]}}

PACKAGE = "gcsb.testing.storage.v2"


def _build():
    fdp = descriptor_pb2.FileDescriptorProto(name="gcsb_storage_v2.proto", package=PACKAGE, syntax="proto3")
    for mname, fields in _MESSAGES.items():
        m = fdp.message_type.add(name=mname)
        oneofs = _ONEOFS.get(mname, {})
        oneof_index = {}
        for i, oname in enumerate(oneofs):
            m.oneof_decl.add(name=oname)
            for f in oneofs[oname]:
                oneof_index[f] = i
        synth = []
        for fname, num, ftype, tname, opt in fields:
            f = m.field.add(name=fname, number=num, type=ftype)
            f.label = _F.LABEL_REPEATED if opt == "repeated" else _F.LABEL_OPTIONAL
            if tname:
                f.type_name = f".{PACKAGE}.{tname}"
            if fname in oneof_index:
                f.oneof_index = oneof_index[fname]
            elif opt is True:  # proto3 `optional`
                synth.append(f)
        for f in synth:
            idx = len(m.oneof_decl)
            m.oneof_decl.add(name="_" + f.name)
            f.oneof_index = idx
            f.proto3_optional = True
    pool = descriptor_pool.DescriptorPool()
    fd = pool.Add(fdp)
    return {name: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{PACKAGE}.{name}"))
            for name in _MESSAGES}


M = _build()
globals().update(M)
