"""Per-read tracing: ratio sampler + batch exporter (OTLP/JSON lines).

Reference (trace_exporter.go): enableTraceExport(ctx, sampleRate) builds a
Cloud Trace exporter, a resource with the GCP detector + telemetry SDK +
service.name=princer-storage-benchmark + transport=<protocol> (:25-35), a
tracer provider with a batcher and TraceIDRatioBased(rate) — not parent based
(:41-45), installs an OpenCensus bridge so the storage library's spans nest
under the app span (:49-52), and returns a cleanup that force-flushes and
shuts down (:55-60).  Each read is one span "ReadObject" with attribute
bucket (main.go:128-132,149).

Here sampling is decided in C++ per read (TraceIDRatioBased: lower 8 bytes of
a random 128-bit trace id >> 1 < rate * 2^63) and the runner records
timestamps; this module turns sampled records into OTLP/JSON spans: the
"ReadObject" span plus child spans for the transport stages the bridged
library spans would have shown (NewReader = request -> first byte, Read =
body streaming, and HBMLanding = last host byte -> bytes in HBM + CRC32C
verified, for the GPU sink).  Cloud Trace is unreachable offline, so batches
go to a local file (one OTLP ExportTraceServiceRequest JSON per line).
"""
from __future__ import annotations

import json
import os
import socket
import threading
import time

TRACER_NAME = "princer-storage-benchmark"
SDK_VERSION = "0.1.0"


def _attr(k: str, v) -> dict:
    if isinstance(v, bool):
        return {"key": k, "value": {"boolValue": v}}
    if isinstance(v, int):
        return {"key": k, "value": {"intValue": str(v)}}
    if isinstance(v, float):
        return {"key": k, "value": {"doubleValue": v}}
    return {"key": k, "value": {"stringValue": str(v)}}


def trace_id_ratio_sampled(trace_lo: int, rate: float) -> bool:
    """OTel TraceIDRatioBased decision on the trace id's lower 8 bytes."""
    if rate >= 1.0:
        return True
    if rate <= 0.0:
        return False
    bound = int(rate * (1 << 63))
    return (trace_lo >> 1) < bound


def resource_attributes(transport: str, extra: dict | None = None) -> list[dict]:
    attrs = {
        "service.name": TRACER_NAME,
        "transport": transport,
        "telemetry.sdk.name": "gcsb-native",
        "telemetry.sdk.language": "cpp",
        "telemetry.sdk.version": SDK_VERSION,
        "host.name": socket.gethostname(),
        "cloud.provider": os.environ.get("GCSB_CLOUD_PROVIDER", "none"),
        "process.pid": os.getpid(),
    }
    attrs.update(extra or {})
    return [_attr(k, v) for k, v in attrs.items()]


def record_to_spans(rec: dict, bucket: str, gpu: bool) -> list[dict]:
    """One sampled read record -> [ReadObject, NewReader, Read, (HBMLanding)]."""
    trace_id = f"{rec['trace_hi']:016x}{rec['trace_lo']:016x}"
    root_id = f"{rec['span_id']:016x}"
    wall0 = rec["start_wall_ns"]
    t0 = rec["start_ns"]

    def at(ns: int) -> str:
        return str(wall0 + (ns - t0))

    status = {"code": 1} if rec["ok"] else {"code": 2, "message": rec.get("error", "")}
    root = {
        "traceId": trace_id, "spanId": root_id, "name": "ReadObject", "kind": 1,
        "startTimeUnixNano": at(t0), "endTimeUnixNano": at(rec["end_ns"]),
        "attributes": [_attr("bucket", bucket), _attr("object", rec["object"]), _attr("bytes", int(rec["bytes"])),
                       _attr("attempts", int(rec["attempts"])), _attr("worker", int(rec["worker"])),
                       _attr("crc32c.verified", bool(rec["verified"]))],
        "status": status,
    }
    spans = [root]
    sid = rec["span_id"]

    def child(name: str, a: int, b: int, k: int) -> dict:
        return {"traceId": trace_id, "spanId": f"{(sid + k) & 0xFFFFFFFFFFFFFFFF:016x}", "parentSpanId": root_id,
                "name": name, "kind": 3 if name == "NewReader" else 1,
                "startTimeUnixNano": at(a), "endTimeUnixNano": at(b), "attributes": [], "status": {"code": 0}}

    if rec["ttfb_ns"]:
        spans.append(child("NewReader", t0, rec["ttfb_ns"], 1))
        if rec["host_done_ns"]:
            spans.append(child("Read", rec["ttfb_ns"], rec["host_done_ns"], 2))
    if gpu and rec["host_done_ns"]:
        spans.append(child("HBMLanding", rec["host_done_ns"], rec["end_ns"], 3))
    return spans


class BatchTraceExporter:
    """BatchSpanProcessor equivalent writing OTLP/JSON lines to `path`."""

    def __init__(self, path: str, transport: str, bucket: str, gpu: bool, max_batch: int = 512,
                 interval_s: float = 5.0, resource_extra: dict | None = None):
        self.path = path
        self.bucket = bucket
        self.gpu = gpu
        self.max_batch = max_batch
        self.interval_s = interval_s
        self.resource = resource_attributes(transport, resource_extra)
        self._q: list[dict] = []
        self._mu = threading.Lock()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._loop, name="trace-exporter", daemon=True)
        self.exported_spans = 0
        self._thread.start()

    def on_records(self, records: list[dict]):
        spans = []
        for r in records:
            if r.get("sampled"):
                spans.extend(record_to_spans(r, self.bucket, self.gpu))
        if not spans:
            return
        with self._mu:
            self._q.extend(spans)
            full = len(self._q) >= self.max_batch
        if full:
            self.force_flush()

    def _loop(self):
        while not self._stop.wait(self.interval_s):
            self.force_flush()

    def force_flush(self):
        with self._mu:
            batch, self._q = self._q, []
        if not batch:
            return
        doc = {"resourceSpans": [{"resource": {"attributes": self.resource},
                                  "scopeSpans": [{"scope": {"name": TRACER_NAME, "version": SDK_VERSION},
                                                  "spans": batch}]}]}
        with open(self.path, "a") as f:
            f.write(json.dumps(doc) + "\n")
        self.exported_spans += len(batch)

    def shutdown(self):
        self._stop.set()
        self._thread.join(timeout=5)
        self.force_flush()


def enable_trace_export(path: str, transport: str, bucket: str, gpu: bool = False, **kw):
    """Mirror of enableTraceExport: returns (exporter, cleanup)."""
    exp = BatchTraceExporter(path, transport, bucket, gpu, **kw)
    return exp, exp.shutdown
