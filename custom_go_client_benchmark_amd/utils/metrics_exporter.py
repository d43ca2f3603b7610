"""Read-latency metric: view registration + periodic exporter.

Reference (metrics_exporter.go): an OpenCensus float64 measure `readLatency`
("Complete read latency", unit ms, :17) recorded once per read with the
integer-truncated milliseconds (main.go:146); a view
`princer_go_client_read_latency` with tag key `princer_read_latency` and
aggregation ochttp.DefaultLatencyDistribution (:22-34); a Stackdriver exporter
with metric prefix `custom.googleapis.com/custom-go-client/` reporting every
30 s (:36-58); closeSDExporter meant to stop+flush but is a no-op because of
a shadowed variable (:37,60-67).

Here the same view (name, description, tag key, bucket bounds, 30 s cadence)
is exported offline — Cloud Monitoring is unreachable from the benchmark
boxes — as (a) a Prometheus text exposition file, (b) JSONL records shaped
like Cloud Monitoring TimeSeries with the same metric type, and optionally (c)
a prometheus_client HTTP endpoint.  close() DOES flush (Q2 fixed).  The
histogram itself is accumulated in C++ by the runner (atomic bucket counts);
this module only snapshots and writes it.
"""
from __future__ import annotations

import json
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Callable

from .. import _native

MEASURE_NAME = "readLatency"
MEASURE_DESCRIPTION = "Complete read latency"
MEASURE_UNIT = "ms"
VIEW_NAME = "princer_go_client_read_latency"
VIEW_DESCRIPTION = "Complete read latency for a given go-client"
TAG_KEY = "princer_read_latency"
METRIC_PREFIX = "custom.googleapis.com/custom-go-client/"
REPORTING_INTERVAL_S = 30.0
# ochttp.DefaultLatencyDistribution (ms) — also the C++ runner's buckets
BUCKET_BOUNDS_MS = list(_native.oc_latency_bounds_ms())


@dataclass
class Distribution:
    bucket_counts: list[int] = field(default_factory=lambda: [0] * (len(BUCKET_BOUNDS_MS) + 1))
    count: int = 0
    sum_ms: float = 0.0

    @property
    def mean(self) -> float:
        return self.sum_ms / self.count if self.count else 0.0


@dataclass
class View:
    name: str = VIEW_NAME
    description: str = VIEW_DESCRIPTION
    measure: str = MEASURE_NAME
    unit: str = MEASURE_UNIT
    tag_keys: tuple = (TAG_KEY,)
    bounds: tuple = tuple(BUCKET_BOUNDS_MS)


_registered: dict[str, View] = {}


def register_latency_view() -> View:
    """Mirror of registerLatencyView(); idempotent."""
    v = View()
    _registered[v.name] = v
    return v


def bucket_index(ms: float) -> int:
    """OpenCensus bucketing: i such that bounds[i-1] <= ms < bounds[i]."""
    return _native.oc_bucket_index(float(ms))


def prometheus_text(view: View, dist: Distribution, labels: dict[str, str] | None = None) -> str:
    lab = dict(labels or {})
    lab.setdefault(TAG_KEY, "")

    def fmt(extra: dict[str, str]) -> str:
        items = {**lab, **extra}
        return "{" + ",".join(f'{k}="{v}"' for k, v in items.items()) + "}"

    lines = [f"# HELP {view.name} {view.description}", f"# TYPE {view.name} histogram"]
    cum = 0
    for b, c in zip(view.bounds, dist.bucket_counts):
        cum += c
        lines.append(f"{view.name}_bucket{fmt({'le': f'{b:g}'})} {cum}")
    cum += dist.bucket_counts[-1]
    lines.append(f"{view.name}_bucket{fmt({'le': '+Inf'})} {cum}")
    lines.append(f"{view.name}_sum{fmt({})} {dist.sum_ms:.6f}")
    lines.append(f"{view.name}_count{fmt({})} {dist.count}")
    return "\n".join(lines) + "\n"


def timeseries_record(view: View, dist: Distribution, project: str, start_time: float,
                      labels: dict[str, str] | None = None) -> dict:
    """A Cloud Monitoring TimeSeries-shaped record (what Stackdriver would get)."""
    return {
        "metric": {"type": METRIC_PREFIX + view.name, "labels": {TAG_KEY: "", **(labels or {})}},
        "resource": {"type": "global", "labels": {"project_id": project}},
        "metricKind": "CUMULATIVE",
        "valueType": "DISTRIBUTION",
        "points": [{
            "interval": {"startTime": start_time, "endTime": time.time()},
            "value": {"distributionValue": {
                "count": dist.count,
                "mean": dist.mean,
                "bucketOptions": {"explicitBuckets": {"bounds": list(view.bounds)}},
                "bucketCounts": list(dist.bucket_counts),
            }},
        }],
    }


class MetricsExporter:
    """Periodic exporter; `source()` returns the current cumulative Distribution."""

    def __init__(self, source: Callable[[], Distribution], project: str, prom_file: str = "",
                 jsonl_file: str = "", http_port: int = 0, interval_s: float = REPORTING_INTERVAL_S,
                 labels: dict[str, str] | None = None):
        self.view = _registered.get(VIEW_NAME) or register_latency_view()
        self.source = source
        self.project = project
        self.prom_file = prom_file
        self.jsonl_file = jsonl_file
        self.interval_s = interval_s
        self.labels = labels or {}
        self.start_time = time.time()
        self.exports = 0
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self._prom_metric = None
        if http_port:
            self._start_http(http_port)

    def _start_http(self, port: int):
        import prometheus_client as pc

        reg = pc.CollectorRegistry()
        exporter = self

        class _Collector:
            def collect(self):
                from prometheus_client.core import HistogramMetricFamily

                d = exporter.source()
                cum, buckets = 0, []
                for b, c in zip(exporter.view.bounds, d.bucket_counts):
                    cum += c
                    buckets.append((f"{b:g}", cum))
                buckets.append(("+Inf", cum + d.bucket_counts[-1]))
                h = HistogramMetricFamily(exporter.view.name, exporter.view.description, labels=[TAG_KEY])
                h.add_metric([""], buckets, d.sum_ms)
                yield h

        reg.register(_Collector())
        pc.start_http_server(port, addr="127.0.0.1", registry=reg)

    def start(self) -> "MetricsExporter":
        self._thread = threading.Thread(target=self._loop, name="metrics-exporter", daemon=True)
        self._thread.start()
        return self

    def _loop(self):
        while not self._stop.wait(self.interval_s):
            self.export_once()

    def export_once(self):
        d = self.source()
        if self.prom_file:
            tmp = self.prom_file + ".tmp"
            with open(tmp, "w") as f:
                f.write(prometheus_text(self.view, d, self.labels))
            os.replace(tmp, self.prom_file)
        if self.jsonl_file:
            with open(self.jsonl_file, "a") as f:
                f.write(json.dumps(timeseries_record(self.view, d, self.project, self.start_time, self.labels)) + "\n")
        self.exports += 1

    def close(self):
        """Stop the periodic loop and flush once (reference Q2: this was a no-op)."""
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)
        self.export_once()


def distribution_from_summary(summary: dict) -> Distribution:
    d = Distribution()
    d.bucket_counts = list(summary["oc_buckets"])
    d.count = sum(d.bucket_counts)
    # the runner records integer-truncated ms into the buckets; the mean uses
    # the measured float latencies
    d.sum_ms = summary["avg_ms"] * d.count
    return d


def write_once(dist: Distribution, project: str, prom_file: str = "", jsonl_file: str = "",
               labels: dict[str, str] | None = None, start_time: float | None = None) -> None:
    """One export of `dist` (e.g. the node-level view rank 0 writes after the
    per-rank histograms were summed over RCCL, parallel/dist.py R3)."""
    view = _registered.get(VIEW_NAME) or register_latency_view()
    if prom_file:
        tmp = prom_file + ".tmp"
        with open(tmp, "w") as f:
            f.write(prometheus_text(view, dist, labels))
        os.replace(tmp, prom_file)
    if jsonl_file:
        with open(jsonl_file, "a") as f:
            f.write(json.dumps(timeseries_record(view, dist, project, start_time or time.time(), labels)) + "\n")


def node_distribution(ctx, local: Distribution) -> Distribution:
    """Sum a rank's distribution over all ranks (collective: every rank calls
    it).  One node-level distribution, like the reference's single process
    exports (metrics_exporter.go:22-34), out of one histogram per GPU rank."""
    from ..parallel import dist as gdist

    counts = gdist.reduce_histogram(ctx, list(local.bucket_counts) + [local.count])
    st = gdist.reduce_stats(ctx, sum_ms=float(local.sum_ms))
    d = Distribution()
    d.bucket_counts = counts[:-1]
    d.count = counts[-1]
    d.sum_ms = st["sum_ms_sum"]
    return d
