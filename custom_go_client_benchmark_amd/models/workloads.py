"""Workload drivers on top of the native runner / client.

All byte movement happens in C++ (csrc/bench/runner.cc, csrc/storage/*,
csrc/gpu/engine.hip) with the GIL released; this module wires options,
drains per-read records for the exporters, and gathers results.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field
from typing import Callable

from .. import _native
from ..utils import cpuacct


@dataclass
class RunOptions:
    protocol: str = "http"                 # http | http2 | grpc (reference: -client-protocol)
    endpoint: str = "http://127.0.0.1:8080"
    bucket: str = "princer-working-dirs"   # reference main.go:44
    object_prefix: str = "princer_100M_files/file_"  # reference main.go:52
    object_suffix: str = ""
    workers: int = 48                      # reference main.go:36
    reads_per_worker: int = 1000000        # reference main.go:38
    duration_s: float = 0.0
    worker_id_offset: int = 0
    http_api: str = "xml"
    read_chunk: int = 2 << 20
    max_conns_per_host: int = 100
    grpc_conn_pool_size: int = 1
    sink: str = "discard"                  # discard | gpu
    host_crc: bool = True
    device: int = 0
    ring_slot_bytes: int = 8 << 20
    ring_slots: int = 4
    landing: str = "object"
    gpu_verify: bool = True
    latency_fd: int = -1
    trace_sample_rate: float = 0.0
    stop_on_error: bool = True
    cpus: list = field(default_factory=list)
    reader_cpus: list = field(default_factory=list)  # multiplexed connections' reader threads (empty = cpus)
    rcvbuf: int = 0                        # client SO_RCVBUF (0 = kernel autotuning, as the Go client)
    auth: str = "none"                     # none | static | adc | key_file
    token: str = ""
    key_file: str = ""
    token_uri: str = ""
    user_agent: str = "prince"
    tls_ca_file: str = ""
    tls_verify: bool = True
    retry_initial_s: float = 1.0
    retry_max_s: float = 30.0
    retry_multiplier: float = 2.0
    retry_max_total_s: float = 0.0
    retry_max_attempts: int = 0
    read_timeout_s: float = 0.0            # idle limit per read (0 = none, as the reference's Timeout: 0)
    tcp_congestion: str = ""               # client sockets' congestion control ("" = host default)
    loopback_rto_min: bool = False         # node-local endpoint: loopback-sized minimum RTO
    conn_ring: bool = True                 # GPU sink on one multiplexed connection: one shared receive ring
    object_names: list | None = None
    keep_records: bool = True
    slices: int = 1                        # >1: sliced (parallel ranged) reads, see csrc/storage/sliced.h
    slice_min_bytes: int = 8 << 20
    slice_piece_bytes: int = 8 << 20       # sliced reads: dynamic pieces (0 = fixed shares)
    slice_piece_min_bytes: int = 0         # >0: taper pieces toward the end down to this

    def client_dict(self) -> dict:
        return {
            "protocol": self.protocol, "endpoint": self.endpoint, "http_api": self.http_api,
            "read_chunk": self.read_chunk, "max_conns_per_host": self.max_conns_per_host,
            "max_idle_conns_per_host": self.max_conns_per_host, "grpc_conn_pool_size": self.grpc_conn_pool_size,
            "auth": self.auth, "token": self.token, "key_file": self.key_file, "token_uri": self.token_uri,
            "user_agent": self.user_agent, "retry_initial_s": self.retry_initial_s, "retry_max_s": self.retry_max_s,
            "retry_multiplier": self.retry_multiplier, "retry_max_total_s": self.retry_max_total_s,
            "retry_max_attempts": self.retry_max_attempts, "cpus": list(self.cpus),
            "reader_cpus": list(self.reader_cpus) or None,
            "rcvbuf": int(self.rcvbuf),
            "io_timeout_ms": int(round(self.read_timeout_s * 1000)),
            "tls_ca_file": self.tls_ca_file, "tls_verify": self.tls_verify,
            "tcp_congestion": self.tcp_congestion,
            "loopback_rto_min": self.loopback_rto_min,
        }

    def runner_dict(self) -> dict:
        d = self.client_dict()
        d.update({
            "bucket": self.bucket, "object_prefix": self.object_prefix, "object_suffix": self.object_suffix,
            "workers": self.workers, "reads_per_worker": self.reads_per_worker, "duration_s": self.duration_s,
            "worker_id_offset": self.worker_id_offset, "sink": self.sink, "host_crc": self.host_crc,
            "device": self.device, "ring_slot_bytes": self.ring_slot_bytes, "ring_slots": self.ring_slots,
            "landing": self.landing, "gpu_verify": self.gpu_verify, "latency_fd": self.latency_fd,
            "trace_sample_rate": self.trace_sample_rate, "stop_on_error": self.stop_on_error,
            "keep_records": self.keep_records, "slices": self.slices, "slice_min_bytes": self.slice_min_bytes,
            "slice_piece_bytes": self.slice_piece_bytes,
            "slice_piece_min_bytes": self.slice_piece_min_bytes, "conn_ring": self.conn_ring,
        })
        if self.object_names:
            d["object_names"] = list(self.object_names)
        return d


@dataclass
class WorkloadResult:
    summary: dict
    records_seen: int = 0
    extra: dict = field(default_factory=dict)

    @property
    def ok(self) -> bool:
        return self.summary.get("errors", 0) == 0


def _drive(runner, on_records: Callable[[list], None] | None, poll_s: float = 0.2,
           before_start: Callable[[], None] | None = None) -> int:
    """Starts the runner, drains records until it finishes. Returns #records."""
    if before_start:
        before_start()
    runner.start()
    done = threading.Event()

    def waiter():
        runner.wait()
        done.set()

    t = threading.Thread(target=waiter, name="runner-wait", daemon=True)
    t.start()
    seen = 0
    try:
        while not done.wait(poll_s):
            recs = runner.drain()
            seen += len(recs)
            if on_records and recs:
                on_records(recs)
    except KeyboardInterrupt:
        runner.stop()
        done.wait()
    recs = runner.drain()
    seen += len(recs)
    if on_records and recs:
        on_records(recs)
    t.join()
    return seen


def run_read(opts: RunOptions, on_records=None, before_start=None) -> WorkloadResult:
    runner = _native.Runner(opts.runner_dict())
    seen = _drive(runner, on_records, before_start=before_start)
    return WorkloadResult(runner.summary(), seen)


def run_list_read(opts: RunOptions, prefix: str, on_records=None, before_start=None,
                  page_size: int = 1000) -> WorkloadResult:
    """Config 3: list `prefix`, then read every listed object once per pass."""
    client = _native.Client(opts.client_dict())
    t0 = time.perf_counter()
    objs = client.list_all(opts.bucket, prefix, page_size)
    list_ms = (time.perf_counter() - t0) * 1e3
    if not objs:
        raise RuntimeError(f"no objects under gs://{opts.bucket}/{prefix}")
    names = [o["name"] for o in objs]
    o2 = RunOptions(**{**opts.__dict__})
    o2.object_names = names
    # every worker reads a disjoint stride of the listing; one pass reads all
    passes = max(1, opts.reads_per_worker)
    o2.reads_per_worker = passes * ((len(names) + opts.workers - 1) // opts.workers)
    runner = _native.Runner(o2.runner_dict())
    seen = _drive(runner, on_records, before_start=before_start)
    return WorkloadResult(runner.summary(), seen, {"listed": len(names), "list_ms": list_ms,
                                                   "list_bytes": sum(int(o["size"]) for o in objs)})


def run_write(opts: RunOptions, nobjects: int, size: int, name_prefix: str = "upload/obj_",
              resumable: bool = True, chunk_bytes: int = 16 << 20, verify_readback: bool = False,
              warmup: int = 1) -> WorkloadResult:
    """Config 5: objects generated in HBM (K3 fill kernel), staged HBM ->
    pinned (D2H on a side stream), uploaded via a resumable session (HTTP) or
    StartResumableWrite + WriteObject (gRPC); the server checks CRC32C."""
    import torch

    client = _native.Client(opts.client_dict())
    # slices > 1: parallel composite upload (parts on their own connections,
    # composed server-side; csrc/storage/sliced.h SlicedWriter)
    writer = _native.SlicedWriter({**opts.client_dict(), "slices": opts.slices,
                                   "slice_min_bytes": opts.slice_min_bytes}) if opts.slices > 1 else None
    dev = opts.device
    buf = torch.empty(size, dtype=torch.uint8, device=f"cuda:{dev}")
    # untimed warm-up uploads: connections, pinned staging rings (PinnedPool)
    for i in range(warmup):
        wname = f"{name_prefix}warmup_{opts.worker_id_offset}_{i}"
        _native.gpu_fill_pattern(dev, buf.data_ptr(), size, wname, 0)
        if writer is not None:
            writer.write_from_device(opts.bucket, wname, buf.data_ptr(), size, dev, resumable, chunk_bytes,
                                     opts.ring_slot_bytes, opts.ring_slots)
        else:
            client.write_from_device(opts.bucket, wname, buf.data_ptr(), size, dev, resumable, chunk_bytes,
                                     opts.ring_slot_bytes, opts.ring_slots)
    lat = []
    setup = []
    total = 0
    th0 = cpuacct.thread_cpu()
    t_all = time.perf_counter()
    for i in range(nobjects):
        gid = opts.worker_id_offset + i
        name = f"{name_prefix}{gid}"
        _native.gpu_fill_pattern(dev, buf.data_ptr(), size, name, 0)
        t0 = time.perf_counter()
        if writer is not None:
            m = writer.write_from_device(opts.bucket, name, buf.data_ptr(), size, dev, resumable, chunk_bytes,
                                         opts.ring_slot_bytes, opts.ring_slots)
            lat.append((time.perf_counter() - t0) * 1e3)
            # SlicedWriter already checked the composed CRC32C against the
            # combine of the parts' GPU CRCs
            if m["size"] != size:
                raise RuntimeError(f"upload of {name} not confirmed: {m}")
        else:
            m = client.write_from_device(opts.bucket, name, buf.data_ptr(), size, dev, resumable, chunk_bytes,
                                         opts.ring_slot_bytes, opts.ring_slots)
            lat.append((time.perf_counter() - t0) * 1e3)
            setup.append(m["gpu_crc_ms"])
            if m["size"] != size or m["crc32c"] != m["gpu_crc32c"]:
                raise RuntimeError(f"upload of {name} not confirmed: {m}")
        total += size
        if verify_readback:
            got = client.read(opts.bucket, name)
            if not got["verified"]:
                raise RuntimeError(f"read-back of {name} failed CRC32C")
    elapsed = time.perf_counter() - t_all
    s = sorted(lat)

    def pct(p):
        return s[min(len(s) - 1, len(s) * p // 100)] if s else 0.0

    summary = {"reads": 0, "writes": nobjects, "warmup_writes": warmup, "errors": 0, "bytes": total,
               "elapsed_s": elapsed,
               "mib_per_s": total / elapsed / 2**20 if elapsed else 0.0, "p50_ms": pct(50), "p99_ms": pct(99),
               "min_ms": s[0] if s else 0.0, "max_ms": s[-1] if s else 0.0, "avg_ms": sum(s) / len(s) if s else 0.0}
    summary["gpu_setup_p50_ms"] = sorted(setup)[len(setup) // 2] if setup else 0.0  # staging ring + GPU CRC32C
    summary["cpu_s_per_gib_by_thread"] = cpuacct.per_gib(cpuacct.delta_by_group(th0, cpuacct.thread_cpu()), total)
    return WorkloadResult(summary, 0, {"latencies_ms": lat})
