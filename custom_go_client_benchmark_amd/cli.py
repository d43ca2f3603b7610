"""`gcsbench` — the benchmark CLI (reference main.go:158-220).

Keeps the reference's flags, defaults and usage strings (main.go:36-57):

    -worker 48  -read-call-per-worker 1000000  -bucket princer-working-dirs
    -project gcs-fuse-test  -client-protocol http  -enable-tracing=false
    -trace-sample-rate 1.0

and its output contract as the reference's drivers expect it: one latency
line per read on stdout ("12.345ms", so execute_pb.sh's `tr 'ms' ' '` turns
it into a float the README histogram script can read), all
status text on stderr.  Everything else is additive (endpoint, object naming,
GPU sink, exporters, auth, retry knobs, multi-GPU).

Fixed reference quirks: Q1 client-creation errors exit 1;
Q2 the metric exporter flushes on exit; Q3 no shared error variable; Q9
-client-protocol must be http|http2|grpc; Q11 first error cancels the other
workers; Q12 optional -duration bound.

Multi-GPU: launch with torchrun, one rank per GPU; rank r's workers read
file_<r*W + w>; RCCL barriers bracket the timed region and a stats
all-reduce produces the node view (parallel/dist.py).
"""
from __future__ import annotations

import json
import os
import sys
import time

from . import _native
from .models import workloads
from .utils import cpuacct, metrics_exporter, trace_exporter
from .utils.goflags import FlagSet


def build_flags() -> FlagSet:
    fs = FlagSet("gcsbench")
    # --- reference flags (main.go:36-57), same names/defaults/usage -------------
    fs.int("worker", 48, "Number of concurrent worker to read")
    fs.int("read-call-per-worker", 1000000, "Number of read call per worker")
    fs.string("bucket", "princer-working-dirs", "GCS bucket name.")
    fs.string("project", "gcs-fuse-test", "GCP project name.")
    fs.string("client-protocol", "http", "Network protocol.")
    fs.bool("enable-tracing", False, "Enable tracing with Cloud Trace export")
    fs.float("trace-sample-rate", 1.0, "Sampling rate for Cloud Trace")
    # --- additive ---------------------------------------------------------------
    fs.string("endpoint", "", "Storage endpoint URL (default $GCSB_ENDPOINT or $STORAGE_EMULATOR_HOST)")
    fs.string("object-prefix", "princer_100M_files/file_", "Object name = prefix + worker id + suffix")
    fs.string("object-suffix", "", "Object name suffix")
    fs.string("workload", "read", "read | list-read | write")
    fs.string("list-prefix", "", "list-read: prefix to list (default: -object-prefix)")
    fs.int("write-objects", 1, "write: objects per rank")
    fs.int("write-size", 64 << 20, "write: object size in bytes")
    fs.bool("resumable", True, "write: resumable session (HTTP) / StartResumableWrite (gRPC)")
    fs.int("write-warmup", 1, "write: untimed warm-up uploads first (connections, pinned staging rings)")
    fs.string("http-api", "xml", "HTTP media API: xml (library default) | json (alt=media)")
    fs.int("read-chunk", 2 << 20, "Bytes per receive into the sink (reference intent: 2 MiB buffer)")
    fs.bool("conn-ring", True, "-sink gpu on one multiplexed connection (gRPC pool 1, http2): every worker's stream "
            "lands through one 4 x 1 MiB receive ring of the connection instead of a ring per worker "
            "(profiles/r4_ringgeom)")
    fs.int("rcvbuf", 0, "Client SO_RCVBUF in bytes (0 = kernel autotuning, as the Go client; the bench's headline "
           "and list-read request 64 MiB, capped by net.core.rmem_max)")
    fs.int("grpc-conn-pool-size", 1, "gRPC connections (reference GrpcConnPoolSize = 1)")
    fs.bool("grpc-directpath", True, "Request DirectPath while creating the gRPC client (reference sets "
            "GOOGLE_CLOUD_ENABLE_DIRECT_PATH_XDS=true around NewGRPCClient; falls back to CloudPath)")
    fs.int("max-conns-per-host", 100, "HTTP connection cap (reference MaxConnsPerHost = 100)")
    fs.string("sink", "discard", "discard (reference io.Discard) | gpu (pinned ring -> HBM, CRC32C on GPU)")
    fs.int("gpu-device", -1, "HIP device (default: LOCAL_RANK)")
    fs.int("ring-slot-bytes", 0, "Pinned ring slot size (0 = auto: 2 MiB for one worker, 1 MiB for several)")
    fs.int("ring-slots", 0, "Pinned ring slots per worker (0 = auto: 8 for one worker, 2 for several: the "
           "workers' receive destinations stay within an L3, profiles/r3_mux_thp/listring)")
    fs.string("landing", "object", "object (whole object in HBM) | ring (HBM ring, discard semantics)")
    fs.bool("gpu-verify", True, "Verify CRC32C with the GPU kernels")
    fs.int("slices", 1, "Sliced reads: N concurrent ranged streams per object, each on its own connection "
           "(1 = one stream per read, as the reference)")
    fs.int("slice-min-bytes", 8 << 20, "Smallest slice; smaller objects use fewer slices")
    fs.int("slice-piece-bytes", 8 << 20, "Sliced reads: streams pull pieces of this size from a shared cursor "
           "(dynamic load balance; 0 = one fixed share per stream)")
    fs.int("slice-piece-min-bytes", 0, "Sliced reads: taper pieces toward the end of the object down to this "
           "(guided self-scheduling; 0 = fixed-size pieces)")
    fs.bool("host-crc", True, "discard sink: verify CRC32C on the host (what the Go library does)")
    fs.duration("duration", 0.0, "Stop after this long (0 = only -read-call-per-worker)")
    fs.string("latency-file", "", "Write per-read latency lines here instead of stdout")
    fs.string("metrics-file", "", "Prometheus text file for the read-latency view")
    fs.string("metrics-jsonl", "", "Cloud-Monitoring-shaped JSONL time series file")
    fs.int("metrics-port", 0, "Serve the view on 127.0.0.1:<port>/metrics")
    fs.duration("metrics-interval", metrics_exporter.REPORTING_INTERVAL_S, "Export interval (reference: 30s)")
    fs.string("trace-file", "traces.jsonl", "OTLP/JSON span batches (with -enable-tracing)")
    fs.string("auth", "none", "none | static | adc | key_file")
    fs.string("token", "", "Bearer token for -auth static")
    fs.string("key-file", "", "Service-account JSON key (-auth key_file)")
    fs.string("token-uri", "", "Override the key file's token_uri")
    fs.string("user-agent", "prince", "User-Agent (reference userAgentRoundTripper)")
    fs.string("tcp-congestion", "", "Client sockets' TCP congestion control, set before connect (\"\" = the "
              "host default; with -start-fake-server: cubic, which avoids BBR's per-skb pacing timers on a "
              "loopback link)")
    fs.string("tls-ca-file", "", "PEM CA bundle for https endpoints (default: system roots)")
    fs.bool("tls-insecure", False, "Skip TLS certificate verification (test endpoints only)")
    fs.duration("retry-initial", 1.0, "Initial backoff (gax default 1s)")
    fs.duration("retry-max", 30.0, "Max backoff (reference MaxRetryDuration 30s)")
    fs.float("retry-multiplier", 2.0, "Backoff multiplier (reference RetryMultiplier 2)")
    fs.duration("retry-max-total", 0.0, "Give up retrying after this long (0 = never, as the reference)")
    fs.int("retry-max-attempts", 0, "Give up after this many attempts (0 = unlimited)")
    fs.duration("read-timeout", 0.0, "Fail an attempt (retryably) when no byte arrives for this long; the read "
                "resumes at the delivered offset (0 = none, as the reference's http.Client Timeout 0)")
    fs.string("affinity", "auto", "CPU placement: auto | quota | share | same | split | numa | none")
    fs.bool("start-fake-server", False, "Start a node-local synthetic GCS endpoint (no network)")
    fs.int("fake-object-size", 100 << 20, "Synthetic object size (reference objects are ~100 MB)")
    fs.int("fake-objects", -1, "Synthetic objects per rank (default: -worker)")
    fs.bool("fake-retain-uploads", True, "Synthetic endpoint keeps uploaded bytes (false: verifies size + CRC32C "
            "and keeps metadata only, the server-side io.Discard for write benchmarks)")
    fs.string("summary-json", "", "Write the run summary (p50/p99/MiB/s, node view) as JSON here")
    return fs


def _err(msg: str):
    sys.stderr.write(msg.rstrip("\n") + "\n")
    sys.stderr.flush()


def auto_affinity(sink: str, proto: str, workers: int, pool: int, slices: int, workload: str) -> str:
    """`-affinity auto`: the CPU placement (parallel/affinity.py plan mode).

    - GPU sink: one reader with one stream per read gets the bench's
      placement, a quiet core each for the receive thread, the endpoint and
      the GPU submitter (profiles/r2_placement). Several readers share one L3
      domain; sliced reads spread over the rank's share.
    - Discard sink, gRPC / HTTP/2 with more workers than connections: each
      connection's one reader copies every byte, and its receive copy, the
      workers' CRC passes and the endpoint's sends want one L3 domain
      (48 x 1 MiB gRPC: 16.0-19.5k MiB/s against 8.4-8.8k over the quota's
      cores, profiles/r3_mux_thp/refplace).
    - Other discard-sink runs: no GPU to be near; under a CPU quota the threads
      keep to as many cores as the quota pays for.
    - Uploads from HBM (spliced send, endpoint CRC on its write worker): three
      quiet cores of one L3 domain -- the uploader, the endpoint's receive
      thread, its CRC worker -- 18.0-21.6k MiB/s against 7.7-19.7k with the
      threads spread (profiles/r3_write/placement); composite uploads
      (slices > 1) and CPU-only uploads stay unpinned (profiles/r1_session4/).
    """
    if workload == "write":
        return "pair" if sink == "gpu" and slices <= 1 else "none"
    if sink == "gpu":
        return "share" if slices > 1 else ("pair" if workers == 1 else "same")
    if proto in ("grpc", "http2") and workers > max(1, pool):
        return "same"
    return "quota"


def auto_ring(workers: int, slices: int) -> tuple[int, int]:
    """(slot bytes, slots) of each GPU sink's pinned ring when the flags are 0.

    The receive copy write-allocates its destination, so the rings' total
    footprint matters: a 32 MiB ring cost one receiving core 25-35%
    (profiles/r3_ring_thp). One worker gets the headline's 4 x 1 MiB: the copy
    engine then reads lines still in the receiving CCD's L3, which took the
    receive copy from 0.046 to 0.036 CPU-s/GiB and 22.0k to 27.5k MiB/s
    against 8 x 2 MiB (profiles/r4_main8, r4_recvcost); several
    get 2 x 1 MiB each (8 list-readers: 18.6-18.8k MiB/s against 15.5-17.0k
    with 8 x 2 MiB, profiles/r3_mux_thp/listring); sliced reads 2 x 2 MiB per
    slice sink (profiles/r3_ring_thp/sliced)."""
    if slices > 1:
        return 2 << 20, 2
    if workers == 1:
        return 1 << 20, 4
    return 1 << 20, 2


def main(argv: list[str] | None = None) -> int:
    fs = build_flags().parse(sys.argv[1:] if argv is None else argv)
    proto = fs.get("client-protocol")
    if proto not in ("http", "http2", "grpc"):  # Q9
        _err(f'invalid -client-protocol "{proto}": want http, http2 or grpc')
        return 2
    if fs.get("worker") <= 0:
        _err("worker count not valid")
        return 2

    from .parallel import dist

    rank, world, local_rank = dist.env_rank()
    ctx = None
    sink = fs.get("sink")
    device = fs.get("gpu-device") if fs.get("gpu-device") >= 0 else local_rank
    if world > 1 or sink == "gpu":
        ctx = dist.init(local_rank=local_rank, world=world, rank=rank)
        if fs.get("gpu-device") < 0 and ctx.gpu >= 0:
            device = ctx.gpu
    workers = fs.get("worker")
    first = rank * workers

    placement = {"client": [], "server": []}
    aff = fs.get("affinity")
    if aff == "auto":
        aff = auto_affinity(sink, proto, workers, fs.get("grpc-conn-pool-size"), fs.get("slices"), fs.get("workload"))
    if aff != "none" and (sink == "gpu" or aff in ("quota", "same")):
        from .parallel import affinity

        try:
            placement = affinity.plan(device, aff)
        except Exception:  # noqa: BLE001 - no GPU to place near (CPU-only host): the quota's cores
            if sink == "gpu":
                raise
            placement = affinity.plan(device, "quota")
        if (aff == "same" and proto in ("grpc", "http2") and workers > max(1, fs.get("grpc-conn-pool-size"))
                and fs.get("workload") != "write"):
            # the connection's one reader and (a node-local endpoint's) send
            # thread on a physical core each: ref_default_grpc 21.1k -> 24.2k
            # MiB/s in the bench (profiles/r5_muxiso)
            placement = affinity.isolate_reader(placement)
            if fs.get("start-fake-server"):
                placement = affinity.isolate_sender(placement)
            if sink == "gpu" and placement.get("reader_cpus"):
                # the GPU hand-off thread with the workers, off the reader's core
                _native.set_submitter_cpus(placement["client"])
        if fs.get("workload") == "write" and aff == "pair":
            # the endpoint's receive thread and CRC worker get a core each;
            # this (uploading) thread the client core
            placement = {**placement, "server": sorted(placement["server"] + placement.get("aux", []))}
            if placement["client"]:
                os.sched_setaffinity(0, placement["client"])
        elif placement.get("aux"):
            _native.set_submitter_cpus(placement["aux"])

    endpoint = fs.get("endpoint") or os.environ.get("GCSB_ENDPOINT", "") or os.environ.get("STORAGE_EMULATOR_HOST", "")
    ep_handle = None
    if fs.get("start-fake-server"):
        from . import server

        n_obj = fs.get("fake-objects") if fs.get("fake-objects") >= 0 else workers
        ep_handle = server.start_inprocess(fs.get("bucket"), fs.get("object-prefix"), fs.get("object-suffix"), first,
                                           n_obj, fs.get("fake-object-size"), md5=True, cpus=placement["server"],
                                           retain_uploads=fs.get("fake-retain-uploads"),
                                           send_cpus=placement.get("send_cpus"))
        endpoint = ep_handle.url
        _err(f"synthetic GCS endpoint {endpoint}: {n_obj} objects of {fs.get('fake-object-size')} bytes")
    if not endpoint:
        _err("while creating the client: no endpoint (set -endpoint, $GCSB_ENDPOINT or -start-fake-server; "
             "this environment has no network)")
        return 1
    if endpoint and "://" not in endpoint:
        endpoint = "http://" + endpoint

    latency_fd = 1
    lat_file = None
    lat_path = fs.get("latency-file")
    if lat_path:
        if world > 1:  # one file per rank; scripts/merge_latency.py gives exact node percentiles
            root, ext = os.path.splitext(lat_path)
            lat_path = f"{root}.rank{rank}{ext}"
        lat_file = open(lat_path, "w")
        latency_fd = lat_file.fileno()
    sys.stdout.flush()

    auto_bytes, auto_slots = auto_ring(workers, fs.get("slices"))
    ring_slot_bytes = fs.get("ring-slot-bytes") or auto_bytes
    ring_slots = fs.get("ring-slots") or auto_slots
    opts = workloads.RunOptions(
        protocol=proto, endpoint=endpoint, bucket=fs.get("bucket"), object_prefix=fs.get("object-prefix"),
        object_suffix=fs.get("object-suffix"), workers=workers, reads_per_worker=fs.get("read-call-per-worker"),
        duration_s=fs.get("duration"), worker_id_offset=first, http_api=fs.get("http-api"),
        read_chunk=fs.get("read-chunk"), max_conns_per_host=fs.get("max-conns-per-host"),
        grpc_conn_pool_size=fs.get("grpc-conn-pool-size"), sink=sink, host_crc=fs.get("host-crc"), device=device,
        ring_slot_bytes=ring_slot_bytes, ring_slots=ring_slots, landing=fs.get("landing"),
        gpu_verify=fs.get("gpu-verify"), latency_fd=latency_fd, slices=fs.get("slices"),
        slice_min_bytes=fs.get("slice-min-bytes"), slice_piece_bytes=fs.get("slice-piece-bytes"),
        slice_piece_min_bytes=fs.get("slice-piece-min-bytes"),
        trace_sample_rate=fs.get("trace-sample-rate") if fs.get("enable-tracing") else 0.0,
        cpus=placement["client"], reader_cpus=placement.get("reader_cpus") or [], rcvbuf=fs.get("rcvbuf"),
        auth=fs.get("auth"), token=fs.get("token"), key_file=fs.get("key-file"),
        token_uri=fs.get("token-uri"), user_agent=fs.get("user-agent"), tls_ca_file=fs.get("tls-ca-file"),
        tls_verify=not fs.get("tls-insecure"), retry_initial_s=fs.get("retry-initial"),
        retry_max_s=fs.get("retry-max"), retry_multiplier=fs.get("retry-multiplier"),
        retry_max_total_s=fs.get("retry-max-total"), retry_max_attempts=fs.get("retry-max-attempts"),
        read_timeout_s=fs.get("read-timeout"),
        # a node-local synthetic endpoint is a loopback link: cubic unless set
        tcp_congestion=fs.get("tcp-congestion") or ("cubic" if fs.get("start-fake-server") else ""),
        loopback_rto_min=bool(fs.get("start-fake-server")), conn_ring=bool(fs.get("conn-ring")))

    # tracing (reference main.go:162-165)
    tracer, trace_cleanup = None, None
    if fs.get("enable-tracing"):
        path = fs.get("trace-file")
        if world > 1:
            root, ext = os.path.splitext(path)
            path = f"{root}.rank{rank}{ext or '.jsonl'}"
        tracer, trace_cleanup = trace_exporter.enable_trace_export(path, proto, fs.get("bucket"), gpu=sink == "gpu")
        _err(f"trace export enabled -> {path} (sample rate {fs.get('trace-sample-rate')})")

    # metrics view + exporter (reference main.go:190-197)
    metrics_exporter.register_latency_view()
    live = {"summary": None, "runner": None}

    def source():
        # the exporter's 30 s tick: counts + OC buckets only (percentiles
        # would sort every sample under the lock the workers record into)
        r = live["runner"]
        s = r.summary(False) if r is not None else live["summary"]
        return metrics_exporter.distribution_from_summary(s) if s else metrics_exporter.Distribution()

    exporter = None
    if fs.get("metrics-file") or fs.get("metrics-jsonl") or fs.get("metrics-port"):
        sfx = f".rank{rank}" if world > 1 else ""
        exporter = metrics_exporter.MetricsExporter(
            source, fs.get("project"),
            prom_file=(fs.get("metrics-file") + sfx) if fs.get("metrics-file") else "",
            jsonl_file=(fs.get("metrics-jsonl") + sfx) if fs.get("metrics-jsonl") else "",
            http_port=fs.get("metrics-port") + (local_rank if fs.get("metrics-port") else 0),
            interval_s=fs.get("metrics-interval"), labels={"rank": str(rank)} if world > 1 else None).start()
        _err("metrics exporter started successfully")

    def before_start():
        if ctx is not None:
            dist.barrier(ctx, "R1 start barrier")  # synchronized start

    def on_records(recs):
        if tracer:
            tracer.on_records(recs)

    t0 = time.perf_counter()
    cg0 = cpuacct.cgroup_cpu_stat()
    th0 = cpuacct.thread_cpu()
    rc = 0
    try:
        wl = fs.get("workload")
        if wl == "read":
            res = _run_with_live(opts, on_records, before_start, live, fs.get("grpc-directpath"))
        elif wl == "list-read":
            res = workloads.run_list_read(opts, fs.get("list-prefix") or fs.get("object-prefix"), on_records,
                                          before_start)
        elif wl == "write":
            before_start()
            res = workloads.run_write(opts, fs.get("write-objects"), fs.get("write-size"),
                                      resumable=fs.get("resumable"), warmup=fs.get("write-warmup"))
        else:
            _err(f"unknown -workload {wl}")
            return 2
        live["summary"] = res.summary
    except _native.StorageError as e:
        _err(f"while creating the client: {e}")
        return 1
    finally:
        if ctx is not None:
            try:
                dist.barrier(ctx, "R2 stop barrier")  # synchronized stop
            except Exception:
                pass
    wall = time.perf_counter() - t0
    s = res.summary
    s.update(cpuacct.cgroup_delta(cg0, cpuacct.cgroup_cpu_stat()))
    s["cpu_s_by_group"] = {k: round(v, 4) for k, v in
                           cpuacct.delta_by_group(th0, cpuacct.thread_cpu()).items()}
    if exporter:
        exporter.close()  # flushes (reference Q2)
    if trace_cleanup:
        trace_cleanup()
    if lat_file:
        lat_file.close()

    # node-level latency distribution (R3): the per-rank histograms summed
    # over the process group; rank 0 exports it under the un-suffixed names
    if exporter and ctx is not None and ctx.world > 1 and "oc_buckets" in s:
        node = metrics_exporter.node_distribution(ctx, metrics_exporter.distribution_from_summary(s))
        if rank == 0:
            metrics_exporter.write_once(node, fs.get("project"), prom_file=fs.get("metrics-file"),
                                        jsonl_file=fs.get("metrics-jsonl"),
                                        labels={"scope": "node", "ranks": str(ctx.world)})
            _err(f"node latency distribution: {node.count} reads over {ctx.world} ranks")

    # node view (R3/R4)
    if ctx is not None and ctx.world > 1:
        st = dist.reduce_stats(ctx, nbytes=float(s["bytes"]), reads=float(s.get("reads", 0) + s.get("writes", 0)),
                               errors=float(s["errors"]), wall=wall, p50=s["p50_ms"], p99=s["p99_ms"])
        if rank == 0:
            _err(f"node: {int(st['reads_sum'])} ops, {st['nbytes_sum'] / 2**20 / st['wall_max']:.1f} MiB/s over "
                 f"{ctx.world} ranks; per-rank p50 {['%.2f' % x for x in st['p50_per_rank']]} ms, "
                 f"p99 {['%.2f' % x for x in st['p99_per_rank']]} ms")
    if fs.get("summary-json") and rank == 0:
        out = {k: v for k, v in s.items() if isinstance(v, (int, float, str, bool))}
        out["cpu_s_by_group"] = s.get("cpu_s_by_group", {})
        out.update({"workload": fs.get("workload"), "protocol": proto, "sink": sink, "workers": workers,
                    "world": world, "wall_s": wall, "extra": res.extra})
        if ctx is not None and ctx.world > 1:
            out["node"] = st
        with open(fs.get("summary-json"), "w") as f:
            json.dump(out, f, indent=1, default=str)
    ops = s.get("reads", 0) or s.get("writes", 0)
    _err(f"[rank {rank}] {ops} ops, {s['errors']} errors, {s['bytes'] / 2**20:.1f} MiB, "
         f"p50 {s['p50_ms']:.3f} ms, p99 {s['p99_ms']:.3f} ms, {s.get('mib_per_s', 0):.1f} MiB/s")
    if s["errors"]:
        _err(f"Error while running benchmark: {s.get('first_error', '')}")
        rc = 1
    else:
        _err("Read benchmark completed successfully!" if fs.get("workload") != "write"
             else "Write benchmark completed successfully!")
    if ep_handle:
        ep_handle.stop()
    if ctx is not None:
        dist.shutdown(ctx)
    return rc


def _make_runner(opts, directpath: bool):
    """Creates the native runner (and its storage client).  For gRPC the
    reference sets GOOGLE_CLOUD_ENABLE_DIRECT_PATH_XDS=true only while the
    client is constructed and unsets it afterwards (main.go:106-117)."""
    if opts.protocol != "grpc" or not directpath:
        return _native.Runner(opts.runner_dict())
    key = "GOOGLE_CLOUD_ENABLE_DIRECT_PATH_XDS"
    old = os.environ.get(key)
    os.environ[key] = "true"
    try:
        runner = _native.Runner(opts.runner_dict())
    finally:
        if old is None:
            os.environ.pop(key, None)
        else:
            os.environ[key] = old
    _err(f"gRPC transport: {runner.transport_path()}")
    return runner


def _run_with_live(opts, on_records, before_start, live, directpath: bool = True):
    runner = _make_runner(opts, directpath)
    live["runner"] = runner

    seen = workloads._drive(runner, on_records, before_start=before_start)
    return workloads.WorkloadResult(runner.summary(), seen)


if __name__ == "__main__":
    sys.exit(main())
