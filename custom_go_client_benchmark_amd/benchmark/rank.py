"""One bench rank: the headline and the side blocks (moved out of bench.py).

Headline (BASELINE config 2/4): ONE gRPC ReadObject stream per 256 MiB
object read (/root/reference/main.go:134-140), bytes landed in HBM through
the pinned ring + hipMemcpyAsync, every CRC32C verified by the CDNA4
kernels.  Rank r reads file_<r> (weak scaling; the reference's worker
fan-out main.go:200-210 spread over GPUs).

Paired headline (`--paired`, on at every N): the K timed headline reads run
in 4 chunks; between them, untimed for the headline, chunks of the same size
of two twins on the same endpoint, placement and object (and a raw TCP
probe):
  base   reference semantics -- discard sink + host CRC32C (main.go:140,
         the Go library's reader), on the headline's two cores;
  nodma  the headline's own ring and receive path, the ring never DMA-read
         (GpuSinkConfig gpu_stage none): the receive-side ceiling of the
         headline's exact byte path.
Each chunk is bracketed by a barrier + device sync on both sides; the
headline's value is its bytes over the sum of its chunks' slowest-rank
times.  vs_baseline_paired / headline_vs_nodma are the medians of the
per-chunk ratios, so a slow host window hits both arms of one chunk.
"""
from __future__ import annotations

import json
import os
import signal
import sys
import time

from . import report as rp
from .blocks import SideBlocks
from .hostio import Meter, maybe_hang, parse_size, stash, tcp_sysctls

METRIC = "p50/p99 read latency (ms) + MB/s per GPU; HTTP vs gRPC at 1/2/4/8 MI355X"

# side blocks a multi-GPU run does by default (the rest with --blocks all)
SCALE_BLOCKS = ("cpu_baseline", "compare", "write", "fanout")

# HTTP/2 receive settings of the gRPC clients (--h2-framing).  ref: what the
# reference's grpc-go client (go.mod:20, built with library defaults at
# main.go:106-117) leaves its peer with -- no SETTINGS_MAX_FRAME_SIZE, so
# 16,384-byte DATA frames, and windows its BDP estimator grows to at most
# 16 MiB [lib, parity-unpinned].  large: 16 MiB - 1 frames (one DATA frame
# per <= 2 MiB gRPC message, as in rounds 2-5) with the reference's 16 MiB
# windows.  Rounds 2-5 advertised 2 GiB - 1 windows; at 16 MiB the headline
# reads the same (median 26.1k against 25.7k MiB/s over 6 paired runs, p99/p50
# 1.09 against 1.18) and so do the multiplexed blocks, while the window caps
# the faster reference-semantics twins of one stream (profiles/r6_ag - r6_ai).
FRAMING = {"ref": {"h2_max_frame_size": 0, "h2_window": 16 << 20},
           "large": {"h2_max_frame_size": (1 << 24) - 1, "h2_window": 16 << 20}}
FRAME_LABEL = {"ref": "16KiB", "large": "16MiB"}

# Settings fixed by measurement in rounds 2-6 (no longer flags; the profiles/
# that chose each are cited where it is used).  GCSB_FIXED overrides them for
# an A/B session (fixed_overrides).
FIXED = {
    "conn_ring": "4x1MiB",        # multiplexed gRPC -> HBM: one 4 x 1 MiB ring per connection (r4_ringgeom)
    "async_submit": 1,            # slot hand-off on the device submitter thread (r2_single_stream)
    "submit_cpus": "aux",         # ... on a core of its own from the placement plan
    "rcvbuf": "64MiB",            # one-stream reads' SO_RCVBUF request (r2_rcvbuf)
    "sliced_slot_bytes": "2MiB",  # sliced block: 2 x 2 MiB ring per sink (r2_sliced, r3_ring_thp/sliced)
    "sliced_slots": 2,
    "sliced_async_submit": 0,
    "piece_bytes": "8MiB",        # sliced reads pull 8 MiB pieces from a shared cursor
    "piece_min_bytes": "0",
    "event_wait": "block",        # GPU sinks wait on slot events by blocking (the CPU quota)
    "list_placement": "same",     # config 3: readers and endpoint in one L3 domain (r2_check_s4b)
    "list_ring_wc": "on",         # config 3: write-combined rings (r3_ring_thp/wc)
    "list_rcvbuf": "64MiB",
    "list_async_submit": 0,       # config 3: each reader issues its own copy + CRC launch; the shared
                                  # submitter thread, ~2/3 busy, queued the 8 readers' hand-offs (r6_w)
    "list_wait_poll_us": 10,      # config 3: end-of-read event poll period (0: hipEventSynchronize; 5 ~ 10, r6_w)
    "ceiling": "on",              # the ceiling block (--blocks selects it away)
    "ref_grpc_placement": "same",        # 48 workers on one connection in one L3 domain (r3_mux_thp/refplace)
    "ref_http_placement": "share_quota",  # 48 HTTP receivers over the quota's cores
    "ref_gpu_ring": "2x2MiB",
    "ref_grpc_rcvbuf": "0",
    "write_placement": "pair",    # config 5: uploader + endpoint on three quiet cores (r3_write/placement)
    "mux_send": "isolate",        # multiplexed blocks: the endpoint send thread and the
    "mux_reader": "isolate",      # connection reader on physical cores of their own (r5_muxiso)
    "client_cc": "cubic",         # client sockets' congestion control, set before connect (r4_recvcost)
    "write_async_stage": "on",    # config 5: staging past the first slots issued on the submitter (r6_f, r6_g)
    "write_verify": "on",         # config 5: the endpoint CRC-checks every message (off: attribution A/B only)
    "write_slot_bytes": "2MiB",   # config 5: upload staging slot = one 2 MiB WriteObject message (r6_j)
    "write_composite_placement": "split",  # the 8-part upload: writers and endpoint on two L3 domains
                                           # (median 31.2k against 23.0k MiB/s spread over the share, r6_ad)
    "write_crc_core": "own",      # config 5: the endpoint's receive thread and its CRC worker pinned to
                                  # different physical cores ("shared": both over both, r6_u)
}


def fixed_overrides(env: str | None) -> dict:
    """GCSB_FIXED="key=value,key=value": experiments override FIXED values
    (A/B sessions) without a bench flag each; unknown keys are an error."""
    out = {}
    for item in (env or "").split(","):
        if not item.strip():
            continue
        k, sep, v = item.partition("=")
        k = k.strip()
        if not sep or k not in FIXED:
            raise SystemExit(f"GCSB_FIXED: unknown or malformed item {item!r} (keys: {', '.join(FIXED)})")
        out[k] = type(FIXED[k])(v.strip())
    return out


class RankBench(SideBlocks):
    """One rank's benchmark: its endpoint, placement and blocks."""

    def __init__(self, args):
        import torch

        import custom_go_client_benchmark_amd as pkg
        from ..ops import hbm
        from ..parallel import affinity
        from ..parallel import dist as gdist

        self.args = args
        self.torch = torch
        self.hbm = hbm
        self.affinity = affinity
        self.gdist = gdist
        self.n = pkg._native
        fixed = {**FIXED, **fixed_overrides(os.environ.get("GCSB_FIXED"))}
        for k, v in fixed.items():
            if not hasattr(args, k):
                setattr(args, k, v)
        self.rank, self.world, self.local_rank = gdist.env_rank()
        self.use_gpu = args.sink == "gpu"
        self.rehearsal = os.environ.get("GCSB_DIST_BACKEND") == "gloo"
        self.diag: dict = {}  # the sidecar (rank 0 writes it)
        self.last_start_ns = 0  # steady clock of the last timed_segment's start() (CLOCK_MONOTONIC, as now_ns())

    # ------------------------------------------------------------------ setup
    def setup(self) -> int:
        args, n, torch, gdist, affinity = self.args, self.n, self.torch, self.gdist, self.affinity
        if args.gpus != self.world:
            print(f"bench: --gpus {args.gpus} but the launcher started {self.world} rank(s) (WORLD_SIZE); "
                  f"they must match", file=sys.stderr)
            return 2
        if self.use_gpu:
            self.hbm.gpu_required()
            ndev = torch.cuda.device_count()
            if self.world > ndev and not self.rehearsal:
                print(f"bench: {self.world} ranks but only {ndev} visible GPU(s); one rank per GPU "
                      f"(set GCSB_DIST_BACKEND=gloo for a shared-GPU rehearsal)", file=sys.stderr)
                return 2
        # process group even at world 1: RCCL init + barriers + reductions run in every GPU bench
        self.ctx = gdist.init(local_rank=self.local_rank, world=self.world, rank=self.rank, always_pg=self.use_gpu)
        if self.rank == 0:
            # a peer that never reaches a barrier ends this rank through the
            # watchdog, and the launcher ends a hung rank with SIGTERM: either
            # way the stashed headline line is printed first
            gdist.on_fatal(lambda: stash.emit_stash("a barrier timed out"))

            def _term(signum, frame):
                stash.emit_stash("terminated")
                os._exit(128 + signum)
            signal.signal(signal.SIGTERM, _term)
        protocol = args.protocol
        if protocol == "auto":
            protocol = "grpc" if "grpc" in self.hbm.available_protocols() else "http"
        self.protocol = protocol
        self.size = parse_size(args.object_size)
        self.side_steps = args.steps if args.side_steps < 0 else args.side_steps
        # side blocks get the headline's warm-up too: each opens fresh
        # connections (and an endpoint of its own), so one warm-up read left
        # its first timed one carrying setup (profiles/r2_write/tail_probe_*.json)
        self.side_warm = max(1, args.warmup)

        # node-local synthetic GCS endpoint for this rank (no network on the box)
        self.gpu = self.ctx.gpu if self.ctx.gpu >= 0 else 0
        aff = args.affinity
        if aff == "auto":
            aff = "pair" if args.slices == 1 else "share"
        self.aff = aff
        # ranks sharing one GPU (rehearsal) spread over L3 domains instead of stacking
        self.slot = self.local_rank // max(1, torch.cuda.device_count()) if self.use_gpu and self.rehearsal else 0
        self.placement = affinity.plan(self.gpu, aff, self.slot) if self.use_gpu else {"client": [], "server": []}
        if self.use_gpu and args.submit_cpus == "aux" and self.placement.get("aux"):
            n.set_submitter_cpus(self.placement["aux"])
        self.srv = n.Server({"port": 0, "md5": False, "cpus": self.placement["server"], "retain_uploads": False})
        self.srv.start()
        self.bucket = "princer-working-dirs"
        self.prefix = "princer_100M_files/file_"
        self.first = self.rank * args.workers
        self.srv.add_synthetic(self.bucket, self.prefix, "", self.first, args.workers, self.size)
        self.cfg = {
            "protocol": protocol,
            "endpoint": self.srv.url,
            "bucket": self.bucket,
            "object_prefix": self.prefix,
            "workers": args.workers,
            "reads_per_worker": args.warmup,
            "worker_id_offset": self.first,
            "sink": args.sink,
            "device": self.gpu if self.use_gpu else 0,
            "ring_slot_bytes": parse_size(args.slot_bytes),
            "ring_slots": args.slots,
            "conn_ring": args.conn_ring != "off",
            "conn_ring_slots": int(args.conn_ring.partition("x")[0]) if "x" in args.conn_ring else 4,
            "conn_ring_slot_bytes": parse_size(args.conn_ring.partition("x")[2]) if "x" in args.conn_ring else 1 << 20,
            "landing": "object",
            "grpc_conn_pool_size": args.grpc_pool,
            "keep_records": False,
            "cpus": self.placement["client"],
            "retry_initial_s": 0.05,
            "slices": args.slices,
            "slice_piece_bytes": parse_size(args.piece_bytes),
            "slice_piece_min_bytes": parse_size(args.piece_min_bytes),
            "blocking_sync": args.event_wait == "block",
            "async_submit": bool(args.async_submit),
            "rcvbuf": parse_size(args.rcvbuf),
            "tcp_congestion": args.client_cc,
            "loopback_rto_min": True,
        }
        self.framing_name = getattr(args, "h2_framing", "large")
        self.framing = dict(FRAMING[self.framing_name])
        self.cfg.update(self.framing)
        return 0

    def sync(self) -> None:
        if self.torch.cuda.is_available():
            self.torch.cuda.synchronize()

    # --------------------------------------------------------- read blocks
    def read_ok(self, s: dict, reads: int, cfg: dict) -> tuple[bool, str]:
        if s["errors"]:
            return False, s["first_error"] or "read error"
        if s["reads"] != reads:
            return False, f"{s['reads']} of {reads} reads completed"
        # every read must have had its checksums verified (GPU CRC or host CRC)
        if (cfg.get("sink") == "gpu" or cfg.get("host_crc", True)) and s["verified"] != reads:
            return False, f"only {s['verified']} of {reads} reads had their CRC32C verified"
        return True, ""

    def open_runner(self, overrides: dict, warmup: int):
        """A Runner for cfg + overrides, its warm-up reads done (connections,
        rings, sinks survive into the timed reads).  (runner, error)."""
        r1, err = None, ""
        try:
            r1 = self.n.Runner({**self.cfg, **overrides, "reads_per_worker": warmup})
            if warmup > 0:
                r1.start()
                r1.wait()
                sw = r1.summary()
                if sw["errors"]:
                    err = f"warmup: {sw['first_error']}"
            r1.reset_stats()
        except Exception as e:  # noqa: BLE001 - reported in the block, collectives still run
            err = err or f"{type(e).__name__}: {e}"
        # runtime helper threads the warm-up may have started: "hip-rt", not "python3"
        from ..utils import cpuacct
        cpuacct.label_runtime_threads()
        return r1, err

    def timed_segment(self, r1, reads: int, what: str, err: str, meter: Meter | None) -> float:
        """`reads` reads per worker of an open runner between two barriers,
        each followed by a device sync.  Every rank makes every collective
        call whatever happens locally.  Returns this rank's elapsed s."""
        gdist = self.gdist
        if r1 is not None and not err:
            r1.set_reads_per_worker(reads)
        gdist.barrier(self.ctx, f"R1 {what} start barrier")
        self.sync()
        if meter is not None and not err:
            meter.begin()
        t1 = time.perf_counter()
        self.last_start_ns = time.monotonic_ns()
        if not err:
            r1.start()
            r1.wait()
        self.sync()
        gdist.barrier(self.ctx, f"R2 {what} stop barrier")
        e1 = time.perf_counter() - t1
        if meter is not None and not err:
            meter.end(e1)
        return e1

    def read_block(self, overrides: dict, steps: int, warmup: int, what: str, endpoint=None) -> dict:
        """warm-up reads, then `steps` timed reads of a config variant between
        two barriers (one contiguous timed region)."""
        from ..utils import sysdiag

        r1, err = self.open_runner(overrides, warmup)
        ep_stats = (endpoint or self.srv).stats
        before = self._counters(ep_stats)
        diag_cpus = sorted(set(overrides.get("cpus") or self.cfg.get("cpus") or [])
                           | set(self.placement.get("server") or []) | set(self.placement.get("aux") or []))
        # the host view starts before the CPU bracket and reports after it
        win = sysdiag.Window(clock_cpus=diag_cpus if 0 < len(diag_cpus) <= 16 else None) if not err else None
        meter = Meter()
        e1 = self.timed_segment(r1, steps, what, err, meter)
        return self.finish_block(r1, err, overrides, steps, e1, meter, before, ep_stats, win, diag_cpus)

    def _counters(self, ep_stats, reset_hip: bool = True) -> dict:
        n = self.n
        if self.use_gpu and reset_hip:
            n.reset_slow_hip_calls()
        return {"rv": n.recv_stats(), "rd": n.recv_diag(), "h2": n.h2_reader_stats(), "sv": ep_stats()}

    def finish_block(self, r1, err: str, overrides: dict, steps: int, e1: float, meter: Meter, before: dict,
                     ep_stats, win, diag_cpus) -> dict:
        """Checks, per-GiB CPU, transport counters and the cross-rank
        reduction of one read block (all of it outside the timed region)."""
        from ..utils import cpuacct, sysdiag

        n = self.n
        cfg = {**self.cfg, **overrides}
        workers = cfg.get("workers", self.args.workers)
        cpu = {}
        s1 = None
        if not err:
            s1 = r1.summary()
            ok, why = self.read_ok(s1, steps * workers, cfg)
            if not ok:
                err = why
            nb = float(s1["bytes"])
            gib = max(nb, 1.0) / (1 << 30)
            cpu = meter.delta(nb)
            if win is not None:
                # what else ran on the block's CPUs: run-queue delay of our
                # threads, interrupts and softirqs there (utils/sysdiag.py)
                cpu["host"] = win.report(diag_cpus or None, max(1, int(s1["reads"])))
            names = dict(meter.threads)
            groups: dict[str, float] = {}
            for k, v in names.items():
                g = cpuacct.group_of(k)
                groups[g] = groups.get(g, 0.0) + v
            cpu["cpu_s_per_gib_by_thread"] = cpuacct.per_gib(groups, nb)
            # worker threads exit at the end of the run: their CPU comes from the runner
            names.pop("gcsb-worker", None)
            names["gcsb-worker (exited)"] = s1.get("worker_cpu_s", 0.0)
            cpu["cpu_s_per_gib_by_name"] = {k: v for k, v in cpuacct.per_gib(names, nb).items() if v >= 0.0005}
            h2s1 = n.h2_reader_stats()
            h2s0 = before["h2"]
            if h2s1["frames"] > h2s0["frames"]:
                # the HTTP/2 connection readers (gRPC): where their time went, per GiB
                d = {k: h2s1[k] - h2s0[k] for k in h2s1}
                cpu["h2_reader"] = {"frames_per_read": round(d["frames"] / max(1, s1["reads"]), 2),
                                    # waits over 5 ms are apart: an idle connection's
                                    # next frame after a pause is not this block's time
                                    "wait_s_per_gib": round((d["header_wait_ns"] - d.get("long_wait_ns", 0))
                                                            / 1e9 / gib, 4),
                                    "long_waits": d.get("long_waits", 0),
                                    "long_wait_s": round(d.get("long_wait_ns", 0) / 1e9, 4),
                                    "readers_alive": h2s1.get("readers_alive", 0),
                                    "data_s_per_gib": round(d["data_ns"] / 1e9 / gib, 4),
                                    "headers_s_per_gib": round(d["headers_ns"] / 1e9 / gib, 4),
                                    "other_s_per_gib": round(d["other_ns"] / 1e9 / gib, 4),
                                    "avg_data_frame_kib": round(d["data_bytes"] / max(1, d["data_frames"]) / 1024, 1)}
            cr = r1.conn_ring_stats()
            if cr:
                # the multiplexed connection's shared receive ring (warmup included)
                cpu["conn_ring"] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in cr.items()}
            g1 = s1.get("gpu") or {}
            if g1.get("slot_waits") or g1.get("flag_reuses"):
                cpu["slot_reuse"] = {"waits": g1["slot_waits"], "on_kernel_status": g1.get("flag_reuses", 0),
                                     "s_per_gib": round(g1["slot_wait_s"] / gib, 4),
                                     "handoff_s_per_gib": round(g1.get("handoff_s", 0.0) / gib, 5)}
            sv0, sv1 = before["sv"], ep_stats()
            if sv1.get("h2_data_frames", 0) > sv0.get("h2_data_frames", 0):
                fr = sv1["h2_data_frames"] - sv0["h2_data_frames"]
                rs = max(1, sv1["h2_responses"] - sv0["h2_responses"])
                cpu["endpoint_h2"] = {"frames": fr,
                                      "queue_wait_avg_us": round((sv1["h2_queue_wait_us"] - sv0["h2_queue_wait_us"]) / fr, 1),
                                      "queue_wait_max_us": sv1["h2_queue_wait_max_us"],
                                      "ttfb_avg_us": round((sv1["h2_ttfb_us"] - sv0["h2_ttfb_us"]) / rs, 1),
                                      "ttfb_max_us": sv1["h2_ttfb_max_us"]}
            if sv1.get("body_sends", 0) > sv0.get("body_sends", 0):
                wall = max(1, sv1["body_wall_us"] - sv0["body_wall_us"])
                sends = sv1["body_sends"] - sv0["body_sends"]
                cpu["endpoint_tcp"] = {
                    "busy_frac": round((sv1["tcp_busy_us"] - sv0["tcp_busy_us"]) / wall, 3),
                    "rwnd_limited_frac": round((sv1["tcp_rwnd_limited_us"] - sv0["tcp_rwnd_limited_us"]) / wall, 3),
                    "sndbuf_limited_frac": round((sv1["tcp_sndbuf_limited_us"] - sv0["tcp_sndbuf_limited_us"]) / wall,
                                                 3),
                    "cwnd_kib_at_end": round((sv1["tcp_cwnd_bytes_sum"] - sv0["tcp_cwnd_bytes_sum"]) / sends / 1024, 1)}
            rv0, rv1 = before["rv"], n.recv_stats()
            calls = rv1[0] - rv0[0]
            if calls:
                cpu["recv_calls"] = calls
                cpu["recv_avg_kib"] = round((rv1[1] - rv0[1]) / calls / 1024.0, 1)
            rd0, rd1 = before["rd"], n.recv_diag()
            dc = rd1["calls"] - rd0["calls"]
            if dc:
                cpu["recv_queue"] = {"payload_recvs": dc,
                                     "empty_frac": round((rd1["empty"] - rd0["empty"]) / dc, 3),
                                     "short_frac": round((rd1["short"] - rd0["short"]) / dc, 3),
                                     "avg_queued_kib": round((rd1["inq_bytes"] - rd0["inq_bytes"]) / dc / 1024, 1),
                                     "avg_asked_kib": round((rd1["want_bytes"] - rd0["want_bytes"]) / dc / 1024, 1),
                                     "recv_s_per_gib": round((rd1["recv_ns"] - rd0["recv_ns"]) / 1e9 / gib, 4)}
        slow_hip = n.slow_hip_calls() if self.use_gpu else {}
        use_gpu_sink = self.use_gpu and cfg.get("sink") == "gpu"
        ring_numa = r1.ring_numa(0) if (r1 is not None and use_gpu_sink) else []
        ring_thp = r1.ring_thp_fraction(0) if (r1 is not None and use_gpu_sink) else -1.0
        s1 = s1 or {"bytes": 0, "p50_ms": 0.0, "p99_ms": 0.0, "host_p50_ms": 0.0, "ttfb_p50_ms": 0.0,
                    "slice_skew_ms": 0.0, "verified": 0, "reads": 0}
        recv = rp.recv_cost(cpu) or 0.0
        py = (cpu.get("cpu_s_per_gib_by_name") or {}).get(cpuacct.process_name(), 0.0)
        del r1
        st = self.gdist.reduce_stats(self.ctx, elapsed=e1, nbytes=float(s1["bytes"]), p50=s1["p50_ms"],
                                     p99=s1["p99_ms"], host_p50=s1["host_p50_ms"],
                                     ttfb_p50=s1.get("ttfb_p50_ms", 0.0), skew=s1.get("slice_skew_ms", 0.0),
                                     first_p50=s1.get("first_read_p50_ms", 0.0),
                                     steady_p99=s1.get("steady_p99_ms", 0.0), verified=float(s1["verified"]),
                                     recv_cpu=recv, py_cpu=py, ok=0.0 if err else 1.0)
        st["error"] = err
        st["cpu"] = cpu
        st["ring_numa"] = ring_numa
        st["ring_thp"] = ring_thp
        # this rank's slowest reads [index in the timed run, ms, host-landed ms, TTFB ms]
        st["slowest"] = [[int(x[0])] + [round(v, 3) for v in x[1:]] for x in (s1.get("slowest") or [])]
        if s1.get("slowest_diag"):
            st["slowest_diag"] = [
                {"read": int(x[0]), "ms": round(x[1], 3),
                 "cause": sysdiag.attribute(dg, x[1], s1["p50_ms"]),
                 "threads": {k: {f: (round(v, 3) if isinstance(v, float) else v) for f, v in row.items()}
                             for k, row in dg["threads"].items()},
                 "softirqs": dg["softirqs"], "tcp": dg.get("tcp", {}), "softnet": dg.get("softnet", {})}
                for x, dg in zip(s1["slowest"], s1["slowest_diag"])]
        st["slow_hip"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in slow_hip.items()}
        return st

    # ============================================================ the run
    def run(self) -> int:
        rc = self.setup()
        if rc:
            return rc
        args, gdist, ctx = self.args, self.gdist, self.ctx
        world, rank, protocol = self.world, self.rank, self.protocol
        side_steps, side_warm = self.side_steps, self.side_warm
        use_gpu = self.use_gpu

        only = {b.strip() for b in args.blocks.split(",") if b.strip()}
        explicit = only - {"all"}
        base_on = args.baseline == "on" and (not explicit or "cpu_baseline" in explicit) and side_steps > 0
        bracket = args.baseline_bracket == "on" or (args.baseline_bracket == "auto" and world == 1)
        # paired at every N: every rank runs the same arm
        # order between the same barriers, so the scaling run is credited on
        # the same estimator as the 1-GPU bench
        paired = args.workload == "read" and base_on and args.steps >= 2 and args.paired in ("on", "auto")
        self.base_before = None
        self.paired = None
        if args.workload == "read" and use_gpu and bracket and base_on:
            # the reference-semantics read once more BEFORE the headline, so
            # the two baselines bracket it and a drifting host cancels
            self.base_before = self.read_block(self.baseline_over(), side_steps, side_warm,
                                               f"{protocol} cpu baseline (before)")
        if args.workload == "read":
            # --read-diag samples the headline's threads around every read
            diag_avoid = sorted(set(self.placement.get("client", [])) | set(self.placement.get("server", []))
                                | set(self.placement.get("aux", []) or []))
            head_over = {"read_diag": bool(args.read_diag), "diag_avoid_cpus": diag_avoid}
            if paired:
                nodma = {"gpu_stage": "none", "gpu_verify": False} if use_gpu else None
                head, self.paired = self.paired_headline(head_over, self.baseline_over(), nodma, args.steps,
                                                         args.warmup, args.paired_chunks)
            else:
                head = self.read_block(head_over, args.steps, args.warmup, "headline")
            self.headline_model = (f"{protocol} ReadObject {args.object_size} object, "
                                   f"{'one stream per read' if args.slices == 1 else f'{args.slices} ranged streams'}"
                                   + (" -> HBM (CRC32C on GPU)" if use_gpu else " -> discard (CPU baseline)"))
        else:
            if not use_gpu:
                print("bench: --workload write needs --sink gpu (uploads are staged from HBM)", file=sys.stderr)
                return 2
            head = self.write_block(args.steps, args.warmup)
            self.headline_model = (f"{protocol} resumable upload {args.write_size} object from HBM "
                                   f"(D2H -> pinned -> upload)")
        self.head = head

        # R4: which HIP device each rank used -> distinct GPUs in the job (before
        # the side blocks: the fan-out block may leave the communicator aborted)
        devs = gdist.gather_floats(ctx, [float(ctx.gpu if use_gpu else -1)])
        self.distinct = sorted({int(d[0]) for d in devs if d[0] >= 0})
        self.n_gpus = len(self.distinct) if use_gpu else world

        other = {"grpc": "http", "http": "grpc"}.get(protocol)
        protos = self.hbm.available_protocols()
        ref100 = parse_size(args.ref100_object_size)
        self.blocks = {}
        blocks = self.blocks
        if not only and world > 1:
            # N > 1: the blocks the scaling run needs; the rest only when asked for
            only = set(SCALE_BLOCKS)
        if "all" in only:
            only = set()

        def want(name: str) -> bool:
            ok = not only or name in only
            if ok:
                maybe_hang(name, rank)
            return ok
        if side_steps > 0 and args.workload == "read":
            if base_on and want("cpu_baseline"):
                # right after the headline: the reference's semantics on the
                # headline config -- same endpoint, placement, object and
                # steps; bytes to a discard sink, CRC32C of every byte on the
                # host (/root/reference/main.go:133-146).  vs_baseline divides by it.
                for p in [protocol] + ([other] if other and other in protos else []):
                    key = "cpu_baseline" if p == protocol else f"cpu_baseline_{p}"
                    over = {**self.baseline_over(), "protocol": p}
                    blocks[key] = (self.read_block(over, side_steps, side_warm, f"{p} cpu baseline"),
                                   {"protocol": p, "sink": "discard", "_conns": 1, "_place": "pair",
                                    "note": "reference semantics: io.Discard + host CRC32C; client + submitter cores"})
            self.stash_headline()
            alt = "large" if self.framing_name == "ref" else "ref"
            twin_on = protocol == "grpc" and getattr(args, "framing_twin", "on") == "on"
            if twin_on and base_on and want("framing_twin"):
                # the headline config at the OTHER framing, paired chunk by
                # chunk with its reference-semantics baseline at that framing
                fo = FRAMING[alt]
                st_t, pr_t = self.paired_headline(dict(fo), {**self.baseline_over(), **fo}, None, side_steps,
                                                  side_warm, args.paired_chunks, probe_tcp=False,
                                                  what=f"{alt} framing")
                blocks[f"{alt}_framing"] = (st_t, {"protocol": protocol, "sink": args.sink, "_conns": 1,
                                                   "_place": "pair", "h2_frames": FRAME_LABEL[alt],
                                                   "vs_baseline_paired": pr_t.get("vs_baseline_paired"),
                                                   "base_mib_s": pr_t.get("base_mib_s"),
                                                   "note": "headline config at the other HTTP/2 framing, paired "
                                                           "with its reference-semantics baseline"})
            if (world == 1 and protocol == "grpc" and args.ref_effective == "on" and want("ref_effective")):
                # the reference's EFFECTIVE read on the headline config: the
                # baseline (same endpoint, cores, object and steps) whose
                # consumer also copies every decoded message out in 8 KiB
                # reads, as io.Discard.ReadFrom pulls them out of the library's
                # reader (main.go:123-125,140).  Parity-unpinned.
                over = {**self.baseline_over(), "discard_read_bytes": 8192}
                blocks["ref_effective_head"] = (
                    self.read_block(over, side_steps, side_warm, f"{protocol} effective read (headline config)"),
                    {"protocol": protocol, "sink": "discard", "_conns": 1, "_place": "pair",
                     "note": "parity-unpinned: grpc-go's message decode + 8 KiB io.Discard reads, modelled"})
            if other and other in protos and want("compare"):
                blocks["compare"] = (self.read_block({"protocol": other}, side_steps, side_warm, f"{other} compare"),
                                     {"protocol": other, "sink": self.args.sink, "_conns": 1, "_place": "pair"})
            if self.base_before is not None:
                blocks["cpu_baseline_before"] = (self.base_before,
                                                 {"protocol": protocol, "sink": "discard", "_conns": 1,
                                                  "_place": "pair",
                                                  "note": "the cpu_baseline block, run before the headline"})
            if args.sliced_streams > 1 and args.slices == 1 and want("sliced"):
                # 8 receive + 8 send threads: a share-placed endpoint of its own
                srv_sl, sh = self.share_endpoint()
                sliced_cfg = {"slices": args.sliced_streams, "ring_slot_bytes": parse_size(args.sliced_slot_bytes),
                              "ring_slots": args.sliced_slots, "async_submit": bool(args.sliced_async_submit),
                              "rcvbuf": 0, "endpoint": srv_sl.url, "cpus": sh["client"]}
                st_sl = self.read_block(sliced_cfg, side_steps, side_warm, "sliced")
                srv_sl.stop()
                blocks["sliced"] = (st_sl, {"streams_per_read": args.sliced_streams, "sink": self.args.sink,
                                            "ring": f"{args.sliced_slots}x{args.sliced_slot_bytes}",
                                            "_conns": args.sliced_streams, "affinity": "share",
                                            "piece_bytes": parse_size(args.piece_bytes),
                                            "note": "extension, not parity"})
            if args.ceiling == "on" and want("ceiling"):
                blocks["ceiling"] = (self.ceiling_block(rp.mib_s(head) / max(1, world)), None)
            if args.ref_workers > 0 and want("ref_default"):
                for p in ["http"] + [x for x in ("grpc",) if x in protos]:
                    blocks[f"ref_default_{p}"] = (self.ref_default_block(p),
                                                  {"protocol": p, "workers": args.ref_workers, "sink": "discard",
                                                   "object_bytes": parse_size(args.ref_object_size),
                                                   "reads_per_worker": args.ref_reads,
                                                   "_conns": 1 if p == "grpc" else args.ref_workers, "_place": "same",
                                                   "h2_frames": FRAME_LABEL[self.framing_name] if p == "grpc" else None,
                                                   "note": "reference default experiment (execute_pb.sh)"})
                if "grpc" in protos and twin_on:
                    blocks[f"ref_default_grpc_{alt}"] = (
                        self.ref_default_block("grpc", extra=dict(FRAMING[alt])),
                        {"protocol": "grpc", "workers": args.ref_workers, "sink": "discard",
                         "object_bytes": parse_size(args.ref_object_size), "reads_per_worker": args.ref_reads,
                         "_conns": 1, "_place": "same", "h2_frames": FRAME_LABEL[alt],
                         "note": "ref_default_grpc at the other HTTP/2 framing"})
            if args.ref_workers > 0 and args.ref_effective == "on" and "grpc" in protos and want("ref_effective"):
                # the reference's EFFECTIVE read path: io.Discard.ReadFrom ignores
                # the 2 MiB buffer and pulls 8 KiB reads out of each decoded
                # <= 2 MiB message (main.go:123-125,140)
                blocks["ref_effective_grpc"] = (
                    self.ref_default_block("grpc", ref100, args.ref100_reads, "discard", warmup=1,
                                           extra={"discard_read_bytes": 8192}),
                    {"protocol": "grpc", "workers": args.ref_workers, "sink": "discard", "object_bytes": ref100,
                     "_conns": 1, "_place": "same",
                     "note": "parity-unpinned: grpc-go's message decode + 8 KiB io.Discard reads, modelled"})
            if args.ref_workers > 0 and args.ref100_reads > 0 and want("ref_default_100m"):
                # the reference's real operating point: 48 workers x 100 MiB
                # (princer_100M_files, main.go:36,52), both transports, into
                # the discard sink (reference semantics) and into HBM
                for p in ["http"] + [x for x in ("grpc",) if x in protos]:
                    for sk in ["discard"] + (["gpu"] if use_gpu else []):
                        key = f"ref_default_100m_{p}_{sk}"
                        blocks[key] = (self.ref_default_block(p, ref100, args.ref100_reads, sk, warmup=1),
                                       {"protocol": p, "workers": args.ref_workers, "object_bytes": ref100,
                                        "reads_per_worker": args.ref100_reads, "sink": sk,
                                        "ring": args.ref_gpu_ring if sk == "gpu" else None,
                                        "_conns": 1 if p == "grpc" else args.ref_workers, "_place": "same",
                                        "note": "reference default experiment at its object size"})
            if "http" in protos and want("c1_http_cpu"):
                # config 1: one 1 MiB object over the HTTP JSON API, CPU only
                self.srv.add_synthetic(self.bucket, "c1/file_", "", self.first, 1, 1 << 20)
                blocks["c1_http_cpu"] = (
                    self.read_block({"protocol": "http", "http_api": "json", "sink": "discard", "host_crc": True,
                                     "object_prefix": "c1/file_", "workers": 1, "rcvbuf": 0},
                                    max(side_steps, 100), side_warm, "config 1"),
                    {"protocol": "http", "api": "json", "object_bytes": 1 << 20, "sink": "discard", "workers": 1,
                     "config": "BASELINE config 1"})
            if args.list_objects > 0 and want("list_read"):
                for p in [protocol] + ([other] if other and other in protos else []):
                    blocks[f"list_read_{p}"] = (self.list_read_block(p, 1),
                                                {"protocol": p, "objects": args.list_objects, "object_bytes": 1 << 20,
                                                 "workers": args.list_workers, "ring": args.list_ring,
                                                 "sink": self.args.sink,
                                                 "_conns": 1 if p == "grpc" else args.list_workers, "_place": "same",
                                                 "h2_frames": FRAME_LABEL[self.framing_name] if p == "grpc" else None,
                                                 "config": "BASELINE config 3"})
                if "grpc" in protos and twin_on:
                    blocks[f"list_read_grpc_{alt}"] = (
                        self.list_read_block("grpc", 1, extra=dict(FRAMING[alt])),
                        {"protocol": "grpc", "objects": args.list_objects, "object_bytes": 1 << 20,
                         "workers": args.list_workers, "ring": args.list_ring, "sink": self.args.sink, "_conns": 1,
                         "_place": "same", "h2_frames": FRAME_LABEL[alt],
                         "note": "list_read_grpc at the other HTTP/2 framing"})
            if use_gpu and want("write"):
                blocks["write"] = (self.write_block(side_steps, side_warm),
                                   {"protocol": protocol, "object_bytes": parse_size(args.write_size),
                                    "config": "BASELINE config 5"})
            if use_gpu and args.write_parts > 1 and want("write_composite"):
                blocks["write_composite"] = (self.write_block(side_steps, side_warm, args.write_parts),
                                             {"protocol": protocol, "object_bytes": parse_size(args.write_size),
                                              "parts": args.write_parts,
                                              "note": "extension: parallel composite upload, not parity"})
            if world > 1 and args.fanout == "on" and want("fanout"):
                blocks["fanout"] = (self.fanout_block(side_steps, side_warm),
                                    {"object_bytes": self.size, "slice_bytes": self.size // world,
                                     "collective": f"{ctx.backend} all_gather_into_tensor"
                                     if ctx.device.type == "cuda" else f"{ctx.backend} all_gather via host",
                                     "note": "extension: read once per node, fan out over xGMI"})
        # (a write headline runs no side blocks)
        stash.disarm()
        self.srv.stop()

        rc = 0
        if rank == 0:
            res = self.assemble()
            if res is None:
                print(f"benchmark failed: {head['error'] or 'a rank failed'}", file=sys.stderr)
                rc = 1
            else:
                line, diag = res
                self.write_diag(diag)
                text = json.dumps(line)
                stash.final(text)
                if args.json_out:
                    with open(args.json_out, "w") as f:
                        f.write(text + "\n")
        elif head["ok_min"] < 1.0:
            rc = 1
        gdist.shutdown(ctx)
        return rc

    def stash_headline(self) -> None:
        """The headline line, complete but for the later side blocks: printed
        on stderr at once, and kept for the fatal paths (a side block that
        hangs: barrier watchdog, side-block deadline, SIGTERM from the
        launcher), so a measured headline is never lost."""
        if self.rank == 0:
            res = self.assemble()
            if res is not None:
                line = dict(res[0])
                line["partial"] = "side blocks after cpu_baseline did not finish"
                text = json.dumps(line)
                stash.stash(text)
                print(f"bench: headline measured: {text}", file=sys.stderr, flush=True)
        stash.arm(self.args.side_deadline)

    def write_diag(self, diag: dict) -> None:
        path = self.args.diag_out
        if not path:
            return
        try:
            with open(path, "w") as f:
                json.dump(diag, f)
            print(f"bench: diagnostics in {os.path.abspath(path)}", file=sys.stderr, flush=True)
        except OSError as e:
            print(f"bench: could not write {path}: {e}", file=sys.stderr, flush=True)

    # ----------------------------------------------------------- the line
    def full_block(self, key: str, st: dict, extra: dict) -> dict:
        """The sidecar's (verbose) view of one side block."""
        b = {"ok": st["ok_min"] >= 1.0, "mib_s": round(rp.mib_s(st), 2), "p50_ms": round(st["p50_max"], 3),
             "p99_ms": round(st["p99_max"], 3)}
        b.update({k: v for k, v in extra.items() if v is not None and not k.startswith("_")})
        if st.get("error"):
            b["error"] = st["error"][:300]
        cpu = st.get("cpu") or {}
        if cpu:
            b["cpu_s_per_gib_by_thread"] = cpu.get("cpu_s_per_gib_by_name", {})
            for k in ("cpus_busy", "process_cpu_s_per_gib", "h2_reader", "recv_avg_kib", "recv_queue", "endpoint_tcp",
                      "endpoint_h2", "conn_ring", "slot_reuse", "host", "cgroup_nr_throttled"):
                if cpu.get(k) is not None:
                    b[k] = cpu[k]
        if "recv_cpu_max" in st and st["recv_cpu_max"] > 0:
            b["recv_cpu_s_per_gib"] = round(st["recv_cpu_max"], 4)
        if "py_cpu_max" in st and st["py_cpu_max"] > 0:
            b["py_cpu_s_per_gib"] = round(st["py_cpu_max"], 4)
        if key.startswith(("ref_default_", "ref_effective")) and "first_p50_max" in st:
            b["first_read_p50_ms"] = round(st["first_p50_max"], 3)
            b["steady_p99_ms"] = round(st["steady_p99_max"], 3)
        if key == "fanout":
            # mib_s: whole objects landed in every GPU's HBM, job-wide
            b["per_gpu_mib_s"] = round(b["mib_s"] / max(1, self.world), 2)
            b["crc_verified_ranks"] = int(st.get("crc_ok_sum", 0))
        if st.get("slowest"):
            b["rank0_slowest"] = st["slowest"]
        if st.get("slow_hip", {}).get("slow"):
            b["slow_hip_calls"] = st["slow_hip"]
        if st.get("cpu_s_per_gib_by_thread"):
            b["cpu_s_per_gib_by_thread"] = st["cpu_s_per_gib_by_thread"]
        if key.startswith("list_read_"):
            b["list_ms"] = round(st["list_ms_max"], 3)
            if "host_p50_max" in st:
                # the read's last byte on the host (the reference's stop
                # point); p50_ms - this = the GPU tail (last H2D copy + CRC)
                b["host_landed_p50_ms"] = round(st["host_p50_max"], 3)
        if st.get("phases_ms"):
            b["phases_ms"] = st["phases_ms"]
        if st.get("upload_probe"):
            b["upload_probe"] = st["upload_probe"]
        if key == "sliced":
            b["host_landed_p50_ms"] = round(st["host_p50_max"], 3)
            b["slice_skew_ms"] = round(st["skew_max"], 3)
        return b

    def assemble(self) -> tuple[dict, dict] | None:
        """(the bench line, the sidecar) from the headline and the side blocks
        run so far; None if the headline failed."""
        head, args = self.head, self.args
        if head["ok_min"] < 1.0:
            return None
        value = rp.mib_s(head)
        world = self.world
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "MiB/s",
            "n_gpus": self.n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(head["elapsed_max"] / args.steps * 1000.0, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8",
            "data": "synthetic",
            "config": {
                "model": self.headline_model,
                "global_batch": world * args.workers,
                "seq_len": self.size if args.workload == "read" else parse_size(args.write_size),
                "parallelism": f"dp{world}",
                "workload": args.workload,
                "protocol": self.protocol,
                "object_bytes": self.size if args.workload == "read" else parse_size(args.write_size),
                "readers_per_gpu": args.workers,
                "sink": args.sink,
                "ring": f"{args.slots}x{args.slot_bytes}",
                "streams_per_read": args.slices if args.workload == "read" else 1,
            },
            "p50_ms": round(head["p50_max"], 3),
            "p99_ms": round(head["p99_max"], 3),
        }
        diag = {"config": {**out["config"], "event_wait": args.event_wait, "async_submit": bool(args.async_submit),
                           "rcvbuf": parse_size(args.rcvbuf), "sysctl": tcp_sysctls()},
                "endpoint": "loopback synthetic GCS (one per rank)",
                "endpoint_send": "vmsplice (THP copy of the pattern)",
                "endpoint_congestion_control": os.environ.get("GCSB_SRV_CC") or "cubic",
                "client_congestion_control": args.client_cc or "host default",
                "affinity": self.aff,
                "placement": {k: self.placement.get(k) for k in ("client", "server", "aux", "picked_by", "busy")
                              if self.placement.get(k) is not None}}
        ceil = None
        if "ceiling" in self.blocks:
            ceil = self.blocks["ceiling"][0]
        if self.paired:
            pr = self.paired
            for k in ("vs_baseline_paired", "headline_vs_nodma", "headline_vs_tcp_paired"):
                if k in pr:
                    out[k] = pr[k]
            diag["paired"] = pr
        # ONE ceiling: the best of every TCP probe of the run (paired chunks +
        # the ceiling block) and the H2D copy rate (report.unified_ceiling)
        uc = rp.unified_ceiling(value / max(1, self.n_gpus), (self.paired or {}).get("tcp_mib_s"), ceil, world,
                                self.use_gpu)
        if uc:
            out["headline_frac_of_ceiling"] = uc["headline_frac_of_ceiling"]
            diag["ceiling"] = uc
        out["h2_frames"] = FRAME_LABEL[self.framing_name] if self.protocol == "grpc" else None
        # the HTTP/2 windows the client advertised (MiB): the reference's 16
        out["h2_window_mib"] = (self.framing["h2_window"] >> 20) if self.protocol == "grpc" else None
        if args.workload == "read":
            out["ttfb_p50_ms"] = round(head["ttfb_p50_max"], 3)
            out["host_landed_p50_ms"] = round(head["host_p50_max"], 3)
            out["verified_reads"] = int(head["verified_sum"])
        out["per_gpu_mib_s"] = round(value / max(1, self.n_gpus), 2)
        out["per_rank_mib_s"] = [round(b / max(e, 1e-12) / (1 << 20), 1)
                                 for b, e in zip(head["nbytes_per_rank"], head["elapsed_per_rank"])]
        out["ranks"] = world
        out["control_plane"] = self.ctx.backend + (" (RCCL init failed: fallback)" if self.ctx.fallback else "")
        out["devices"] = self.distinct if self.use_gpu else "none (cpu rehearsal)"
        if self.paired:
            pr = self.paired
            out["paired"] = {k: pr[k] for k in ("chunks", "pair_ratios", "nodma_ratios", "tcp_ratios", "head_mib_s",
                                                "base_mib_s", "nodma_mib_s", "tcp_mib_s", "rewarm_reads") if k in pr}
            cf = (pr.get("chunk_first") or {}).get("head")
            if cf:
                out["paired"]["head_first_vs_median"] = cf["first_vs_median"]
            if pr.get("slow_windows"):
                out["paired"]["slow_windows"] = [[w["chunk"], w["cause"][:120]] for w in pr["slow_windows"][:2]]
        # host-memory placement of the object's page cache and the pinned ring
        numa = {"gpu_node": self.placement.get("numa_node"), "object_pages": _by_node(self.n.pattern_memfd_numa())}
        if head.get("ring_numa"):
            slots = head["ring_numa"]
            total = [sum(c[i] for c in slots) for i in range(len(slots[0]))]
            numa["ring_pages"] = _by_node(total)
            numa["ring_slot_nodes"] = [max(range(len(c) - 1), key=lambda i: c[i]) if sum(c[:-1]) else -1
                                       for c in slots]
        if head.get("ring_thp", -1.0) >= 0:
            numa["ring_thp_fraction"] = round(head["ring_thp"], 3)
        diag["numa"] = numa
        if args.workload == "write":
            diag["rank0_cpu_s_per_gib_by_thread"] = head.get("cpu_s_per_gib_by_thread", {})
        else:
            diag["rank0_cpu"] = head.get("cpu", {})
            if head.get("slowest_diag"):
                diag["rank0_slowest_diag"] = head["slowest_diag"]
            if head.get("slow_hip"):
                diag["slow_hip_calls"] = head["slow_hip"]
            if head.get("cpu"):
                gib_s = value / max(1, world) / 1024.0
                diag["cpus_needed_per_gpu"] = round(head["cpu"].get("process_cpu_s_per_gib", 0.0) * gib_s, 2)
        out["rank0_slowest"] = [r[:2] for r in (head.get("slowest") or [])[:3]]
        base = self.blocks.get("cpu_baseline")
        if base is not None and base[0]["ok_min"] >= 1.0 and rp.mib_s(base[0]) > 0:
            runs = [base[0]]
            bb = self.base_before
            if bb is not None and bb["ok_min"] >= 1.0 and rp.mib_s(bb) > 0:
                runs = [bb, base[0]]
            # pooled over the runs bracketing the headline: all their bytes over all their time
            pooled = sum(r["nbytes_sum"] for r in runs) / max(sum(r["elapsed_max"] for r in runs), 1e-12) / (1 << 20)
            p50 = sum(r["p50_max"] for r in runs) / len(runs)
            out["vs_baseline"] = round(value / pooled, 3)
            b = {"mib_s": round(pooled, 2), "p50_ms": round(p50, 3),
                 "p50_ratio": round(p50 / max(head["p50_max"], 1e-9), 3)}
            if len(runs) == 2:
                b["mib_s_before"] = round(rp.mib_s(bb), 2)
                b["mib_s_after"] = round(rp.mib_s(base[0]), 2)
            flag = rp.receiver_interference(head.get("cpu") or {}, [(r.get("cpu") or {}) for r in runs])
            if flag:
                b["cost_ratio"] = flag.get("cost_ratio")
                diag["baseline_receiver"] = flag
            out["baseline"] = b
            diag["baseline_what"] = ("cpu_baseline: same config, reference semantics (discard sink + host CRC32C), "
                                     "same run" + (", run right before and right after the headline, pooled"
                                                   if len(runs) == 2 else ", run right after the headline"))
        full = {}
        tcp_best_gbps = (uc["tcp_best_mib_s"] / rp.MIB_PER_GBPS) if uc else 0.0
        for key, (st, extra) in self.blocks.items():
            if extra is None:  # already a JSON block (ceiling)
                full[key] = dict(st)
                continue
            b = self.full_block(key, st, extra)
            if key == "write" and st.get("upload_tcp_min", 0.0) > 0:
                # config 5's bound: one loopback TCP stream in the upload's
                # direction and placement (write_block), per GPU
                bmib = st["upload_tcp_min"] * max(1, world)
                if b["mib_s"] > bmib:
                    # the upload beat its probe: the rate it reached is the bound
                    diag.setdefault("bounds_raised_to_observed", {})[f"tcp_upload@{round(bmib, 1)}"] = b["mib_s"]
                    bmib = b["mib_s"]
                b.update({"bound": "tcp_upload", "bound_mib_s": round(bmib, 1),
                          "frac_of_bound": round(b["mib_s"] / bmib, 3)})
                full[key] = b
                continue
            if ceil and ceil.get("ok"):
                # the headline's placement: the run's best probe; one L3 domain: its own probe
                tcp = (ceil.get("tcp_gbps_same", 0.0) if extra.get("_place") == "same"
                       else max(tcp_best_gbps, ceil.get("tcp_gbps", 0.0))) or 0.0
                b.update(rp.frac_of_bound(b["mib_s"] / max(1, world), ceil.get("h2d_gbps", 0.0) or 0.0, tcp,
                                          extra.get("_conns"), extra.get("sink") == "gpu" and self.use_gpu))
                if "bound_mib_s" in b:  # per GPU: each rank's bound is its own link / copy engines
                    b["bound_mib_s"] = round(b["bound_mib_s"] * max(1, world), 1)
            full[key] = b
        head_bound = (value, "tcp_1conn", uc["tcp_best_mib_s"] * max(1, world)) if uc else None
        raised = rp.observed_bounds(full, head_bound)
        if raised:
            diag.setdefault("bounds_raised_to_observed", {}).update(raised)
            hb = raised.get(f"tcp_1conn@{round(uc['tcp_best_mib_s'] * max(1, world), 1)}") if uc else None
            if hb and uc.get("ceiling_bound") == "tcp_1conn":
                # a block of the headline's own bound beat every probe: that rate is the ceiling
                out["headline_frac_of_ceiling"] = round(value / hb, 3)
        for key, b in full.items():
            if key.startswith("ref_default_100m_") and key.endswith("_gpu"):
                twin = full.get(key[:-len("_gpu")] + "_discard")
                if twin and twin.get("ok") and twin.get("mib_s"):
                    b["vs_discard_twin"] = round(b["mib_s"] / twin["mib_s"], 3)
        eff_h = full.get("ref_effective_head")
        if eff_h and eff_h.get("ok") and eff_h.get("mib_s") and value > 0:
            # next to, never instead of, vs_baseline (parity-unpinned)
            out["headline_vs_ref_effective"] = round(value / eff_h["mib_s"], 3)
        eff = full.get("ref_effective_grpc")
        if eff and eff.get("ok") and eff.get("mib_s"):
            for key in ("ref_default_100m_grpc_gpu", "ref_default_100m_grpc_discard"):
                if key in full and full[key].get("mib_s"):
                    full[key]["vs_ref_effective"] = round(full[key]["mib_s"] / eff["mib_s"], 3)
        diag["blocks"] = full
        out["diag_file"] = os.path.basename(args.diag_out) if args.diag_out else None
        line = rp.ordered(rp.fit_line(out, full))
        diag["line"] = line
        return line, diag


def _by_node(counts):
    d = {str(i): c for i, c in enumerate(counts[:-1]) if c}
    if counts and counts[-1]:
        d["absent"] = counts[-1]
    return d


def run_rank(args) -> int:
    stash.claim_stdout()
    return RankBench(args).run()
