#!/usr/bin/env python3
"""Headline benchmark: whole-object reads from a (synthetic, loopback) GCS
endpoint into MI355X HBM, one reader process per GPU.

Metric (BASELINE.json): p50/p99 read latency (ms) + MB/s per GPU, HTTP vs gRPC
at 1/2/4/8 MI355X.  Config 2/4: 256 MiB objects, gRPC ReadObject, ONE stream
per object read (the reference's one NewReader + io.CopyBuffer per read,
/root/reference/main.go:134-140); bytes land in HBM through the pinned ring +
hipMemcpyAsync and every ChecksummedData CRC32C and the object CRC32C are
verified by the CDNA4 kernels.  One rank per GPU; rank r reads file_<r>, so
per-GPU work is fixed as N grows (weak scaling, the reference's worker fan-out
/root/reference/main.go:200-210 spread over GPUs).

Timed region: W untimed warm-up reads, then K reads bracketed by an RCCL
barrier + torch.cuda.synchronize() on both sides; `value` = all ranks' bytes /
the slowest rank's elapsed time (MiB/s for the whole job).

After the timed region, as labelled side blocks (same endpoint, every rank):
  compare  the other transport (HTTP vs gRPC) on the headline config;
  sliced   extension, not parity: each read split into N ranged streams on
           their own connections pulling 8 MiB pieces (csrc/storage/sliced.h);
  write    config 5: 64 MiB object in HBM -> D2H into the pinned ring ->
           resumable upload (gRPC StartResumableWrite + WriteObject), GPU CRC.

Launch:
  python bench.py --gpus 1                         one rank on cuda:0
  python bench.py --gpus 8                         spawns 8 rank processes itself
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8
`--workload write` makes config 5 the headline instead.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "p50/p99 read latency (ms) + MB/s per GPU; HTTP vs gRPC at 1/2/4/8 MI355X"


# side blocks a multi-GPU run does by default (the rest with --blocks all)
SCALE_BLOCKS = ("cpu_baseline", "compare", "write", "fanout")


class _Report:
    """Rank 0's output line.  The normal path prints ONE line at the end.
    Once the headline and its baseline are measured, the line so far is
    stashed: if a later side block hangs, the fatal paths -- the barrier
    watchdog (parallel/dist.py on_fatal), the side-block deadline, SIGTERM
    from the rank launcher -- print the stash before the process ends, with
    a non-zero exit status."""

    def __init__(self):
        import threading

        self._lock = threading.Lock()
        self._line = None
        self._printed = False
        self._timer = None

    def stash(self, line: str) -> None:
        with self._lock:
            self._line = line

    def emit_stash(self, why: str = "") -> None:
        with self._lock:
            if self._line is None or self._printed:
                return
            self._printed = True
            line = self._line
        if why:
            print(f"bench: {why}; printing the headline measured so far", file=sys.stderr, flush=True)
        print(line, flush=True)

    def final(self, line: str) -> None:
        with self._lock:
            if self._printed:  # a fatal path already printed the stash
                return
            self._printed = True
        print(line, flush=True)

    def arm(self, seconds: float) -> None:
        """Side blocks must be done within `seconds` (0 = no limit)."""
        import threading

        if seconds <= 0 or self._timer is not None:
            return

        def fire():
            self.emit_stash(f"side blocks still running after {seconds:.0f} s")
            sys.stderr.flush()
            os._exit(3)
        self._timer = threading.Timer(seconds, fire)
        self._timer.daemon = True
        self._timer.start()

    def disarm(self) -> None:
        if self._timer is not None:
            self._timer.cancel()


report = _Report()


def maybe_hang(block: str, rank: int) -> None:
    """Fault injection for the resilience tests: GCSB_TEST_HANG=<block>:<rank>
    makes that rank hang at the start of that side block."""
    spec = os.environ.get("GCSB_TEST_HANG", "")
    if not spec:
        return
    b, _, r = spec.partition(":")
    if b == block and str(rank) == (r or "0"):
        print(f"bench: GCSB_TEST_HANG: rank {rank} hangs in side block {block}", file=sys.stderr, flush=True)
        while True:
            time.sleep(0.2)


def parse_size(s: str) -> int:
    s = s.strip()
    mult = {"k": 1 << 10, "kib": 1 << 10, "m": 1 << 20, "mib": 1 << 20, "g": 1 << 30, "gib": 1 << 30}
    for suf in sorted(mult, key=len, reverse=True):
        if s.lower().endswith(suf):
            return int(float(s[: -len(suf)]) * mult[suf])
    return int(s)


VMSTAT_KEYS = ("numa_hint_faults", "numa_pages_migrated", "thp_fault_alloc", "thp_collapse_alloc", "compact_stall",
               "pgmajfault", "pgfault")


def cpu_snapshot() -> dict:
    """Process CPU time (client + node-local endpoint share this process) and
    the cgroup's CFS throttling counters: on the GPU boxes the container runs
    under a CPU quota (profiles/r1_gpu_box_env.txt), and loopback TCP costs CPU
    at both ends, so these explain throughput and the p99 tail."""
    import resource

    ru = resource.getrusage(resource.RUSAGE_SELF)
    snap = {"user_s": ru.ru_utime, "sys_s": ru.ru_stime, "minflt": ru.ru_minflt, "nivcsw": ru.ru_nivcsw}
    # host-wide memory-management events: NUMA-balancing hinting faults and
    # migrations, THP faults / collapses, compaction stalls -- the kernel
    # work that can slow a receive copy without showing in our own counters
    try:
        with open("/proc/vmstat") as f:
            for line in f:
                k, _, v = line.partition(" ")
                if k in VMSTAT_KEYS:
                    snap["vm_" + k] = int(v)
    except OSError:
        pass
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, _, v = line.partition(" ")
                if k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec"):
                    snap[k] = int(v)
    except OSError:
        pass
    return snap


def receiver_interference(head_cpu: dict, base_cpus: list[dict]) -> dict:
    """The receiving thread's CPU-s per GiB in the headline against the same
    thread in the bracketing baseline runs (both copy every byte out of one
    socket on the same core).  Normally 0.9 - 1.0 (profiles/r4_dist); a
    headline whose receiver cost several times its baseline's while it never
    waited for a CPU ran under host interference (profiles/r4_dist b_4: 3.3x,
    host-wide page faults 10x, function-call IPIs 2x on the placement)."""
    def recv_cost(cpu: dict):
        by = cpu.get("cpu_s_per_gib_by_name") or {}
        for name in ("gcsb-h2-reader", "gcsb-worker", "gcsb-worker (exited)"):
            if by.get(name):
                return float(by[name])
        return None
    h = recv_cost(head_cpu)
    b = [c for c in (recv_cost(x) for x in base_cpus) if c]
    if not h or not b:
        return {}
    ratio = h / (sum(b) / len(b))
    out = {"cpu_s_per_gib": round(h, 4), "baseline_cpu_s_per_gib": round(sum(b) / len(b), 4),
           "cost_ratio": round(ratio, 2)}
    clock = (head_cpu.get("host") or {}).get("clock_mhz_on_placement") or {}
    for k, v in ((head_cpu.get("host") or {}).get("threads") or {}).items():
        if k.startswith(("gcsb-h2-reader", "gcsb-worker")) and v.get("last_cpus"):
            c = clock.get(str(v["last_cpus"][0]))
            if c:
                # the receiving core's clock through the headline
                out["clock_mhz"] = c["mean"]
                out["clock_mhz_min"] = c["min"]
            break
    if ratio >= 2.0:
        th = ((head_cpu.get("host") or {}).get("threads") or {})
        rd = max((v.get("run_delay_ms_per_read", 0.0) for k, v in th.items() if k.startswith("gcsb-h2-reader")
                  or k.startswith("gcsb-worker")), default=0.0)
        out["note"] = ("receive copy ran {:.1f}x its same-run baseline cost per GiB on the same core, run-queue delay "
                       "{:.2f} ms per read, host-wide page faults {} over the headline: host interference, not the "
                       "client path".format(ratio, rd, (head_cpu.get("host_vmstat") or {}).get("pgfault", "n/a")))
    return out


def tcp_sysctls() -> dict:
    """Socket-buffer limits of the box: an explicit SO_RCVBUF is capped at
    net.core.rmem_max (and doubled by the kernel)."""
    out = {}
    for k, path in (("rmem_max", "/proc/sys/net/core/rmem_max"), ("tcp_rmem", "/proc/sys/net/ipv4/tcp_rmem"),
                    ("wmem_max", "/proc/sys/net/core/wmem_max"), ("tcp_wmem", "/proc/sys/net/ipv4/tcp_wmem")):
        try:
            with open(path) as f:
                out[k] = f.read().split()
                if len(out[k]) == 1:
                    out[k] = int(out[k][0])
                else:
                    out[k] = [int(x) for x in out[k]]
        except (OSError, ValueError):
            pass
    try:
        with open("/proc/sys/net/ipv4/tcp_congestion_control") as f:
            out["tcp_congestion_control"] = f.read().strip()
    except OSError:
        pass
    return out


def cpu_delta(a: dict, b: dict, nbytes: float, elapsed: float) -> dict:
    gib = max(nbytes, 1.0) / (1 << 30)
    cpu_s = b["user_s"] + b["sys_s"] - a["user_s"] - a["sys_s"]
    out = {"process_cpu_s_per_gib": round(cpu_s / gib, 4),
           "process_sys_fraction": round((b["sys_s"] - a["sys_s"]) / max(1e-9, cpu_s), 3),
           # CPUs this rank kept busy during the timed region (client + its endpoint)
           "cpus_busy": round(cpu_s / max(elapsed, 1e-9), 2)}
    for k in ("nr_periods", "nr_throttled", "throttled_usec"):
        if k in a and k in b:
            out["cgroup_" + k] = b[k] - a[k]
    out["process_minflt"] = b.get("minflt", 0) - a.get("minflt", 0)
    out["process_involuntary_cs"] = b.get("nivcsw", 0) - a.get("nivcsw", 0)
    vm = {k[3:]: b[k] - a[k] for k in b if k.startswith("vm_") and k in a and b[k] != a[k]}
    if vm:
        out["host_vmstat"] = vm
    return out


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs = rank processes (one per GPU). Without torchrun env, N>1 spawns the ranks itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--write-parts", type=int, default=8,
                    help="write_composite side block: parts of a parallel composite upload (0/1 = off)")
    ap.add_argument("--workload", default="read", choices=["read", "write"],
                    help="read: configs 2/4 (headline); write: config 5 as the headline")
    ap.add_argument("--protocol", default="auto", help="grpc | http | auto (grpc when built)")
    ap.add_argument("--object-size", default="256MiB")
    ap.add_argument("--workers", type=int, default=1, help="readers per GPU (config: 1)")
    ap.add_argument("--sink", default="gpu", help="gpu (HBM landing + GPU CRC) | discard (CPU baseline)")
    ap.add_argument("--slot-bytes", default="1MiB",
                    help="pinned ring slot (one H2D copy + CRC launch each). 4 x 1 MiB: the copy engine reads lines "
                         "still in the receiving CCD's L3; against 8 x 2 MiB the receive copy went 0.046 -> 0.036 "
                         "CPU-s/GiB, 22.0k -> 27.5k MiB/s interleaved (profiles/r4_main8, profiles/r4_recvcost)")
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--conn-ring", default="4x1MiB",
                    help="GPU sink on one multiplexed gRPC connection (list_read_grpc, ref_default_100m_grpc_gpu): "
                         "every worker's stream through one connection ring of SLOTSxBYTES instead of a ring per "
                         "worker (profiles/r4_bigring, r4_connring); off: a ring per worker")
    ap.add_argument("--crc-slice8", default="on", choices=["on", "off"],
                    help="slot CRC kernel stages slice-by-8 tables (8 KiB) instead of slice-by-16 "
                         "(profiles/r4_crc8)")
    ap.add_argument("--crc-slot-waves", type=int, default=0, choices=[0, 1, 2, 4, 8],
                    help="slot CRC kernel waves per workgroup (0: by slot size); A/B of the kernel's table staging")
    ap.add_argument("--async-submit", type=int, default=1, choices=[0, 1],
                    help="slot hand-off (H2D copy + CRC launches) on a per-device submitter thread instead of the "
                         "receiving thread: one stream per read is bound by its receiving core, so taking the HIP "
                         "calls off it gave +15-35%% (profiles/r2_single_stream)")
    ap.add_argument("--submit-cpus", default="aux", choices=["aux", "inherit"],
                    help="aux: the per-device submitter thread gets a core of its own from the placement plan; "
                         "inherit: it keeps the first posting transport thread's CPU set")
    ap.add_argument("--rcvbuf", default="64MiB",
                    help="client SO_RCVBUF of the headline read (0 = kernel autotuning). An explicit 64 MiB request "
                         "(capped at net.core.rmem_max = 32 MiB on the GPU boxes, doubled by the kernel) won 5 of 8 "
                         "interleaved pairs against autotuning, medians 16.8k/14.0k vs 13.3k/13.4k MiB/s over two "
                         "boxes (profiles/r2_rcvbuf); the box's limits are reported in the JSON line")
    ap.add_argument("--grpc-pool", type=int, default=1)
    ap.add_argument("--slices", type=int, default=1,
                    help="streams per object read in the HEADLINE run (1 = the reference's sequential read)")
    ap.add_argument("--sliced-streams", type=int, default=8,
                    help="streams per read in the `sliced` extension block (0 = skip the block)")
    ap.add_argument("--sliced-slot-bytes", default="2MiB",
                    help="sliced block: ring slot per sink (2 MiB x 8 won 2 of 2 interleaved reps against 4 x 4 MiB, "
                         "8 MiB x 2, 4/16 pool streams and async hand-off: profiles/r2_sliced)")
    ap.add_argument("--sliced-slots", type=int, default=2,
                    help="sliced block: ring slots per sink. With the THP endpoint the receive copies are the "
                         "bound and each stream's 2 sinks x ring is its destination footprint: 2 x 2 MiB ran "
                         "46.3-49.9k MiB/s against 41.5-45.0k with 8 x 2 MiB (profiles/r3_ring_thp/sliced)")
    ap.add_argument("--sliced-async-submit", type=int, default=0, choices=[0, 1],
                    help="sliced block: slot hand-off on the device submitter thread (default inline)")
    ap.add_argument("--piece-bytes", default="8MiB",
                    help="sliced reads: streams pull pieces of this size from a shared cursor (0 = fixed shares)")
    ap.add_argument("--piece-min-bytes", default="0",
                    help="sliced reads: taper the piece size toward the end of the object down to this")
    ap.add_argument("--affinity", default="auto",
                    help="CPU placement of client/endpoint threads: auto|pair|share|same|split|numa|none "
                         "(parallel/affinity.py). auto: pair for one stream per read (won 3 of 3 interleaved "
                         "reps, profiles/r2_placement), share for sliced reads; the sliced block always runs "
                         "on its own share-placed endpoint")
    ap.add_argument("--event-wait", default="block", choices=["spin", "block"],
                    help="how GPU sinks wait on slot events: block (interrupt) or spin")
    ap.add_argument("--side-steps", type=int, default=-1,
                    help="timed reads/uploads per side block (compare / sliced / write); -1: = --steps, 0: skip all")
    ap.add_argument("--fanout", default="on", choices=["on", "off"],
                    help="N > 1 side block: each rank reads 1/N of one shared object, an all-gather over the "
                         "GPUs gives every GPU the whole object (extension)")
    ap.add_argument("--list-objects", type=int, default=1000,
                    help="config 3 side block: list this many 1 MiB objects, read each into HBM (0 = off)")
    ap.add_argument("--list-workers", type=int, default=8, help="config 3 side block: readers")
    ap.add_argument("--list-ring", default="2x1MiB",
                    help="config 3 side block: pinned ring per reader, SLOTSxSLOT_BYTES (1 MiB objects). 2 x 1 MiB "
                         "keeps the 8 readers' receive destinations at 16 MiB: gRPC 18.6-18.8k MiB/s at p50 "
                         "0.42 ms against 15.5-17.0k at 0.46-0.49 with 8 x 2 MiB (profiles/r3_mux_thp/listring)")
    ap.add_argument("--list-ring-wc", default="on", choices=["on", "off"],
                    help="config 3 side block: the readers' rings in write-combined pinned memory (p50 0.346-0.379 "
                         "ms against 0.412-0.519 with cached THP rings, profiles/r3_ring_thp/wc)")
    ap.add_argument("--write-size", default="64MiB", help="config 5 object size")
    ap.add_argument("--write-chunk", default="16MiB", help="resumable upload chunk (HTTP) / message batch")
    ap.add_argument("--baseline", default="on", choices=["on", "off"],
                    help="cpu_baseline side blocks: the headline config with the reference's semantics (discard "
                         "sink, host CRC32C; /root/reference/main.go:133-146) on the same endpoint, placement and "
                         "steps, for the headline protocol and the other one; vs_baseline = value / it")
    ap.add_argument("--baseline-bracket", default="auto", choices=["auto", "on", "off"],
                    help="also run the reference-semantics baseline right before the headline (cpu_baseline_before): "
                         "vs_baseline then divides by the pooled rate of the two runs that bracket the headline, so a "
                         "host drifting between blocks cancels (the same baseline swung 12%% between two benches on "
                         "one box, profiles/r4_main9).  auto: on at N = 1; off at N > 1, where nothing may run "
                         "before the headline")
    ap.add_argument("--ceiling", default="on", choices=["on", "off"],
                    help="ceiling side block: one loopback TCP stream (sendfile -> recv into a THP ring, no GPU, "
                         "no framing) and pinned -> HBM copies, in the headline's placement")
    ap.add_argument("--ref-workers", type=int, default=48,
                    help="ref_default_* side blocks: the reference's default experiment, -worker 48 on 1 MiB "
                         "objects, gRPC pool 1 vs HTTP keep-alive, discard sink + host CRC (0 = off)")
    ap.add_argument("--ref-reads", type=int, default=50, help="ref_default_*: timed reads per worker")
    ap.add_argument("--ref-grpc-placement", default="same", choices=["share_quota", "same", "share", "pair"],
                    help="ref_default_grpc: CPU placement of the 48 workers, the endpoint and the one connection's "
                         "reader. One L3 domain (same): 16.0-19.5k MiB/s at p50 2.1-2.4 ms against 8.4-8.8k at "
                         "4.5-5.0 ms spread over the quota's cores (profiles/r3_mux_thp/refplace). HTTP keeps "
                         "share_quota: its 48 receiving workers need the cores")
    ap.add_argument("--ref-object-size", default="1MiB", help="ref_default_*: object size")
    ap.add_argument("--ref-http-placement", default="share_quota", choices=["share_quota", "split_quota"],
                    help="ref_default_http*: client workers and endpoint handlers over the rank's quota cores "
                         "together (share_quota) or on separate cores, a quarter for the endpoint (split_quota)")
    ap.add_argument("--ref100-reads", type=int, default=3,
                    help="ref_default_100m_* blocks: the reference's real operating point, 48 workers x 100 MiB "
                         "objects (princer_100M_files), HTTP vs gRPC pool 1, discard + host CRC vs HBM + GPU CRC; "
                         "timed reads per worker (0 = off)")
    ap.add_argument("--ref-gpu-ring", default="2x2MiB",
                    help="ref_default_100m_*_gpu: pinned ring per worker, SLOTSxSLOT_BYTES")
    ap.add_argument("--write-placement", default="pair", choices=["share", "pair"],
                    help="config-5 upload block: pair (uploader on one quiet core, endpoint receive + CRC on two "
                         "more of the same L3 domain; 18.0-21.6k MiB/s in 6 runs) or share (uploader and endpoint "
                         "threads over the rank's share of L3 domains; 7.7-19.7k, profiles/r3_write/placement)")
    ap.add_argument("--list-rcvbuf", default="64MiB",
                    help="config-3 list-read blocks: client SO_RCVBUF (0 = kernel autotuning; 64 MiB as the headline, "
                         "profiles/r3_w48_tail)")
    ap.add_argument("--mux-reader", default="shared", choices=["shared", "isolate"],
                    help="multiplexed blocks (list_read_grpc, ref_default_grpc): isolate gives the connection's "
                         "reader thread a physical core the workers and endpoint do not use (affinity.isolate_reader)")
    ap.add_argument("--blocks", default="",
                    help="comma list of side blocks to run (A/B sessions): cpu_baseline, compare, sliced, ceiling, "
                         "ref_default, c1_http_cpu, list_read, write, write_composite, fanout; 'all' = every block; empty = "
                         "all at N = 1, cpu_baseline,compare,write,fanout at N > 1")
    ap.add_argument("--client-cc", default="cubic",
                    help="client sockets' TCP congestion control, set before connect (\"\" = the host default, BBR "
                         "on the GPU boxes, whose internal pacing arms an hrtimer per 64 KiB skb of an upload on a "
                         "loopback link: profiles/r4_recvcost). Every block uses it, baselines included")
    ap.add_argument("--recv-refill", type=int, default=0, choices=[0, 1],
                    help="client sockets: a payload recv() also reads what follows it (the next HTTP/2 frame "
                         "header) in the same recvmsg (SocketOptions::recv_refill)")
    ap.add_argument("--read-diag", action="store_true",
                    help="per-read stall attribution (Runner read_diag): scheduler and softirq deltas of the "
                         "receiving / sending threads around every timed read; the slowest reads carry them and a "
                         "named cause (rank0_slowest_diag). Costs tens of us per read outside its latency")
    ap.add_argument("--side-deadline", type=float, default=300.0,
                    help="seconds the side blocks after the headline + cpu_baseline may take before rank 0 prints "
                         "the headline line measured so far and exits 3 (0 = no limit)")
    ap.add_argument("--json-out", default="")
    return ap


# ---------------------------------------------------------------------------
# launcher: one process per GPU


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv: list[str]) -> int:
    """Spawns n rank processes (torchrun-style env) running this script and
    waits for them.  The parent never imports torch or touches HIP, so no
    process that initialised the GPU ever starts another program.  If a rank
    fails, the others are terminated (their exact PIDs) and the worst exit
    status is returned."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    live = set(range(n))

    def _forward(signum, frame):  # the driver's time limit: let every rank print what it has
        for q in live:
            procs[q].send_signal(signal.SIGTERM)
    signal.signal(signal.SIGTERM, _forward)
    try:
        while live:
            for r in sorted(live):
                c = procs[r].poll()
                if c is None:
                    continue
                live.discard(r)
                if c != 0:
                    print(f"bench: rank {r} exited with status {c}; stopping the other ranks", file=sys.stderr)
                    rc = rc or (c if c > 0 else 1)
                    for q in live:
                        procs[q].send_signal(signal.SIGTERM)
            time.sleep(0.05)
    except KeyboardInterrupt:
        for q in live:
            procs[q].send_signal(signal.SIGTERM)
        for q in live:
            procs[q].wait()
        return 130
    return rc


# ---------------------------------------------------------------------------
# one rank


def run_rank(args) -> int:
    import torch

    import custom_go_client_benchmark_amd as pkg
    from custom_go_client_benchmark_amd.ops import hbm
    from custom_go_client_benchmark_amd.parallel import affinity
    from custom_go_client_benchmark_amd.parallel import dist as gdist
    from custom_go_client_benchmark_amd.utils import cpuacct, sysdiag

    n = pkg._native
    rank, world, local_rank = gdist.env_rank()
    if args.gpus != world:
        print(f"bench: --gpus {args.gpus} but the launcher started {world} rank(s) (WORLD_SIZE); "
              f"they must match", file=sys.stderr)
        return 2
    use_gpu = args.sink == "gpu"
    rehearsal = os.environ.get("GCSB_DIST_BACKEND") == "gloo"
    if use_gpu:
        hbm.gpu_required()
        ndev = torch.cuda.device_count()
        if world > ndev and not rehearsal:
            print(f"bench: {world} ranks but only {ndev} visible GPU(s); one rank per GPU "
                  f"(set GCSB_DIST_BACKEND=gloo for a shared-GPU rehearsal)", file=sys.stderr)
            return 2
    # process group even at world 1: RCCL init + barriers + reductions run in every GPU bench
    ctx = gdist.init(local_rank=local_rank, world=world, rank=rank, always_pg=use_gpu)
    if rank == 0:
        # a peer that never reaches a barrier ends this rank through the
        # watchdog, and the launcher ends a hung rank with SIGTERM: either
        # way the stashed headline line is printed first
        gdist.on_fatal(lambda: report.emit_stash("a barrier timed out"))

        def _term(signum, frame):
            report.emit_stash("terminated")
            sys.stdout.flush()
            os._exit(128 + signum)
        signal.signal(signal.SIGTERM, _term)
    protocol = args.protocol
    if protocol == "auto":
        protocol = "grpc" if "grpc" in hbm.available_protocols() else "http"
    size = parse_size(args.object_size)
    side_steps = args.steps if args.side_steps < 0 else args.side_steps
    # side blocks get the headline's warm-up too: each opens fresh connections
    # (and an endpoint of its own), so one warm-up read/upload left its first
    # timed one carrying setup -- the write block's p99 of 14 ms over 20
    # uploads against p99 9.4 ms over 200 back-to-back ones on one box
    # (profiles/r2_write/tail_probe_*.json)
    side_warm = max(1, args.warmup)

    # node-local synthetic GCS endpoint for this rank (no network on the box)
    gpu = ctx.gpu if ctx.gpu >= 0 else 0
    aff = args.affinity
    if aff == "auto":
        aff = "pair" if args.slices == 1 else "share"
    # ranks sharing one GPU (rehearsal) spread over L3 domains instead of stacking
    slot = local_rank // max(1, torch.cuda.device_count()) if use_gpu and rehearsal else 0
    placement = affinity.plan(gpu, aff, slot) if use_gpu else {"client": [], "server": []}
    if use_gpu and args.submit_cpus == "aux" and placement.get("aux"):
        n.set_submitter_cpus(placement["aux"])
    if use_gpu and (args.crc_slot_waves or args.crc_slice8 == "off"):
        n.set_crc_options({"slot_waves": args.crc_slot_waves, "slice8": args.crc_slice8 == "on"})
    srv = n.Server({"port": 0, "md5": False, "cpus": placement["server"], "retain_uploads": False})
    srv.start()
    bucket = "princer-working-dirs"
    prefix = "princer_100M_files/file_"
    first = rank * args.workers
    srv.add_synthetic(bucket, prefix, "", first, args.workers, size)

    cfg = {
        "protocol": protocol,
        "endpoint": srv.url,
        "bucket": bucket,
        "object_prefix": prefix,
        "workers": args.workers,
        "reads_per_worker": args.warmup,
        "worker_id_offset": first,
        "sink": args.sink,
        "device": gpu if use_gpu else 0,
        "ring_slot_bytes": parse_size(args.slot_bytes),
        "ring_slots": args.slots,
        "conn_ring": args.conn_ring != "off",
        "conn_ring_slots": int(args.conn_ring.partition("x")[0]) if "x" in args.conn_ring else 4,
        "conn_ring_slot_bytes": parse_size(args.conn_ring.partition("x")[2]) if "x" in args.conn_ring else 1 << 20,
        "landing": "object",
        "grpc_conn_pool_size": args.grpc_pool,
        "keep_records": False,
        "cpus": placement["client"],
        "retry_initial_s": 0.05,
        "slices": args.slices,
        "slice_piece_bytes": parse_size(args.piece_bytes),
        "slice_piece_min_bytes": parse_size(args.piece_min_bytes),
        "blocking_sync": args.event_wait == "block",
        "async_submit": bool(args.async_submit),
        "rcvbuf": parse_size(args.rcvbuf),
        "tcp_congestion": args.client_cc,
        "loopback_rto_min": True,
        "recv_refill": bool(args.recv_refill),
    }
    # the sliced extension: inline slot hand-off (r1_submit_ab), 2 MiB x 8
    # ring per sink (profiles/r2_sliced)
    sliced_cfg = {"slices": args.sliced_streams, "ring_slot_bytes": parse_size(args.sliced_slot_bytes),
                  "ring_slots": args.sliced_slots, "async_submit": bool(args.sliced_async_submit), "rcvbuf": 0}

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def read_ok(s: dict, steps: int, workers: int) -> tuple[bool, str]:
        reads = steps * workers
        if s["errors"]:
            return False, s["first_error"] or "read error"
        if s["reads"] != reads:
            return False, f"{s['reads']} of {reads} reads completed"
        # every read must have had its checksums verified (GPU CRC or host CRC)
        if (use_gpu or cfg.get("host_crc", True)) and s["verified"] != reads:
            return False, f"only {s['verified']} of {reads} reads had their CRC32C verified"
        return True, ""

    def read_block(overrides: dict, steps: int, warmup: int, what: str, endpoint=None) -> dict:
        """warm-up reads, then `steps` timed reads of a config variant between
        two barriers.  Every rank makes every collective call whatever happens
        locally, so one rank's failure cannot strand the others in a barrier."""
        err = ""
        r1 = s1 = None
        c0 = th0 = None
        try:
            r1 = n.Runner({**cfg, **overrides, "reads_per_worker": warmup})
            if warmup > 0:
                r1.start()
                r1.wait()
                sw = r1.summary()
                if sw["errors"]:
                    err = f"warmup: {sw['first_error']}"
            r1.reset_stats()
            r1.set_reads_per_worker(steps)
        except Exception as e:  # noqa: BLE001 - reported in the block, collectives still run
            err = err or f"{type(e).__name__}: {e}"
        gdist.barrier(ctx, f"R1 {what} start barrier")
        sync()
        t1 = time.perf_counter()
        rv0 = n.recv_stats()
        rd0 = n.recv_diag()
        h2s0 = n.h2_reader_stats()
        ep_stats = (endpoint or srv).stats
        sv0 = ep_stats()
        if use_gpu:
            n.reset_slow_hip_calls()
        win = None
        if not err:
            c0, th0 = cpu_snapshot(), cpuacct.thread_cpu()
            diag_cpus = sorted(set(overrides.get("cpus") or cfg.get("cpus") or [])
                               | set(placement.get("server") or []) | set(placement.get("aux") or []))
            # the placement cores' clock through the block (a few cores only)
            win = sysdiag.Window(clock_cpus=diag_cpus if 0 < len(diag_cpus) <= 16 else None)
            t1 = time.perf_counter()
            r1.start()
            r1.wait()
        sync()
        gdist.barrier(ctx, f"R2 {what} stop barrier")
        e1 = time.perf_counter() - t1
        cpu = {}
        if not err:
            s1 = r1.summary()
            ok, why = read_ok(s1, steps, overrides.get("workers", args.workers))
            if not ok:
                err = why
            cpu = cpu_delta(c0, cpu_snapshot(), float(s1["bytes"]), e1)
            # what else ran on the block's CPUs: run-queue delay of our
            # threads, interrupts and softirqs there (utils/sysdiag.py)
            cpu["host"] = win.report(diag_cpus or None, max(1, int(s1["reads"])))
            th1 = cpuacct.thread_cpu()
            cpu["cpu_s_per_gib_by_thread"] = cpuacct.per_gib(cpuacct.delta_by_group(th0, th1), float(s1["bytes"]))
            names = cpuacct.delta_by_name(th0, th1)
            # worker threads exit at the end of the run: their CPU comes from the runner
            names.pop("gcsb-worker", None)
            names["gcsb-worker (exited)"] = s1.get("worker_cpu_s", 0.0)
            cpu["cpu_s_per_gib_by_name"] = {k: v for k, v in cpuacct.per_gib(names, float(s1["bytes"])).items()
                                            if v >= 0.0005}
            h2s1 = n.h2_reader_stats()
            if h2s1["frames"] > h2s0["frames"]:
                # the HTTP/2 connection readers (gRPC): where their time went, per GiB
                d = {k: h2s1[k] - h2s0[k] for k in h2s1}
                g = max(float(s1["bytes"]), 1.0) / (1 << 30)
                cpu["h2_reader"] = {"frames_per_read": round(d["frames"] / max(1, s1["reads"]), 2),
                                    "wait_s_per_gib": round(d["header_wait_ns"] / 1e9 / g, 4),
                                    "data_s_per_gib": round(d["data_ns"] / 1e9 / g, 4),
                                    "headers_s_per_gib": round(d["headers_ns"] / 1e9 / g, 4),
                                    "other_s_per_gib": round(d["other_ns"] / 1e9 / g, 4),
                                    "avg_data_frame_kib": round(d["data_bytes"] / max(1, d["data_frames"]) / 1024, 1)}
            cr = r1.conn_ring_stats()
            if cr:
                # the multiplexed connection's shared receive ring (warmup included)
                cpu["conn_ring"] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in cr.items()}
            g1 = s1.get("gpu") or {}
            if g1.get("slot_waits") or g1.get("flag_reuses"):
                # the receiving thread reusing ring slots: on the CRC kernel's
                # host-visible status (no HIP call), or waiting for the slot's
                # hand-off + its event; then harvesting its CRC results
                gib = max(float(s1["bytes"]) / (1 << 30), 1e-9)
                cpu["slot_reuse"] = {"waits": g1["slot_waits"], "on_kernel_status": g1.get("flag_reuses", 0),
                                     "s_per_gib": round(g1["slot_wait_s"] / gib, 4),
                                     # the receiving thread inside submit + take (bookkeeping, hand-off, waits)
                                     "handoff_s_per_gib": round(g1.get("handoff_s", 0.0) / gib, 5)}
            sv1 = ep_stats()
            if sv1.get("h2_data_frames", 0) > sv0.get("h2_data_frames", 0):
                # the endpoint's HTTP/2 fairness: how long stream handlers
                # queued per DATA frame, and request -> response HEADERS
                fr = sv1["h2_data_frames"] - sv0["h2_data_frames"]
                rs = max(1, sv1["h2_responses"] - sv0["h2_responses"])
                cpu["endpoint_h2"] = {"frames": fr,
                                      "queue_wait_avg_us": round((sv1["h2_queue_wait_us"] - sv0["h2_queue_wait_us"]) / fr, 1),
                                      "queue_wait_max_us": sv1["h2_queue_wait_max_us"],
                                      "ttfb_avg_us": round((sv1["h2_ttfb_us"] - sv0["h2_ttfb_us"]) / rs, 1),
                                      "ttfb_max_us": sv1["h2_ttfb_max_us"]}
            if sv1.get("body_sends", 0) > sv0.get("body_sends", 0):
                # the endpoint's sends of this block's bodies, by the kernel's
                # send chronographs: busy, held by the client's receive window
                # (the client is the bound), held by its own send buffer
                wall = max(1, sv1["body_wall_us"] - sv0["body_wall_us"])
                sends = sv1["body_sends"] - sv0["body_sends"]
                cpu["endpoint_tcp"] = {
                    "busy_frac": round((sv1["tcp_busy_us"] - sv0["tcp_busy_us"]) / wall, 3),
                    "rwnd_limited_frac": round((sv1["tcp_rwnd_limited_us"] - sv0["tcp_rwnd_limited_us"]) / wall, 3),
                    "sndbuf_limited_frac": round((sv1["tcp_sndbuf_limited_us"] - sv0["tcp_sndbuf_limited_us"]) / wall,
                                                 3),
                    "cwnd_kib_at_end": round((sv1["tcp_cwnd_bytes_sum"] - sv0["tcp_cwnd_bytes_sum"]) / sends / 1024, 1)}
            rv1 = n.recv_stats()
            calls = rv1[0] - rv0[0]
            if calls:
                # average bytes per recv() on the client's sockets (every
                # Conn::read_some of the process: client side only here)
                cpu["recv_calls"] = calls
                cpu["recv_avg_kib"] = round((rv1[1] - rv0[1]) / calls / 1024.0, 1)
            rd1 = n.recv_diag()
            dc = rd1["calls"] - rd0["calls"]
            if dc:
                # GCSB_RECV_DIAG=1: the socket queue at each payload recv() --
                # how often the receiver found it empty (it outran the sender)
                cpu["recv_queue"] = {"payload_recvs": dc,
                                     "empty_frac": round((rd1["empty"] - rd0["empty"]) / dc, 3),
                                     "short_frac": round((rd1["short"] - rd0["short"]) / dc, 3),
                                     "avg_queued_kib": round((rd1["inq_bytes"] - rd0["inq_bytes"]) / dc / 1024, 1),
                                     "avg_asked_kib": round((rd1["want_bytes"] - rd0["want_bytes"]) / dc / 1024, 1),
                                     # wall time inside those recv() calls, per GiB read
                                     "recv_s_per_gib": round((rd1["recv_ns"] - rd0["recv_ns"]) / 1e9
                                                             / max(float(s1["bytes"]) / (1 << 30), 1e-9), 4)}
        slow_hip = n.slow_hip_calls() if use_gpu else {}
        ring_numa = r1.ring_numa(0) if (r1 is not None and use_gpu) else []
        ring_thp = r1.ring_thp_fraction(0) if (r1 is not None and use_gpu) else -1.0
        s1 = s1 or {"bytes": 0, "p50_ms": 0.0, "p99_ms": 0.0, "host_p50_ms": 0.0, "ttfb_p50_ms": 0.0, "slice_skew_ms": 0.0,
                    "verified": 0, "reads": 0}
        del r1
        st = gdist.reduce_stats(ctx, elapsed=e1, nbytes=float(s1["bytes"]), p50=s1["p50_ms"], p99=s1["p99_ms"],
                                host_p50=s1["host_p50_ms"], ttfb_p50=s1.get("ttfb_p50_ms", 0.0),
                                skew=s1.get("slice_skew_ms", 0.0), first_p50=s1.get("first_read_p50_ms", 0.0),
                                steady_p99=s1.get("steady_p99_ms", 0.0),
                                verified=float(s1["verified"]), ok=0.0 if err else 1.0)
        st["error"] = err
        st["cpu"] = cpu
        st["ring_numa"] = ring_numa
        st["ring_thp"] = ring_thp
        # this rank's slowest reads [index in the timed run, ms, host-landed ms,
        # TTFB ms] and the slot hand-off HIP calls that blocked (>= 1 ms)
        st["slowest"] = [[int(x[0])] + [round(v, 3) for v in x[1:]] for x in (s1.get("slowest") or [])]
        if s1.get("slowest_diag"):
            # per slow read: what the scheduler / softirqs did meanwhile, and the named cause
            st["slowest_diag"] = [
                {"read": int(x[0]), "ms": round(x[1], 3),
                 "cause": sysdiag.attribute(dg, x[1], s1["p50_ms"]),
                 "threads": {k: {f: (round(v, 3) if isinstance(v, float) else v) for f, v in row.items()}
                             for k, row in dg["threads"].items()},
                 "softirqs": dg["softirqs"], "tcp": dg.get("tcp", {}), "softnet": dg.get("softnet", {})}
                for x, dg in zip(s1["slowest"], s1["slowest_diag"])]
        st["slow_hip"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in slow_hip.items()}
        return st

    def share_endpoint():
        """An endpoint of its own on the rank's share of L3 domains: the
        sliced block's 8 send threads, and uploads, whose receive + CRC32C
        on the endpoint is as heavy as the client's send (the headline's
        one-core pair endpoint halved the upload rate)."""
        sh = affinity.plan(gpu, "share", slot) if use_gpu else {"client": [], "server": []}
        e = n.Server({"port": 0, "md5": False, "cpus": sh["server"], "retain_uploads": False})
        e.start()
        e.add_synthetic(bucket, prefix, "", first, args.workers, size)
        return e, sh

    def write_block(steps: int, warmup: int, parts: int = 1) -> dict:
        """Config 5: each rank uploads a 64 MiB object from HBM `steps` times
        (HBM -> pinned ring D2H on a side stream -> resumable upload; the
        object CRC32C is computed on the GPU and checked by the endpoint).
        parts > 1 [extension]: parallel composite upload -- `parts` slices
        uploaded on their own connections, composed server-side, the composed
        CRC32C checked against the combine of the parts' GPU CRCs
        (csrc/storage/sliced.h SlicedWriter; gsutil's parallel composite
        uploads)."""
        err = ""
        lat = []
        wsize = parse_size(args.write_size)
        chunk = parse_size(args.write_chunk)
        client = buf = None
        ep = None
        saved_aff = os.sched_getaffinity(0)
        try:
            if parts == 1 and use_gpu and args.write_placement == "pair":
                # three quiet cores of one L3 domain: the uploader (this
                # thread) on one, the endpoint's receive and CRC threads on
                # the other two.  Spread over the share, the endpoint's
                # receive thread paid 0.08-0.12 CPU-s/GiB in half the runs
                # (0.043-0.059 paired) and the upload ran at 7.7-11k MiB/s
                # instead of 18-21.6k (profiles/r3_write/placement)
                pl = affinity.plan(gpu, "pair", slot)
                sh = {"client": pl["client"], "server": sorted(pl["server"] + pl.get("aux", []))}
                ep = n.Server({"port": 0, "md5": False, "cpus": sh["server"], "retain_uploads": False})
                ep.start()
            else:
                ep, sh = share_endpoint()
            # the upload runs on this (Python main) thread: keep it, its
            # connection reader and the pinned staging ring it allocates on
            # the GPU's NUMA node (the rank's share of L3 domains); unpinned
            # it could stage from the other socket (p50 6.9 vs 14.3 ms
            # between otherwise identical runs)
            if sh["client"]:
                os.sched_setaffinity(0, sh["client"])
            client = n.Client({"protocol": protocol, "endpoint": ep.url, "retry_initial_s": 0.05,
                               "tcp_congestion": args.client_cc, "loopback_rto_min": True})
            if parts > 1:
                client = n.SlicedWriter({"protocol": protocol, "endpoint": ep.url, "retry_initial_s": 0.05,
                                         "tcp_congestion": args.client_cc, "loopback_rto_min": True,
                                         "slices": parts, "slice_min_bytes": 1 << 20, "cpus": sh["client"]})
            buf = torch.empty(wsize, dtype=torch.uint8, device=f"cuda:{gpu}")
            n.gpu_fill_pattern(gpu, buf.data_ptr(), wsize, f"upload/rank{rank}", 0)
            for i in range(warmup):
                client.write_from_device(bucket, f"upload/warmup_{rank}_{i}", buf.data_ptr(), wsize, gpu, True,
                                         chunk, parse_size(args.slot_bytes), args.slots)
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
        gdist.barrier(ctx, "R1 write start barrier")
        sync()
        n.reset_slow_hip_calls()
        th0 = cpuacct.thread_cpu()
        t1 = time.perf_counter()
        nbytes = 0
        if not err:
            try:
                for i in range(steps):
                    t0 = time.perf_counter()
                    m = client.write_from_device(bucket, f"upload/rank{rank}_{i}", buf.data_ptr(), wsize, gpu,
                                                 True, chunk, parse_size(args.slot_bytes), args.slots)
                    lat.append((time.perf_counter() - t0) * 1e3)
                    # (SlicedWriter checks the composed CRC32C itself)
                    if m["size"] != wsize or (parts == 1 and m["crc32c"] != m["gpu_crc32c"]):
                        err = f"upload {i} not confirmed: {m}"
                        break
                    nbytes += wsize
            except Exception as e:  # noqa: BLE001
                err = f"{type(e).__name__}: {e}"
        sync()
        gdist.barrier(ctx, "R2 write stop barrier")
        e1 = time.perf_counter() - t1
        # where an upload's CPU goes: the sending (Python main) thread and the
        # client's connection reader vs the endpoint's receive and CRC threads
        by_name = {k: v - th0.get(k, 0.0) for k, v in cpuacct.thread_cpu().items()}
        cpu_split = {k: round(v / max(nbytes, 1) * (1 << 30), 4) for k, v in sorted(by_name.items())
                     if v > 0.0005 and nbytes}
        s = sorted(lat)
        p50 = s[len(s) * 50 // 100] if s else 0.0
        p99 = s[min(len(s) - 1, len(s) * 99 // 100)] if s else 0.0
        if ep is not None:
            del client
            ep.stop()
        os.sched_setaffinity(0, saved_aff)
        st = gdist.reduce_stats(ctx, elapsed=e1, nbytes=float(nbytes), p50=p50, p99=p99, ok=0.0 if err else 1.0)
        st["error"] = err
        # this rank's slowest uploads (index in the timed run, ms): where the tail sits
        st["slowest"] = [[i, round(v, 2)] for i, v in sorted(enumerate(lat), key=lambda x: -x[1])[:3]]
        st["slow_hip"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in n.slow_hip_calls().items()}
        st["cpu_s_per_gib_by_thread"] = cpu_split
        return st

    def fanout_block(steps: int, warmup: int) -> dict:
        """[extension, N > 1] read once per node, fan out over xGMI: every rank
        reads only its 1/N slice of ONE shared 256 MiB object (ranged gRPC
        read into HBM, per-message CRC32C on the GPU), then an RCCL
        all-gather over the node's GPUs gives every GPU the whole object,
        whose CRC32C each GPU then checks.  Against the headline (every GPU
        pulls the whole object over its own stream) the network/loopback
        bytes drop N-fold and the rest rides xGMI."""
        err = ""
        lat = []
        crc_ok = 0
        part_n = size // world
        name = "fanout/obj_0"
        full = part = sink = client = None
        try:
            if size % world:
                raise ValueError(f"object size {size} not divisible by {world} ranks")
            srv.add_synthetic(bucket, "fanout/obj_", "", 0, 1, size)
            want = srv.object_info(bucket, name)["crc32c"]
            client = n.Client({"protocol": protocol, "endpoint": srv.url, "retry_initial_s": 0.05,
                               "tcp_congestion": args.client_cc, "loopback_rto_min": True,
                               "cpus": placement["client"], "rcvbuf": parse_size(args.rcvbuf)})
            full = torch.empty(size, dtype=torch.uint8, device=f"cuda:{gpu}" if use_gpu else "cpu")
            # this rank's slice lands in place: the all-gather's input is the
            # slice of its output at rank * part_n (in-place all-gather)
            part = full[rank * part_n:(rank + 1) * part_n]
            if use_gpu:
                sink = n.GpuSink({"device": gpu, "ring_slot_bytes": parse_size(args.slot_bytes),
                                  "ring_slots": args.slots})
                # capacity to the end of the buffer: a ranged read learns the
                # whole object's size and the sink checks it fits
                sink.set_external_destination(part.data_ptr(), size - rank * part_n)
        except Exception as e:  # noqa: BLE001 - reported in the block, collectives still run
            err = f"{type(e).__name__}: {e}"

        for i in range(warmup + steps):
            # every rank makes the same collective calls whatever happened
            # locally: a failed slice read is reported after the all-gather
            flags = gdist.reduce_stats(ctx, ok=0.0 if err else 1.0)
            if flags["ok_min"] < 1.0:
                err = err or "a peer rank failed"
                break
            gdist.barrier(ctx, "fan-out start")
            t0 = time.perf_counter()
            local = ""
            try:
                if use_gpu:
                    r = client.read_gpu(bucket, name, sink, rank * part_n, part_n)
                    if r["bytes"] != part_n or r["crc_mismatch"]:
                        local = f"slice read failed: {r}"
                else:  # CPU rehearsal: the slice through host memory
                    b = client.read_bytes(bucket, name, rank * part_n, part_n)
                    part.copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
            except Exception as e:  # noqa: BLE001
                local = f"{type(e).__name__}: {e}"
            try:
                gdist.all_gather_bytes(ctx, full, part, "fan-out all-gather")
                sync()
            except Exception as e:  # noqa: BLE001 - the process group is gone: no more collectives
                err = f"all-gather: {type(e).__name__}: {e}"
                return {"ok_min": 0.0, "p50_max": 0.0, "p99_max": 0.0, "crc_ok_sum": 0.0, "nbytes_sum": 0.0,
                        "elapsed_max": 0.0, "error": err}
            gdist.barrier(ctx, "fan-out stop")
            if local:
                err = local
            elif i >= warmup:
                lat.append((time.perf_counter() - t0) * 1e3)
        if not err:
            got = n.gpu_crc32c(gpu, full.data_ptr(), size) if use_gpu else n.crc32c(full.numpy().tobytes())
            crc_ok = int(got == want)
            if not crc_ok:
                err = "CRC32C of the gathered object does not match"
        s_ = sorted(lat)
        p50 = s_[len(s_) * 50 // 100] if s_ else 0.0
        p99 = s_[min(len(s_) - 1, len(s_) * 99 // 100)] if s_ else 0.0
        # every GPU ends each step with the whole object: size bytes per rank per step
        st = gdist.reduce_stats(ctx, elapsed=sum(lat) / 1e3, nbytes=float(size * len(lat)), p50=p50, p99=p99,
                                ok=0.0 if err else 1.0, crc_ok=float(crc_ok))
        st["error"] = err
        del part, full, sink
        return st

    def list_read_block(proto: str, warmup_passes: int) -> dict:
        """Config 3 (BASELINE.json): list `--list-objects` 1 MiB objects, then
        `--list-workers` readers read every listed object once into HBM, GPU
        CRC32C on every read (reference list_operation + read_operation; the
        CLI's -workload list-read).  One timed pass after untimed ones; the
        listing's own time is reported apart (list_ms)."""
        nobj, workers = args.list_objects, args.list_workers
        # one L3 domain for the readers and the endpoint, as the CLI's
        # default for several GPU readers: gRPC multiplexes all 8 readers on
        # one connection, whose reader thread loses the sender's L3 when
        # spread over the share's domains (list_read_grpc 6.2k MiB/s with
        # "share" vs 13.5-15.2k with "same", profiles/r2_check_s4b,
        # profiles/r2_cli_geometry)
        sh = affinity.plan(gpu, "same", slot) if use_gpu else {"client": [], "server": []}
        if use_gpu and proto != "http" and args.mux_reader == "isolate":
            sh = affinity.isolate_reader(sh)
        ep = None
        names, list_ms, err = [], 0.0, ""
        try:
            ep = n.Server({"port": 0, "md5": False, "cpus": sh["server"], "retain_uploads": False})
            ep.start()
            ep.add_synthetic(bucket, f"c3_rank{rank}/file_", "", 0, nobj, 1 << 20)
            lister = n.Client({"protocol": proto, "endpoint": ep.url, "retry_initial_s": 0.05})
            t0 = time.perf_counter()
            names = [o["name"] for o in lister.list_all(bucket, f"c3_rank{rank}/file_", 1000)]
            list_ms = (time.perf_counter() - t0) * 1e3
            del lister
            if len(names) != nobj:
                err = f"listed {len(names)} of {nobj} objects"
        except Exception as e:  # noqa: BLE001 - reported in the block, collectives still run
            err = f"{type(e).__name__}: {e}"
        per_pass = (nobj + workers - 1) // workers
        lslots, _, lbytes = args.list_ring.partition("x")
        over = {"protocol": proto, "endpoint": ep.url if ep is not None else "", "workers": workers,
                "object_names": names or [f"c3_rank{rank}/file_0"], "cpus": sh["client"], "worker_id_offset": 0,
                "rcvbuf": parse_size(args.list_rcvbuf), "ring_slots": int(lslots), "ring_slot_bytes": parse_size(lbytes),
                "ring_wc": args.list_ring_wc == "on",
                "reader_cpus": sh.get("reader_cpus")}
        # every rank runs the block (and its collectives) whatever happened here
        st = read_block(over, per_pass, per_pass * warmup_passes, f"{proto} list-read")
        if err:
            st["error"] = err
            st["ok_min"] = 0.0
        if ep is not None:
            ep.stop()
        st["list_ms_max"] = gdist.reduce_stats(ctx, list_ms=list_ms)["list_ms_max"]
        return st

    def ceiling_block(head_mib_s_per_rank: float) -> dict:
        """Same-box bounds of the headline, in its placement: one loopback
        TCP stream with no GPU and no framing (sendfile() by a thread on the
        endpoint's CPUs -> recv() into a THP ring by a thread on the client's
        CPUs, core/ceiling.cc), the client core's memcpy rate, and pinned ->
        HBM copies in the sink's pattern (2 MiB hipMemcpyAsync copies from an
        8-slot THP ring over the pool streams, engine.hip copy_ceiling)."""
        err = ""
        r = {"tcp_gbps": 0.0, "tcp_recv_cpu_s_per_gib": 0.0, "tcp_send_cpu_s_per_gib": 0.0, "memcpy_gbps": 0.0,
             "h2d_gbps": 0.0}
        try:
            ring = args.slots * parse_size(args.slot_bytes)
            reads = max(3, min(10, side_steps))
            t = n.loopback_ceiling({"mode": "tcp", "object_bytes": size, "reads": reads, "ring_bytes": ring,
                                    "rcvbuf": parse_size(args.rcvbuf), "recv_cpus": placement["client"],
                                    "send_cpus": placement["server"], "ring_pages": 1})
            m = n.loopback_ceiling({"mode": "memcpy", "object_bytes": size, "reads": reads, "ring_bytes": ring,
                                    "recv_cpus": placement["client"], "ring_pages": 1})
            r.update(tcp_gbps=t["gbps"], tcp_recv_cpu_s_per_gib=t["recv_cpu_s_per_gib"],
                     tcp_send_cpu_s_per_gib=t["send_cpu_s_per_gib"], memcpy_gbps=m["gbps"])
            if use_gpu:
                h = n.copy_ceiling(gpu, "h2d", size, parse_size(args.slot_bytes), args.slots, args.slots, 5)
                r["h2d_gbps"] = h["gbps"]
        except Exception as e:  # noqa: BLE001 - reported in the block, collectives still run
            err = f"{type(e).__name__}: {e}"
        st = gdist.reduce_stats(ctx, ok=0.0 if err else 1.0, **r)
        out = {"ok": st["ok_min"] >= 1.0}
        for k in r:  # the slowest rank's bound (each rank measures its own)
            out[k] = round(st[k + "_min"], 3)
        head_gbps = head_mib_s_per_rank * (1 << 20) / 1e9
        bounds = [b for b in (out["tcp_gbps"], out["h2d_gbps"] if use_gpu else 0.0) if b > 0]
        if bounds:
            out["bound_gbps"] = round(min(bounds), 3)
            out["headline_gbps_per_gpu"] = round(head_gbps, 3)
            out["headline_frac_of_ceiling"] = round(head_gbps / min(bounds), 3)
        out["note"] = ("one loopback TCP stream, no GPU / h2 / gRPC framing, headline placement; "
                       "h2d: pinned THP ring -> HBM, 2 MiB copies")
        if err:
            out["error"] = err[:300]
        return out

    def ref_default_block(proto: str, osz: int = 0, reads: int = 0, sink: str = "discard",
                          warmup: int = 2) -> dict:
        """The reference's only experiment (execute_pb.sh:4,8; main.go:36,
        30,111): -worker 48 readers, each re-reading its own object
        file_<id>, over gRPC with ONE connection (pool 1) or HTTP/1.1
        keep-alive.  sink "discard": io.Discard with the library's host
        CRC32C (reference semantics); "gpu": every read lands in HBM through
        a small per-worker pinned ring (--ref-gpu-ring) with CRC32C on the
        GPU.  Objects are --ref-object-size (ref_default_*) or 100 MiB
        (ref_default_100m_*, the reference's princer_100M_files,
        main.go:52); a rank's 48 workers read file_<rank*48 + w>.  Threads on
        the rank's GPU-local share of L3 domains trimmed to its CPU-quota
        budget (affinity share_quota) for HTTP, one L3 domain for gRPC."""
        workers = args.ref_workers
        osz = osz or parse_size(args.ref_object_size)
        reads = reads or args.ref_reads
        mode = args.ref_grpc_placement if proto != "http" else args.ref_http_placement
        sh = affinity.plan(gpu, mode, slot) if use_gpu else {"client": [], "server": []}
        if use_gpu and proto != "http" and args.mux_reader == "isolate":
            sh = affinity.isolate_reader(sh)
        ep = None
        err = ""
        prefix = "ref_default/file_" if osz == parse_size(args.ref_object_size) else f"ref_default_{osz >> 20}m/file_"
        try:
            ep = n.Server({"port": 0, "md5": False, "cpus": sh["server"], "retain_uploads": False})
            ep.start()
            ep.add_synthetic(bucket, prefix, "", rank * workers, workers, osz)
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
        over = {"protocol": proto, "endpoint": ep.url if ep is not None else "", "workers": workers,
                "object_prefix": prefix, "worker_id_offset": rank * workers, "sink": sink,
                "host_crc": sink == "discard", "cpus": sh["client"], "rcvbuf": 0, "grpc_conn_pool_size": 1,
                "reader_cpus": sh.get("reader_cpus")}
        if sink == "gpu":
            rs, _, rb = args.ref_gpu_ring.partition("x")
            over.update(ring_slots=int(rs), ring_slot_bytes=parse_size(rb), landing="object")
        st = read_block(over, reads, warmup, f"{proto} reference default {osz >> 20} MiB {sink}", endpoint=ep)
        if err:
            st["error"] = err
            st["ok_min"] = 0.0
        if ep is not None:
            ep.stop()
        return st

    def mib_s(st: dict) -> float:
        return st["nbytes_sum"] / max(st["elapsed_max"], 1e-12) / (1 << 20)

    def block_json(st: dict, **extra) -> dict:
        d = {"ok": st["ok_min"] >= 1.0, "mib_s": round(mib_s(st), 2), "p50_ms": round(st["p50_max"], 3),
             "p99_ms": round(st["p99_max"], 3)}
        d.update(extra)
        if st.get("error"):
            d["error"] = st["error"][:300]
        return d

    def baseline_over() -> dict:
        # The baseline gets the headline's submitter core too: its host CRC
        # runs on the worker (gRPC: apart from the connection's reader, as
        # the Go library's caller goroutine is apart from grpc-go's transport
        # reader), so both designs get two physical cores.
        over = {"protocol": protocol, "sink": "discard", "host_crc": True}
        base_cpus = sorted(set(placement.get("client", [])) | set(placement.get("aux", [])))
        if base_cpus:
            over["cpus"] = base_cpus
        return over

    # ---- headline --------------------------------------------------------
    base_before = None
    bracket = args.baseline_bracket == "on" or (args.baseline_bracket == "auto" and world == 1)
    _only = {b.strip() for b in args.blocks.split(",") if b.strip()} - {"all"}
    if args.workload == "read" and use_gpu and bracket and args.baseline == "on" and \
            (not _only or "cpu_baseline" in _only) and side_steps > 0:
        # the reference-semantics read once more BEFORE the headline, so the
        # two baselines bracket it and a drifting host cancels (A/B sessions)
        base_before = read_block(baseline_over(), side_steps, side_warm, f"{protocol} cpu baseline (before)")
    if args.workload == "read":
        # --read-diag samples the headline's threads around every read (one
        # reader: a handful of threads; not the 48-worker blocks)
        diag_avoid = sorted(set(placement.get("client", [])) | set(placement.get("server", []))
                            | set(placement.get("aux", []) or []))
        head = read_block({"read_diag": bool(args.read_diag), "diag_avoid_cpus": diag_avoid}, args.steps, args.warmup,
                          "headline")
        headline_model = (f"{protocol} ReadObject {args.object_size} object, "
                          f"{'one stream per read' if args.slices == 1 else f'{args.slices} ranged streams'}"
                          + (" -> HBM (CRC32C on GPU)" if use_gpu else " -> discard (CPU baseline)"))
    else:
        if not use_gpu:
            print("bench: --workload write needs --sink gpu (uploads are staged from HBM)", file=sys.stderr)
            return 2
        head = write_block(args.steps, args.warmup)
        headline_model = f"{protocol} resumable upload {args.write_size} object from HBM (D2H -> pinned -> upload)"

    # R4: which HIP device each rank used -> distinct GPUs in the job (before
    # the side blocks: the fan-out block may leave the communicator aborted)
    devs = gdist.gather_floats(ctx, [float(ctx.gpu if use_gpu else -1)])
    distinct = sorted({int(d[0]) for d in devs if d[0] >= 0})
    n_gpus = len(distinct) if use_gpu else world

    def build_line() -> dict | None:
        """Rank 0's bench line from the headline and the side blocks run so
        far (None if the headline failed)."""
        if head["ok_min"] < 1.0:
            return None
        value = mib_s(head)
        tmax = head["elapsed_max"]
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "MiB/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(tmax / args.steps * 1000.0, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8",
            "data": "synthetic",
            "config": {
                "model": headline_model,
                "global_batch": world * args.workers,
                "seq_len": size if args.workload == "read" else parse_size(args.write_size),
                "parallelism": f"dp{world}",
                "workload": args.workload,
                "protocol": protocol,
                "object_bytes": size if args.workload == "read" else parse_size(args.write_size),
                "readers_per_gpu": args.workers,
                "sink": args.sink,
                "ring": f"{args.slots}x{args.slot_bytes}",
                "streams_per_read": args.slices if args.workload == "read" else 1,
                "event_wait": args.event_wait,
                "async_submit": bool(args.async_submit),
                "rcvbuf": parse_size(args.rcvbuf),
                "sysctl": tcp_sysctls(),
            },
            "ranks": world,
            "control_plane": ctx.backend + (" (RCCL init failed: fallback)" if ctx.fallback else ""),
            "devices": distinct if use_gpu else "none (cpu rehearsal)",
            "per_gpu_mib_s": round(value / max(1, n_gpus), 2),
            "p50_ms": round(head["p50_max"], 3),
            "p99_ms": round(head["p99_max"], 3),
            "per_rank_mib_s": [round(b / max(e, 1e-12) / (1 << 20), 1)
                               for b, e in zip(head["nbytes_per_rank"], head["elapsed_per_rank"])],
            "endpoint": "loopback synthetic GCS (one per rank)",
            # how the endpoint sends object bodies (profiles/r3_thp_send)
            "endpoint_send": "vmsplice (THP copy of the pattern)",
            # the endpoint sockets' congestion control (GCSB_SRV_CC; the
            # host default is in config.sysctl, profiles/r3_twins/cc)
            "endpoint_congestion_control": os.environ.get("GCSB_SRV_CC") or "cubic",
            "client_congestion_control": args.client_cc or "host default",
            "affinity": aff,
            "placement": {k: placement.get(k) for k in ("client", "server", "aux", "picked_by", "busy")
                          if placement.get(k) is not None},
        }
        def by_node(counts):
            d = {str(i): c for i, c in enumerate(counts[:-1]) if c}
            if counts and counts[-1]:
                d["absent"] = counts[-1]
            return d
        # host-memory placement: the object's page cache (read by the send
        # path) and the pinned ring (written by the receive thread, read
        # by SDMA) should sit on the GPU's NUMA node
        out["numa"] = {"gpu_node": placement.get("numa_node"),
                       "object_pages": by_node(n.pattern_memfd_numa())}
        if head.get("ring_numa"):
            slots = head["ring_numa"]
            total = [sum(c[i] for c in slots) for i in range(len(slots[0]))]
            out["numa"]["ring_pages"] = by_node(total)
            # per slot: the node holding most of its pages (-1 = not resident)
            out["numa"]["ring_slot_nodes"] = [max(range(len(c) - 1), key=lambda i: c[i]) if sum(c[:-1]) else -1
                                              for c in slots]
        if head.get("ring_thp", -1.0) >= 0:
            # share of the pinned ring on transparent huge pages (the receive copy's TLB reach)
            out["numa"]["ring_thp_fraction"] = round(head["ring_thp"], 3)
        if args.workload == "write":
            out["rank0_slowest"] = head.get("slowest", [])
            out["cpu_s_per_gib_by_thread"] = head.get("cpu_s_per_gib_by_thread", {})
        if args.workload == "read":
            # where a read's time goes: request -> first byte (TTFB), -> last
            # byte in host memory (host_landed), -> last byte + CRC in HBM (p50)
            out["ttfb_p50_ms"] = round(head["ttfb_p50_max"], 3)
            out["host_landed_p50_ms"] = round(head["host_p50_max"], 3)
            out["verified_reads"] = int(head["verified_sum"])
            out["rank0_cpu"] = head["cpu"]
            if head.get("slowest_diag"):
                out["rank0_slowest_diag"] = head["slowest_diag"]
            out["rank0_slowest"] = head.get("slowest", [])
            if head.get("slow_hip"):
                out["slow_hip_calls"] = head["slow_hip"]
            if head["cpu"]:
                gib_s = value / max(1, world) / 1024.0
                out["cpus_needed_per_gpu"] = round(head["cpu"]["process_cpu_s_per_gib"] * gib_s, 2)
        base = blocks.get("cpu_baseline")
        if base is not None and base[1]["ok_min"] >= 1.0 and mib_s(base[1]) > 0:
            bst = base[1]
            runs = [bst]
            if base_before is not None and base_before["ok_min"] >= 1.0 and mib_s(base_before) > 0:
                runs = [base_before, bst]
            # pooled over the runs bracketing the headline: all their bytes over all their time
            pooled = sum(r["nbytes_sum"] for r in runs) / max(sum(r["elapsed_max"] for r in runs), 1e-12) / (1 << 20)
            p50 = sorted(r["p50_max"] for r in runs)[len(runs) // 2] if len(runs) == 1 else \
                sum(r["p50_max"] for r in runs) / len(runs)
            out["vs_baseline"] = round(value / pooled, 3)
            out["baseline"] = {"what": "cpu_baseline: same config, reference semantics (discard sink + host CRC32C), "
                                       "same run" + (", run right before and right after the headline, pooled"
                                                     if len(runs) == 2 else ", run right after the headline"),
                               "mib_s": round(pooled, 2), "p50_ms": round(p50, 3),
                               "p50_ratio": round(p50 / max(head["p50_max"], 1e-9), 3)}
            if len(runs) == 2:
                out["baseline"]["mib_s_before"] = round(mib_s(base_before), 2)
                out["baseline"]["mib_s_after"] = round(mib_s(bst), 2)
            flag = receiver_interference(head.get("cpu") or {}, [(r.get("cpu") or {}) for r in runs])
            if flag:
                out["baseline"]["receiver"] = flag
        for key, (_, st, extra) in blocks.items():
            if extra is None:  # already a JSON block (ceiling)
                out[key] = st
                continue
            b = block_json(st, **{k: v for k, v in extra.items() if v is not None})
            if key.startswith(("ref_default_", "list_read_", "compare", "cpu_baseline")) and st.get("cpu"):
                # where the CPU goes: many streams on one connection (gRPC
                # pool 1), or the headline's twins (one stream each)
                b["cpu_s_per_gib_by_thread"] = st["cpu"].get("cpu_s_per_gib_by_name", {})
                b["cpus_busy"] = st["cpu"].get("cpus_busy")
                if st["cpu"].get("h2_reader"):
                    b["h2_reader"] = st["cpu"]["h2_reader"]
                if st["cpu"].get("recv_avg_kib") is not None:
                    b["recv_avg_kib"] = st["cpu"]["recv_avg_kib"]
                if st["cpu"].get("recv_queue"):
                    b["recv_queue"] = st["cpu"]["recv_queue"]
                if st["cpu"].get("endpoint_tcp"):
                    b["endpoint_tcp"] = st["cpu"]["endpoint_tcp"]
                if st["cpu"].get("endpoint_h2"):
                    b["endpoint_h2"] = st["cpu"]["endpoint_h2"]
                if st["cpu"].get("conn_ring"):
                    b["conn_ring"] = st["cpu"]["conn_ring"]
                if key.startswith(("compare", "cpu_baseline", "ref_default_", "list_read_")) and st["cpu"].get("host"):
                    b["host"] = st["cpu"]["host"]
            if key.startswith("ref_default_100m_") and key.endswith("_gpu"):
                # the HBM landing's own bound: pinned -> HBM copy rate
                # (ceiling block), against min(that, the discard twin's rate)
                ceil = out.get("ceiling") or {}
                twin = out.get(key[:-len("_gpu")] + "_discard")
                if ceil.get("h2d_gbps"):
                    b["h2d_bound_mib_s"] = round(ceil["h2d_gbps"] * 1e9 / (1 << 20), 1)
                    bound = min([b["h2d_bound_mib_s"]] + ([twin["mib_s"]] if twin and twin.get("ok") else []))
                    b["frac_of_bound"] = round(b["mib_s"] / max(bound, 1e-9), 3)
            if key.startswith("ref_default_"):
                b["first_read_p50_ms"] = round(st["first_p50_max"], 3)
                b["steady_p99_ms"] = round(st["steady_p99_max"], 3)
                if st.get("cpu", {}).get("cgroup_nr_throttled") is not None:
                    b["cgroup_nr_throttled"] = st["cpu"]["cgroup_nr_throttled"]
            if key == "fanout":
                # mib_s: whole objects landed in every GPU's HBM, job-wide
                b["per_gpu_mib_s"] = round(b["mib_s"] / max(1, world), 2)
                b["crc_verified_ranks"] = int(st["crc_ok_sum"])
            if st.get("slowest"):
                b["rank0_slowest"] = st["slowest"]
            if st.get("slow_hip", {}).get("slow"):
                b["slow_hip_calls"] = st["slow_hip"]
            if st.get("cpu_s_per_gib_by_thread"):
                b["cpu_s_per_gib_by_thread"] = st["cpu_s_per_gib_by_thread"]
            if key.startswith("list_read_"):
                b["list_ms"] = round(st["list_ms_max"], 3)
            if key == "sliced":
                b["host_landed_p50_ms"] = round(st["host_p50_max"], 3)
                b["slice_skew_ms"] = round(st["skew_max"], 3)
                if st.get("cpu"):
                    b["process_cpu_s_per_gib"] = st["cpu"]["process_cpu_s_per_gib"]
                    b["cpus_busy"] = st["cpu"].get("cpus_busy")
                    if "cgroup_nr_throttled" in st["cpu"]:
                        b["cgroup_nr_throttled"] = st["cpu"]["cgroup_nr_throttled"]
            out[key] = b
        return out

    def stash_headline() -> None:
        """The headline line, complete but for the later side blocks, kept
        for the fatal paths: a side block that hangs (barrier watchdog,
        side-block deadline, SIGTERM from the launcher) prints it before the
        process ends, so a measured headline is never lost."""
        if rank == 0:
            out = build_line()
            if out is not None:
                out["partial"] = "side blocks after cpu_baseline did not finish"
                report.stash(json.dumps(out))
        report.arm(args.side_deadline)

    # ---- side blocks (after the timed region) ----------------------------
    other = {"grpc": "http", "http": "grpc"}.get(protocol)
    blocks = {}
    only = {b.strip() for b in args.blocks.split(",") if b.strip()}
    if not only and world > 1:
        # N > 1: the blocks the scaling run needs; the rest only when asked
        # for (--blocks all or a list), so the first 8-GPU run does not hinge
        # on the least-tested blocks
        only = set(SCALE_BLOCKS)
    if "all" in only:
        only = set()

    def want(name: str) -> bool:
        ok = not only or name in only
        if ok:
            maybe_hang(name, rank)
        return ok
    if side_steps > 0 and args.workload == "read":
        if use_gpu and args.baseline == "on" and want("cpu_baseline"):
            # right after the headline (the boxes drift over a run): the
            # reference's semantics on the headline config -- same endpoint,
            # placement, object and steps; bytes to a discard sink, CRC32C of
            # every byte on the host (the Go library's reader,
            # /root/reference/main.go:133-146).  vs_baseline divides by it.
            for p in [protocol] + ([other] if other and other in hbm.available_protocols() else []):
                key = "cpu_baseline" if p == protocol else f"cpu_baseline_{p}"
                over = {**baseline_over(), "protocol": p}
                blocks[key] = (key, read_block(over, side_steps, side_warm, f"{p} cpu baseline"),
                               {"protocol": p, "sink": "discard", "host_crc": True,
                                "note": "reference semantics: io.Discard + host CRC32C; client + submitter cores"})
        stash_headline()
        if other and other in hbm.available_protocols() and want("compare"):
            blocks["compare"] = ("compare", read_block({"protocol": other}, side_steps, side_warm, f"{other} compare"),
                                 {"protocol": other})
        if base_before is not None:
            blocks["cpu_baseline_before"] = ("cpu_baseline_before", base_before,
                                             {"protocol": protocol, "sink": "discard", "host_crc": True,
                                              "note": "the cpu_baseline block, run before the headline"})
        if args.sliced_streams > 1 and args.slices == 1 and want("sliced"):
            # 8 receive + 8 send threads: a share-placed endpoint of its own
            srv_sl, sh = share_endpoint()
            sliced_cfg.update({"endpoint": srv_sl.url, "cpus": sh["client"]})
            st_sl = read_block(sliced_cfg, side_steps, side_warm, "sliced")
            srv_sl.stop()
            blocks["sliced"] = ("sliced", st_sl,
                                {"streams_per_read": args.sliced_streams,
                                 "ring": f"{args.sliced_slots}x{args.sliced_slot_bytes}", "affinity": "share",
                                 "piece_bytes": parse_size(args.piece_bytes), "note": "extension, not parity"})
        if args.ceiling == "on" and want("ceiling"):
            blocks["ceiling"] = ("ceiling", ceiling_block(mib_s(head) / max(1, world)), None)
        if args.ref_workers > 0 and want("ref_default"):
            for p in ["http"] + ([x for x in ("grpc",) if x in hbm.available_protocols()]):
                blocks[f"ref_default_{p}"] = (f"ref_default_{p}", ref_default_block(p),
                                              {"protocol": p, "workers": args.ref_workers,
                                               "object_bytes": parse_size(args.ref_object_size),
                                               "reads_per_worker": args.ref_reads, "sink": "discard",
                                               "grpc_conn_pool_size": 1 if p == "grpc" else None,
                                               "note": "reference default experiment (execute_pb.sh)"})
        if args.ref_workers > 0 and args.ref100_reads > 0 and want("ref_default_100m"):
            # the reference's real operating point: 48 workers x 100 MiB
            # (princer_100M_files, main.go:36,52), both transports, into the
            # discard sink (reference semantics) and into HBM; the GPU
            # blocks are bounded by the pinned -> HBM copy rate (h2d_gbps)
            for p in ["http"] + ([x for x in ("grpc",) if x in hbm.available_protocols()]):
                for sk in ["discard"] + (["gpu"] if use_gpu else []):
                    key = f"ref_default_100m_{p}_{sk}"
                    blocks[key] = (key, ref_default_block(p, 100 << 20, args.ref100_reads, sk, warmup=1),
                                   {"protocol": p, "workers": args.ref_workers, "object_bytes": 100 << 20,
                                    "reads_per_worker": args.ref100_reads, "sink": sk,
                                    "grpc_conn_pool_size": 1 if p == "grpc" else None,
                                    "ring": args.ref_gpu_ring if sk == "gpu" else None,
                                    "note": "reference default experiment at its object size (princer_100M_files)"})
        if "http" in hbm.available_protocols() and want("c1_http_cpu"):
            # config 1: one 1 MiB object over the HTTP JSON API, CPU only
            # (discard sink, host CRC32C as the Go library), one reader
            srv.add_synthetic(bucket, "c1/file_", "", first, 1, 1 << 20)
            blocks["c1_http_cpu"] = ("c1_http_cpu",
                                     read_block({"protocol": "http", "http_api": "json", "sink": "discard",
                                                 "host_crc": True, "object_prefix": "c1/file_", "workers": 1,
                                                 "rcvbuf": 0}, max(side_steps, 100), side_warm, "config 1"),
                                     {"protocol": "http", "api": "json", "object_bytes": 1 << 20, "sink": "discard",
                                      "workers": 1, "config": "BASELINE config 1"})
        if args.list_objects > 0 and want("list_read"):
            for p in [protocol] + ([other] if other and other in hbm.available_protocols() else []):
                blocks[f"list_read_{p}"] = (f"list_read_{p}", list_read_block(p, 1),
                                            {"protocol": p, "objects": args.list_objects, "object_bytes": 1 << 20,
                                             "workers": args.list_workers, "ring": args.list_ring,
                                             "config": "BASELINE config 3"})
        if use_gpu and want("write"):
            blocks["write"] = ("write", write_block(side_steps, side_warm),
                               {"protocol": protocol, "object_bytes": parse_size(args.write_size),
                                "config": "BASELINE config 5"})
        if use_gpu:
            if args.write_parts > 1 and want("write_composite"):
                blocks["write_composite"] = ("write_composite", write_block(side_steps, side_warm, args.write_parts),
                                             {"protocol": protocol, "object_bytes": parse_size(args.write_size),
                                              "parts": args.write_parts,
                                              "note": "extension: parallel composite upload, not parity"})
        if world > 1 and args.fanout == "on" and want("fanout"):
            blocks["fanout"] = ("fanout", fanout_block(side_steps, side_warm),
                                {"object_bytes": size, "slice_bytes": size // world,
                                 "collective": f"{ctx.backend} all_gather_into_tensor" if ctx.device.type == "cuda"
                                 else f"{ctx.backend} all_gather via host",
                                 "note": "extension: read once per node, fan out over xGMI"})
    # (a write headline runs no side blocks)
    report.disarm()
    srv.stop()

    rc = 0
    if rank == 0:
        out = build_line()
        if out is None:
            print(f"benchmark failed: {head['error'] or 'a rank failed'}", file=sys.stderr)
            rc = 1
        else:
            line = json.dumps(out)
            report.final(line)
            if args.json_out:
                with open(args.json_out, "w") as f:
                    f.write(line + "\n")
    elif head["ok_min"] < 1.0:
        rc = 1
    gdist.shutdown(ctx)
    return rc


def main() -> int:
    args = build_parser().parse_args()
    if args.gpus < 1:
        print("bench: --gpus must be >= 1", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    return run_rank(args)


if __name__ == "__main__":
    sys.exit(main())
