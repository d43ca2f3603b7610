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

The K timed reads run in 4 chunks interleaved with chunks of the
reference-semantics baseline and of a never-DMA-read twin (--paired, at every
N: each rank runs the same arm order between barriers; the headline's value
counts only its own chunks): vs_baseline_paired and headline_vs_nodma are the
medians of the per-chunk ratios.

HTTP/2 framing: the reference's grpc-go client advertises no
SETTINGS_MAX_FRAME_SIZE, so its peer sends 16 KiB DATA frames, and its windows
stop at 16 MiB (/root/reference/go.mod:20, main.go:106-117).  The headline
runs 16 MiB frames (--h2-framing large, one frame per 2 MiB message, as in
rounds 2-5) with the reference's 16 MiB windows; the ref_framing side block runs the headline config at the
reference's settings, paired chunk by chunk with its reference-semantics
baseline at the same settings, and so do list_read_grpc_ref and
ref_default_grpc_ref.  The client receives many 16 KiB frames per recvmsg()
(csrc/h2/h2_client.h H2DataCursor).

Output: rank 0 prints ONE JSON line (<= 8 KiB, the driver keys first, side
blocks as scalars: custom_go_client_benchmark_amd/benchmark/report.py); the
verbose per-block diagnostics go to --diag-out (default bench_diag.json).

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
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

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
    ap.add_argument("--grpc-pool", type=int, default=1)
    ap.add_argument("--slices", type=int, default=1,
                    help="streams per object read in the HEADLINE run (1 = the reference's sequential read)")
    ap.add_argument("--sliced-streams", type=int, default=8,
                    help="streams per read in the `sliced` extension block (0 = skip the block)")
    ap.add_argument("--affinity", default="auto",
                    help="CPU placement of client/endpoint threads: auto|pair|share|same|split|numa|none "
                         "(parallel/affinity.py). auto: pair for one stream per read (won 3 of 3 interleaved "
                         "reps, profiles/r2_placement), share for sliced reads; the sliced block always runs "
                         "on its own share-placed endpoint")
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
    ap.add_argument("--ref-workers", type=int, default=48,
                    help="ref_default_* side blocks: the reference's default experiment, -worker 48 on 1 MiB "
                         "objects, gRPC pool 1 vs HTTP keep-alive, discard sink + host CRC (0 = off)")
    ap.add_argument("--ref-reads", type=int, default=50, help="ref_default_*: timed reads per worker")
    ap.add_argument("--ref-object-size", default="1MiB", help="ref_default_*: object size")
    ap.add_argument("--ref100-reads", type=int, default=3,
                    help="ref_default_100m_* blocks: the reference's real operating point, 48 workers x 100 MiB "
                         "objects (princer_100M_files), HTTP vs gRPC pool 1, discard + host CRC vs HBM + GPU CRC; "
                         "timed reads per worker (0 = off)")
    ap.add_argument("--ref100-object-size", default="100MiB",
                    help="ref_default_100m_* / ref_effective_grpc object size (the reference's princer_100M_files; "
                         "smaller only for CPU rehearsals)")
    ap.add_argument("--blocks", default="",
                    help="comma list of side blocks to run (A/B sessions): cpu_baseline, compare, sliced, ceiling, "
                         "ref_default, c1_http_cpu, list_read, write, write_composite, fanout; 'all' = every block; empty = "
                         "all at N = 1, cpu_baseline,compare,write,fanout at N > 1")
    ap.add_argument("--read-diag", action="store_true",
                    help="per-read stall attribution (Runner read_diag): scheduler and softirq deltas of the "
                         "receiving / sending threads around every timed read; the slowest reads carry them and a "
                         "named cause (rank0_slowest_diag). Costs tens of us per read outside its latency")
    ap.add_argument("--side-deadline", type=float, default=300.0,
                    help="seconds the side blocks after the headline + cpu_baseline may take before rank 0 prints "
                         "the headline line measured so far and exits 3 (0 = no limit)")
    ap.add_argument("--paired", default="auto", choices=["auto", "on", "off"],
                    help="interleave the headline's timed reads in --paired-chunks chunks with chunks of the "
                         "reference-semantics baseline and of the never-DMA-read twin (same endpoint, cores, "
                         "object); vs_baseline_paired / headline_vs_nodma = medians of the per-chunk ratios. "
                         "auto: on (at every N; at N > 1 each chunk's arm rate is summed over the ranks)")
    ap.add_argument("--paired-chunks", type=int, default=4)
    ap.add_argument("--paired-rewarm", type=int, default=1,
                    help="untimed reads of each paired arm right before its chunk (outside the barriers): the "
                         "reference reads back to back, so a chunk's first read should not pay for the connection "
                         "and copy engines idling through the other arms (0 = off)")
    ap.add_argument("--h2-framing", default="large", choices=["ref", "large"],
                    help="HTTP/2 receive settings of the gRPC clients: ref = the reference's grpc-go (no "
                         "SETTINGS_MAX_FRAME_SIZE advertised -> 16 KiB DATA frames, 16 MiB stream/connection "
                         "windows); large = 16 MiB frames and 16 MiB windows (one frame per 2 MiB message).  The "
                         "headline keeps large: at 16 KiB frames the synthetic endpoint's one send thread per "
                         "connection is the bound (~12 GB/s copying frame trains, README), so a ref headline would "
                         "measure the endpoint; the ref_framing block pairs the headline config at 16 KiB frames "
                         "with its reference-semantics baseline")
    ap.add_argument("--framing-twin", default="on", choices=["on", "off"],
                    help="side blocks at the OTHER framing: the headline paired chunk by chunk with its "
                         "reference-semantics baseline, list_read_grpc and ref_default_grpc")
    ap.add_argument("--ref-effective", default="on", choices=["on", "off"],
                    help="ref_effective_grpc block: 48 x 100 MiB over one gRPC connection with the reference's "
                         "effective read path (whole <= 2 MiB messages decoded, CRC per message, copied out in "
                         "8 KiB reads: io.Discard.ReadFrom, main.go:140); parity-unpinned twin")
    ap.add_argument("--diag-out", default="bench_diag.json",
                    help="sidecar JSON with every block's verbose diagnostics (\"\" = none)")
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


def main() -> int:
    args = build_parser().parse_args()
    if args.gpus < 1:
        print("bench: --gpus must be >= 1", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    from custom_go_client_benchmark_amd.benchmark.rank import run_rank

    return run_rank(args)


if __name__ == "__main__":
    sys.exit(main())
