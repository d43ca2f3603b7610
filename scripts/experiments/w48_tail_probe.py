"""48 HTTP workers x 1 MiB (the reference's default, discard + host CRC):
where do the 100-300 ms reads the bench's ref_default_http block shows near
the end of its run come from?  Every read is recorded (worker, seq, start,
TTFB, end); the slow ones are printed with their start time in the run, so a
process- or host-wide stall shows as many workers' reads starting together.
Same endpoint / placement as bench.py (share_quota)."""
import argparse
import json
import re
import threading
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402,F401

import custom_go_client_benchmark_amd as pkg  # noqa: E402
from custom_go_client_benchmark_amd.parallel import affinity  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--protocol", default="http")
ap.add_argument("--workers", type=int, default=48)
ap.add_argument("--reads", type=int, default=50)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--slow-ms", type=float, default=20.0)
ap.add_argument("--warm-reads", type=int, default=2)
ap.add_argument("--isolate-reader", action="store_true", help="affinity.isolate_reader: a core of its own for the h2 reader")
ap.add_argument("--gap-s", type=float, default=0.0, help="sleep between the warm-up and rep 0")
ap.add_argument("--sample-ms", type=float, default=400.0, help="sample thread states for this long per rep (0: off)")
args = ap.parse_args()


def tasks():
    """{tid: (comm, state, run_delay_ns)} of this process's threads."""
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                st = f.read()
            with open(f"/proc/self/task/{tid}/schedstat") as f:
                rd = int(f.read().split()[1])
        except OSError:
            continue
        comm = st[st.index("(") + 1:st.rindex(")")]
        out[tid] = (re.sub(r"[-_]?\d+$", "", comm), st[st.rindex(")") + 2], rd)
    return out


def blocked_in(tid):
    out = []
    for f in ("syscall", "wchan"):
        try:
            with open(f"/proc/self/task/{tid}/{f}") as fh:
                out.append(fh.read().split()[0] if f == "syscall" else fh.read().strip())
        except (OSError, IndexError):
            out.append("?")
    return ":".join(out)


def vmstat():
    keep = ("compact_stall", "compact_fail", "thp_fault_alloc", "thp_fault_fallback", "thp_collapse_alloc",
            "pgmajfault", "allocstall_normal", "allocstall_movable", "pgscan_direct", "pgsteal_kswapd",
            "thp_split_page", "numa_pte_updates", "numa_hint_faults", "pgmigrate_success")
    d = {}
    with open("/proc/vmstat") as f:
        for line in f:
            k, v = line.split()
            if k in keep:
                d[k] = int(v)
    return d


class Sampler(threading.Thread):
    """Every 2 ms for `ms`: how many threads of each name are Running / Sleeping / D (uninterruptible)."""

    def __init__(self, ms):
        super().__init__(daemon=True)
        self.ms, self.timeline = ms, []

    def run(self):
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < self.ms:
            c = {}
            for tid, (comm, state, _) in tasks().items():
                if state != "S":
                    key = f"{comm}:{state}"
                    if state == "D":  # where in the kernel: syscall number and wait channel
                        key += f":sys{blocked_in(tid)}"
                    c[key] = c.get(key, 0) + 1
            self.timeline.append((round((time.perf_counter() - t0) * 1e3, 1), c))
            time.sleep(0.002)

n = pkg._native
sh = affinity.plan(0, "share_quota", 0)
if args.isolate_reader:
    sh = affinity.isolate_reader(sh)
srv = n.Server({"port": 0, "md5": False, "cpus": sh["server"], "retain_uploads": False})
srv.start()
srv.add_synthetic("b", "ref/file_", "", 0, args.workers, 1 << 20)
cfg = {"protocol": args.protocol, "endpoint": srv.url, "bucket": "b", "object_prefix": "ref/file_",
       "workers": args.workers, "reads_per_worker": args.warm_reads, "sink": "discard", "host_crc": True, "cpus": sh["client"],
       "keep_records": True, "grpc_conn_pool_size": 1, "reader_cpus": sh.get("reader_cpus")}
r = n.Runner(cfg)
r.start()
r.wait()
r.drain()
if args.gap_s:
    time.sleep(args.gap_s)
for rep in range(args.reps):
    r.reset_stats()
    r.set_reads_per_worker(args.reads)
    t0 = time.perf_counter_ns()
    rd0, vm0 = tasks(), vmstat()
    smp = Sampler(args.sample_ms) if args.sample_ms else None
    if smp:
        smp.start()
    r.start()
    r.wait()
    rd1, vm1 = tasks(), vmstat()
    delay = {}
    for tid, (comm, _, d1) in rd1.items():
        if tid in rd0:
            delay[comm] = delay.get(comm, 0) + d1 - rd0[tid][2]
    if smp:
        smp.join()
    recs = r.drain()
    s = r.summary()
    base = min(x["start_ns"] for x in recs)
    slow = sorted((x for x in recs if (x["end_ns"] - x["start_ns"]) / 1e6 >= args.slow_ms),
                  key=lambda x: x["start_ns"])
    print(json.dumps({"rep": rep, "reader_cpus": sh.get("reader_cpus"), "mib_s": round(s["mib_per_s"], 1), "p50_ms": round(s["p50_ms"], 3),
                      "p99_ms": round(s["p99_ms"], 3), "max_ms": round(s["max_ms"], 3), "reads": len(recs),
                      "run_ms": round((max(x["end_ns"] for x in recs) - base) / 1e6, 1),
                      "slow": [{"worker": x["worker"], "seq": x["seq"],
                                "start_ms": round((x["start_ns"] - base) / 1e6, 2),
                                "ttfb_ms": round((x["ttfb_ns"] - x["start_ns"]) / 1e6, 2) if x["ttfb_ns"] else None,
                                "ms": round((x["end_ns"] - x["start_ns"]) / 1e6, 2)} for x in slow[:40]],
                      "run_delay_ms_by_name": {k: round(v / 1e6, 1) for k, v in sorted(delay.items()) if v > 1e6},
                      "vmstat": {k: vm1[k] - vm0[k] for k in vm1 if vm1[k] != vm0.get(k)},
                      "states": [t for t in (smp.timeline if smp else []) if t[1]][:200]}),
          flush=True)
srv.stop()
