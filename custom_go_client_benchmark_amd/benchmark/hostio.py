"""Host-side plumbing of a bench rank: the stdout stash that holds the
driver's one JSON line, the hang injection for tests, size parsing, and the
CPU / vmstat meters that bracket a timed region (split out of rank.py)."""
from __future__ import annotations

import os
import sys
import threading
import time

class Stash:
    """Rank 0's output line.  The normal path prints ONE line at the end.
    As soon as the headline is measured its line is printed to stderr (a
    human watching sees it) and stashed: if a later side block hangs, the
    fatal paths -- the barrier watchdog (parallel/dist.py on_fatal), the
    side-block deadline, SIGTERM from the rank launcher -- print the stash on
    stdout before the process ends, with a non-zero exit status."""

    def __init__(self):
        self._lock = threading.Lock()
        self._line = None
        self._printed = False
        self._timer = None
        self._out = None

    def claim_stdout(self) -> None:
        """Keep stdout for the ONE JSON line: the process's fd 1 is pointed
        at stderr, so what native libraries print there (RCCL's version
        banner at communicator init, runtime notices) cannot land in front of
        the line the driver parses; the line goes to a private copy of the
        original stdout."""
        if self._out is not None:
            return
        sys.stdout.flush()
        self._out = os.fdopen(os.dup(1), "w", buffering=1)
        os.dup2(2, 1)

    def _print(self, line: str) -> None:
        out = self._out or sys.stdout
        print(line, file=out, flush=True)

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
        self._print(line)

    def final(self, line: str) -> None:
        with self._lock:
            if self._printed:  # a fatal path already printed the stash
                return
            self._printed = True
        self._print(line)

    def arm(self, seconds: float) -> None:
        """Side blocks must be done within `seconds` (0 = no limit)."""
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


stash = Stash()


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


def vmstat() -> dict:
    out = {}
    try:
        with open("/proc/vmstat") as f:
            for line in f:
                k, _, v = line.partition(" ")
                if k in VMSTAT_KEYS:
                    out[k] = int(v)
    except OSError:
        pass
    return out


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
    snap.update({"vm_" + k: v for k, v in vmstat().items()})
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, _, v = line.partition(" ")
                if k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec"):
                    snap[k] = int(v)
    except OSError:
        pass
    return snap


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


def tcp_sysctls() -> dict:
    """Socket-buffer limits of the box: an explicit SO_RCVBUF is capped at
    net.core.rmem_max (and doubled by the kernel)."""
    out = {}
    for k, path in (("rmem_max", "/proc/sys/net/core/rmem_max"), ("tcp_rmem", "/proc/sys/net/ipv4/tcp_rmem"),
                    ("wmem_max", "/proc/sys/net/core/wmem_max"), ("tcp_wmem", "/proc/sys/net/ipv4/tcp_wmem")):
        try:
            with open(path) as f:
                v = [int(x) for x in f.read().split()]
                out[k] = v[0] if len(v) == 1 else v
        except (OSError, ValueError):
            pass
    try:
        with open("/proc/sys/net/ipv4/tcp_congestion_control") as f:
            out["tcp_congestion_control"] = f.read().strip()
    except OSError:
        pass
    return out


class Meter:
    """Process CPU, per-thread-name CPU and vmstat over one or more timed
    segments of one block.  begin()/end() bracket exactly the timed region:
    host-view snapshots (sysdiag.Window) are taken outside them, so their
    parsing of /proc tables is not charged to the block's python3 threads."""

    def __init__(self):
        self.proc: dict = {}
        self.threads: dict[str, float] = {}
        self.elapsed = 0.0
        self.last: dict[str, float] = {}
        self._c0 = self._t0 = None

    def begin(self) -> None:
        from ..utils import cpuacct

        self._c0, self._t0 = cpu_snapshot(), cpuacct.thread_cpu()

    def end(self, elapsed: float) -> None:
        from ..utils import cpuacct

        t1, c1 = cpuacct.thread_cpu(), cpu_snapshot()
        self.last = cpuacct.delta_by_name(self._t0, t1)  # this segment alone
        for k, v in self.last.items():
            self.threads[k] = self.threads.get(k, 0.0) + v
        for k, v in c1.items():
            if isinstance(v, (int, float)) and k in self._c0:
                self.proc[k] = self.proc.get(k, 0) + (v - self._c0[k])
        self.elapsed += elapsed

    def delta(self, nbytes: float) -> dict:
        zero = {k: 0 for k in self.proc}
        return cpu_delta(zero, self.proc, nbytes, self.elapsed) if self.proc else {}
