"""Per-thread CPU accounting of this process, grouped by thread name.

Loopback reads cost CPU at both ends (the client's receive copy into the
pinned ring and the node-local endpoint's send path run in the same process),
and the GPU boxes run under a CPU quota (profiles/r1_gpu_box_env.txt), so CPU
seconds per GiB -- and WHERE they go -- bound throughput.  The native threads
name themselves (csrc/core/affinity.h name_current_thread):

  gcsb-worker     runner worker (also receives slice 0 of a sliced read)
  gcsb-slice      sliced-read receive threads (slices 1..n-1)
  gcsb-wslice     parallel-composite upload part threads
  gcsb-h2-reader  HTTP/2 connection reader (gRPC receive path)
  gcsb-submit     per-device slot hand-off thread (GpuSinkConfig::async_submit)
  gcsb-srv-*      synthetic endpoint (connection / RPC handler / accept)

Everything else (HIP runtime threads, Python) is grouped by its own name.
"""
from __future__ import annotations

import os

_CLK = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100

GROUPS = (
    ("client", ("gcsb-worker", "gcsb-slice", "gcsb-wslice", "gcsb-h2-reader")),
    ("endpoint", ("gcsb-srv",)),
    ("gpu_submit", ("gcsb-submit",)),
)


def thread_cpu() -> dict[str, float]:
    """{thread name: user+sys CPU seconds} summed over this process's live
    threads (threads that already exited are not included).  From schedstat
    (ns) where the kernel has it: /proc/.../stat counts clock ticks (10 ms),
    too coarse for the paired headline's ~50 ms chunks."""
    out: dict[str, float] = {}
    base = "/proc/self/task"
    try:
        tids = os.listdir(base)
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"{base}/{tid}/stat") as f:
                s = f.read()
        except OSError:
            continue
        # comm is parenthesised and may contain spaces: split after the last ')'
        lp, rp = s.find("("), s.rfind(")")
        if lp < 0 or rp < 0:
            continue
        name = s[lp + 1:rp]
        cpu = None
        try:
            with open(f"{base}/{tid}/schedstat") as f:
                cpu = int(f.read().split()[0]) / 1e9
        except (OSError, ValueError, IndexError):
            cpu = None
        if cpu is None:
            fields = s[rp + 2:].split()
            # fields[0] is state (field 3); utime/stime are fields 14/15
            try:
                cpu = (int(fields[11]) + int(fields[12])) / _CLK
            except (IndexError, ValueError):
                continue
        out[name] = out.get(name, 0.0) + cpu
    return out


def group_of(name: str) -> str:
    for g, prefixes in GROUPS:
        if any(name.startswith(p) for p in prefixes):
            return g
    return "other"


def delta_by_group(before: dict[str, float], after: dict[str, float]) -> dict[str, float]:
    """CPU seconds per group between two thread_cpu() snapshots."""
    out: dict[str, float] = {}
    for name, v in after.items():
        d = v - before.get(name, 0.0)
        if d > 0:
            g = group_of(name)
            out[g] = out.get(g, 0.0) + d
    return out


def delta_by_name(before: dict[str, float], after: dict[str, float]) -> dict[str, float]:
    """CPU seconds per thread name between two thread_cpu() snapshots."""
    return {k: v - before.get(k, 0.0) for k, v in after.items() if v - before.get(k, 0.0) > 0}


def per_gib(groups: dict[str, float], nbytes: float) -> dict[str, float]:
    gib = max(nbytes, 1.0) / (1 << 30)
    return {k: round(v / gib, 4) for k, v in sorted(groups.items())}


def cgroup_cpu_stat() -> dict[str, int]:
    """The container's CFS counters (cgroup v2 cpu.stat): on the GPU boxes the
    benchmark runs under a CPU quota, and a period whose quota is spent stalls
    every thread until the next one -- a latency tail of tens of ms."""
    out: dict[str, int] = {}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, _, v = line.partition(" ")
                if k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec"):
                    out[k] = int(v)
    except OSError:
        pass
    return out


def cgroup_delta(a: dict[str, int], b: dict[str, int]) -> dict[str, float]:
    out: dict[str, float] = {}
    for k in ("nr_periods", "nr_throttled"):
        if k in a and k in b:
            out["cgroup_" + k] = b[k] - a[k]
    if "throttled_usec" in a and "throttled_usec" in b:
        out["cgroup_throttled_ms"] = (b["throttled_usec"] - a["throttled_usec"]) / 1e3
    return out


def process_name() -> str:
    """The process's comm ("python3" under the driver): the name every
    thread nobody renamed carries."""
    try:
        with open(f"/proc/{os.getpid()}/comm") as f:
            return f.read().strip()
    except OSError:
        return "python3"


def label_runtime_threads(label: str = "hip-rt") -> int:
    """Names this process's non-Python helper threads (the HIP / ROCr runtime's
    event and callback threads, torch's pools) `label`, so their CPU shows
    apart from Python's in the by-name tables: they inherit the process name
    ("python3") and so did the round-4 list-read blocks' 0.10 CPU-s/GiB of
    "python3" time.  Python's own threads (threading.enumerate()) and named
    native threads keep their names.  Returns how many were renamed."""
    import threading

    py = {t.native_id for t in threading.enumerate() if t.native_id is not None}
    py.add(os.getpid())
    base = "/proc/self/task"
    proc_name = process_name()
    try:
        tids = os.listdir(base)
    except OSError:
        return 0
    n = 0
    for t in tids:
        tid = int(t)
        if tid in py:
            continue
        try:
            with open(f"{base}/{t}/comm") as f:
                name = f.read().strip()
            if name != proc_name:
                continue
            with open(f"{base}/{t}/comm", "w") as f:
                f.write(label)
            n += 1
        except OSError:
            continue
    return n
