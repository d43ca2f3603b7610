"""Host-side stall attribution for the timed blocks: what, besides our own
threads' CPU time, took a receiving or sending core away.

A loopback read is bound by one receiving core (the h2 reader) and fed by
one sending core (the endpoint's handler).  When either is descheduled, or
its CPU is busy with interrupts, the stream stalls while our own CPU
counters (cpuacct) show nothing.  Three host views, all readable without
privileges and cheap enough to snapshot around every timed block:

  thread_sched()  per thread of this process: run-queue delay (schedstat),
                  voluntary / involuntary context switches, last CPU;
  irq_snapshot()  /proc/interrupts per CPU and source (GPU completion
                  interrupts, NIC, IPIs, timers);
  softirq_snapshot()  /proc/softirqs per CPU (NET_RX / NET_TX, TIMER, RCU);
  ClockSampler    the placement cores' clock (cpufreq cpuinfo_avg_freq, the
                  APERF/MPERF average of the last tick) every 20 ms: a
                  uniform slowdown of unrelated threads (profiles/r4_final6)
                  is a core clock drop or memory, not a scheduler delay.

Reference timed region: /root/reference/main.go:133-145 (request -> last
byte); these views explain a read's stall inside that region, they add
nothing to it.
"""
from __future__ import annotations

import os
import threading

_TASKS = "/proc/self/task"


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def thread_sched() -> dict[int, dict]:
    """{tid: {name, cpu_ns, run_delay_ns, slices, nvcsw, nivcsw, cpu}} for
    every live thread of this process.  run_delay_ns is the time the thread
    was runnable but waiting for a CPU (schedstat field 2)."""
    out: dict[int, dict] = {}
    try:
        tids = os.listdir(_TASKS)
    except OSError:
        return out
    for t in tids:
        st = _read(f"{_TASKS}/{t}/stat")
        ss = _read(f"{_TASKS}/{t}/schedstat")
        if not st or not ss:
            continue
        lp, rp = st.find("("), st.rfind(")")
        f = st[rp + 2:].split()
        try:
            cpu_ns, delay_ns, slices = (int(x) for x in ss.split()[:3])
            last_cpu = int(f[36])
        except (ValueError, IndexError):
            continue
        d = {"name": st[lp + 1:rp], "cpu_ns": cpu_ns, "run_delay_ns": delay_ns, "slices": slices,
             "cpu": last_cpu, "nvcsw": 0, "nivcsw": 0}
        status = _read(f"{_TASKS}/{t}/status") or ""
        for line in status.splitlines():
            if line.startswith("voluntary_ctxt_switches:"):
                d["nvcsw"] = int(line.split()[1])
            elif line.startswith("nonvoluntary_ctxt_switches:"):
                d["nivcsw"] = int(line.split()[1])
        out[int(t)] = d
    return out


def sched_delta(a: dict[int, dict], b: dict[int, dict], reads: int = 1, top: int = 8) -> dict:
    """Per thread name (threads of one name summed): CPU ms, run-queue delay
    ms and involuntary switches between two thread_sched() snapshots, per
    read; only threads that ran.  Also the CPUs each name last ran on."""
    agg: dict[str, dict] = {}
    for tid, y in b.items():
        x = a.get(tid, {"cpu_ns": 0, "run_delay_ns": 0, "nvcsw": 0, "nivcsw": 0})
        dc = y["cpu_ns"] - x["cpu_ns"]
        if dc <= 0:
            continue
        g = agg.setdefault(y["name"], {"threads": 0, "cpu_ms": 0.0, "run_delay_ms": 0.0, "nvcsw": 0, "nivcsw": 0,
                                       "cpus": set()})
        g["threads"] += 1
        g["cpu_ms"] += dc / 1e6
        g["run_delay_ms"] += (y["run_delay_ns"] - x["run_delay_ns"]) / 1e6
        g["nvcsw"] += y["nvcsw"] - x["nvcsw"]
        g["nivcsw"] += y["nivcsw"] - x["nivcsw"]
        g["cpus"].add(y["cpu"])
    r = max(1, reads)
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["cpu_ms"])[:top]
    return {k: {"threads": v["threads"], "cpu_ms_per_read": round(v["cpu_ms"] / r, 3),
                "run_delay_ms_per_read": round(v["run_delay_ms"] / r, 4),
                "nivcsw_per_read": round(v["nivcsw"] / r, 2), "nvcsw_per_read": round(v["nvcsw"] / r, 2),
                "last_cpus": sorted(v["cpus"])}
            for k, v in rows}


def _per_cpu_table(text: str | None) -> tuple[list[int], dict[str, list[int]]]:
    """(cpu ids of the header, {row label: per-cpu counts}) of a
    /proc/interrupts- or /proc/softirqs-shaped table."""
    if not text:
        return [], {}
    lines = text.splitlines()
    cpus = [int(c[3:]) for c in lines[0].split() if c.startswith("CPU")]
    rows: dict[str, list[int]] = {}
    for line in lines[1:]:
        head, _, rest = line.partition(":")
        parts = rest.split()
        vals = []
        for p in parts[:len(cpus)]:
            if not p.isdigit():
                break
            vals.append(int(p))
        if not vals:
            continue
        desc = " ".join(parts[len(vals):])
        label = head.strip()
        if desc:
            # device-named IRQs: keep the driver / device part of the label
            label = f"{label} {desc.split()[-1]}" if label.isdigit() else label
        rows[label] = vals + [0] * (len(cpus) - len(vals))
    return cpus, rows


def irq_snapshot() -> tuple[list[int], dict[str, list[int]]]:
    return _per_cpu_table(_read("/proc/interrupts"))


def softirq_snapshot() -> tuple[list[int], dict[str, list[int]]]:
    return _per_cpu_table(_read("/proc/softirqs"))


def table_delta(a: tuple, b: tuple, cpus: list[int] | None, reads: int = 1, top: int = 6) -> dict:
    """Counts per read that landed on `cpus` (all CPUs if None) between two
    snapshots: {"total": n, "by_source": {label: n, ...}, "by_cpu": {cpu: n}}."""
    ids, ra = a
    ids_b, rb = b
    if not ids or ids != ids_b:
        return {}
    want = set(cpus) if cpus else set(ids)
    idx = [i for i, c in enumerate(ids) if c in want]
    by_src: dict[str, int] = {}
    by_cpu: dict[int, int] = {}
    for label, vb in rb.items():
        va = ra.get(label, [0] * len(ids))
        for i in idx:
            d = vb[i] - va[i]
            if d > 0:
                by_src[label] = by_src.get(label, 0) + d
                by_cpu[ids[i]] = by_cpu.get(ids[i], 0) + d
    r = max(1, reads)
    tops = sorted(by_src.items(), key=lambda kv: -kv[1])[:top]
    return {"total_per_read": round(sum(by_src.values()) / r, 2),
            "by_source_per_read": {k: round(v / r, 2) for k, v in tops},
            "by_cpu_per_read": {str(c): round(v / r, 2) for c, v in sorted(by_cpu.items())}}


# namespace-wide TCP counters that explain a stalled loopback stream: a
# retransmission timeout (RTO, >= 200 ms), tail-loss probes, and the receive
# queue pruning / dropping that precedes them when skb memory (truesize)
# outgrows the socket's receive buffer
TCP_COUNTERS = {"Tcp": ("RetransSegs",),
                "TcpExt": ("TCPTimeouts", "TCPLossProbes", "PruneCalled", "RcvPruned", "TCPRcvQDrop",
                           "TCPRcvCollapsed", "TCPBacklogDrop", "TCPZeroWindowDrop", "TCPOFODrop",
                           # which retransmits, and why
                           "TCPFastRetrans", "TCPSlowStartRetrans", "TCPLostRetransmit", "TCPRetransFail",
                           "TCPSpuriousRtxHostQueues", "TCPSACKReorder", "TCPTSReorder", "TCPRenoReorder",
                           "TCPDSACKRecv", "TCPDSACKOldSent", "TCPSpuriousRTOs", "TCPWinProbe")}


def tcp_snapshot() -> dict[str, int]:
    out: dict[str, int] = {}
    for path in ("/proc/net/snmp", "/proc/net/netstat"):
        text = _read(path)
        if not text:
            continue
        lines = text.splitlines()
        for names, vals in zip(lines[::2], lines[1::2]):
            proto, _, hdr = names.partition(":")
            want = TCP_COUNTERS.get(proto)
            if not want:
                continue
            for k, v in zip(hdr.split(), vals.partition(":")[2].split()):
                if k in want and v.lstrip("-").isdigit():
                    out[k] = int(v)
    return out


def softnet_snapshot() -> dict[int, tuple[int, int]]:
    """{cpu: (dropped, time_squeeze)} from /proc/net/softnet_stat: packets
    the CPU's input backlog dropped (loopback traffic is queued there by the
    sender), and NET_RX rounds that ran out of budget."""
    out: dict[int, tuple[int, int]] = {}
    text = _read("/proc/net/softnet_stat") or ""
    for i, line in enumerate(text.splitlines()):
        f = line.split()
        if len(f) < 3:
            continue
        cpu = int(f[12], 16) if len(f) > 12 else i
        out[cpu] = (int(f[1], 16), int(f[2], 16))
    return out


def softnet_delta(a: dict, b: dict, cpus: list[int] | None) -> dict[str, int]:
    want = set(cpus) if cpus else set(b)
    drop = sum(b[c][0] - a.get(c, (0, 0))[0] for c in b if c in want)
    sq = sum(b[c][1] - a.get(c, (0, 0))[1] for c in b if c in want)
    return {"dropped": drop, "time_squeeze": sq}


def tcp_delta(a: dict[str, int], b: dict[str, int]) -> dict[str, int]:
    """Non-zero counter increases between two tcp_snapshot()s."""
    return {k: b[k] - a.get(k, 0) for k in b if b[k] - a.get(k, 0) > 0}


def attribute(diag: dict, ms: float, p50_ms: float) -> str:
    """A slow read's likely cause from its scheduler / softirq deltas
    (Runner read_diag, core/sched_probe.h): run-queue delay of the receiving
    thread (h2 reader, or the HTTP worker) or of the endpoint's sender,
    preemptions, TCP retransmits, a timer-softirq storm on their CPUs, or --
    none of those --
    a receive copy that simply took longer on the CPU."""
    th = diag.get("threads", {})
    excess = max(ms - p50_ms, 1e-6)
    recv = th.get("gcsb-h2-reader") or th.get("gcsb-worker") or {}
    send = {"cpu_ms": 0.0, "run_delay_ms": 0.0, "nivcsw": 0}
    for k, v in th.items():
        if k.startswith("gcsb-srv"):
            for f in send:
                send[f] += v.get(f, 0)
    causes = []
    for label, row in (("receiving thread", recv), ("endpoint sender", send)):
        if row and row.get("run_delay_ms", 0.0) >= 0.2 * excess:
            causes.append(f"{label} waited {row['run_delay_ms']:.2f} ms for a CPU "
                          f"({row.get('nivcsw', 0)} preemptions)")
    tcp = diag.get("tcp", {})
    if tcp.get("TCPTimeouts", 0) or tcp.get("RetransSegs", 0) > tcp.get("TCPLossProbes", 0):
        causes.append(f"{tcp.get('RetransSegs', 0)} TCP retransmits ({tcp.get('TCPTimeouts', 0)} RTOs, "
                      f"{tcp.get('TCPLossProbes', 0)} loss probes) in the namespace")
    dropped = tcp.get("RcvPruned", 0) + tcp.get("TCPRcvQDrop", 0) + tcp.get("TCPBacklogDrop", 0)
    if dropped:
        causes.append(f"{dropped} receive-queue prunes / drops (skb memory over the receive buffer)")
    sn = diag.get("softnet", {})
    if sn.get("dropped", 0):
        causes.append(f"{sn['dropped']} packets dropped at a CPU's input backlog (softnet; loopback packets "
                      f"wait there for NET_RX)")
    soft = diag.get("softirqs", {})
    if soft.get("HRTIMER", 0) >= 100:
        causes.append(f"{soft['HRTIMER']} HRTIMER softirqs on the busy CPUs (pacing timers)")
    if not causes and recv:
        busy = recv.get("cpu_ms", 0.0) / max(diag.get("wall_ms", ms), 1e-6)
        if busy >= 0.9:
            causes.append(f"receiving thread on-CPU {recv['cpu_ms']:.2f} of {ms:.2f} ms: the receive copy itself "
                          f"ran slower (no scheduler delay, no timer storm)")
        else:
            causes.append(f"receiving thread idle {ms - recv.get('cpu_ms', 0.0):.2f} ms without run-queue delay: "
                          f"waiting for data (sender {send['cpu_ms']:.2f} ms on CPU)")
    return "; ".join(causes) or "no cause found"


def _freq_file(cpu: int) -> str | None:
    base = f"/sys/devices/system/cpu/cpu{cpu}/cpufreq/"
    for name in ("cpuinfo_avg_freq", "scaling_cur_freq"):
        if os.path.exists(base + name):
            return base + name
    return None


class ClockSampler:
    """Samples the given CPUs' clock (kHz from cpufreq) every `period_s` on a
    daemon thread until .stop(); .report() gives MHz per CPU (mean, min, max
    over the samples).  No cpufreq (VMs, this build container): no thread,
    an empty report.  One small sysfs read per CPU per sample, off the
    placement's CPUs (the thread inherits the main thread's affinity)."""

    def __init__(self, cpus: list[int] | None, period_s: float = 0.02):
        self.files = {c: f for c in (cpus or []) for f in [_freq_file(c)] if f}
        self.samples: dict[int, list[int]] = {c: [] for c in self.files}
        self.period = period_s
        self._halt = threading.Event()
        self._thread = None
        if self.files:
            self._thread = threading.Thread(target=self._run, name="gcsb-clock", daemon=True)
            self._thread.start()

    def _sample(self) -> None:
        for c, path in self.files.items():
            v = _read(path)
            if v and v.strip().isdigit():
                self.samples[c].append(int(v))

    def _run(self) -> None:
        while not self._halt.wait(self.period):
            self._sample()

    def stop(self) -> None:
        self._halt.set()
        if self._thread is not None:
            self._thread.join(timeout=1.0)
            self._thread = None

    def report(self) -> dict[str, dict]:
        self.stop()
        out = {}
        for c, v in sorted(self.samples.items()):
            if v:
                out[str(c)] = {"mean": round(sum(v) / len(v) / 1000.0), "min": round(min(v) / 1000.0),
                               "max": round(max(v) / 1000.0), "n": len(v)}
        return out


class Window:
    """Snapshot everything at construction; .report(cpus, reads) after the
    timed region.  With `clock_cpus`, those CPUs' clock is sampled through
    the window (ClockSampler)."""

    def __init__(self, clock_cpus: list[int] | None = None):
        self.sched = thread_sched()
        self.irq = irq_snapshot()
        self.soft = softirq_snapshot()
        self.tcp = tcp_snapshot()
        self.softnet = softnet_snapshot()
        self.clock = ClockSampler(clock_cpus) if clock_cpus else None

    def report(self, cpus: list[int] | None, reads: int) -> dict:
        out = {"threads": sched_delta(self.sched, thread_sched(), reads),
               "irq_on_placement": table_delta(self.irq, irq_snapshot(), cpus, reads),
               "softirq_on_placement": table_delta(self.soft, softirq_snapshot(), cpus, reads),
               # whole block, not per read: any RTO / drop names a stalled read
               "tcp": tcp_delta(self.tcp, tcp_snapshot()),
               "softnet_on_placement": softnet_delta(self.softnet, softnet_snapshot(), cpus)}
        if self.clock is not None:
            mhz = self.clock.report()
            if mhz:
                out["clock_mhz_on_placement"] = mhz
        return out
