"""GPU-local CPU placement for the transport threads of one rank.

MI355X nodes (measured on the GPU box, see csrc/core/affinity.h): 2 sockets x
64 cores (SMT2), 16 L3 domains of 8 cores, 4 GPUs per NUMA node.  One rank
(= one GPU) gets two of its NUMA node's L3 domains: one for the client's
receive/worker threads (which also first-touch the pinned ring, so it is
NUMA-local to the GPU's PCIe root), one for the node-local endpoint's send
threads.  Nothing here is needed for correctness; it removes the ~1.5x
run-to-run swing of a single loopback stream and keeps the 8 ranks of a node
off each other's cores.
"""
from __future__ import annotations

import glob
import os

from .. import _native


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _gpu_local(device: int) -> tuple[list[int], bool]:
    """(CPUs of the GPU's NUMA node within our affinity, True) or, when that
    is unknown or empty, (every CPU we may use, False)."""
    allowed = sorted(os.sched_getaffinity(0))
    try:
        bus = _native.gpu_pci_bus_id(device).lower()
    except Exception:
        return allowed, False
    cl = _read(f"/sys/bus/pci/devices/{bus}/local_cpulist")
    if not cl:
        return allowed, False
    local = [c for c in _native.parse_cpulist(cl) if c in set(allowed)]
    return (local, True) if local else (allowed, False)


def gpu_local_cpus(device: int) -> list[int]:
    """CPUs of the GPU's NUMA node (intersected with our affinity)."""
    return _gpu_local(device)[0]


def gpu_numa_node(device: int) -> int:
    try:
        bus = _native.gpu_pci_bus_id(device).lower()
    except Exception:
        return -1
    v = _read(f"/sys/bus/pci/devices/{bus}/numa_node")
    return int(v) if v and v.lstrip("-").isdigit() else -1


def l3_groups(cpus: list[int]) -> list[list[int]]:
    """Partition cpus by shared L3 (in first-cpu order)."""
    groups: dict[str, list[int]] = {}
    for c in cpus:
        key = _read(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") or "all"
        groups.setdefault(key, []).append(c)
    return sorted(groups.values(), key=lambda g: g[0])


def cpu_quota() -> float:
    """CPUs' worth of the container's CFS quota (cgroup v2 cpu.max), 0 if
    unlimited.  The GPU boxes run under one (16 CPUs per GPU,
    profiles/r1_gpu_box_env.txt)."""
    v = _read("/sys/fs/cgroup/cpu.max")
    if not v:
        return 0.0
    parts = v.split()
    if len(parts) != 2 or parts[0] == "max":
        return 0.0
    try:
        return float(parts[0]) / float(parts[1])
    except ValueError:
        return 0.0


def core_first(cpus: list[int]) -> list[int]:
    """cpus reordered so one hardware thread of every physical core comes
    before any SMT sibling (a receive thread gets a core to itself first)."""
    seen, first, rest = set(), [], []
    for c in cpus:
        core = (_read(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id"),
                _read(f"/sys/devices/system/cpu/cpu{c}/topology/core_id"))
        if core[1] is None or core not in seen:
            seen.add(core)
            first.append(c)
        else:
            rest.append(c)
    return first + rest


def _same_core(a: int, b: int) -> bool:
    def key(c):
        return (_read(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id"),
                _read(f"/sys/devices/system/cpu/cpu{c}/topology/core_id"))
    ka = key(a)
    return ka[1] is not None and ka == key(b)


def cpu_busy(sample_s: float = 0.15) -> dict[int, float]:
    """Busy fraction of every host CPU over `sample_s` (/proc/stat is host-wide
    inside the container).  The GPU boxes are slices of shared hosts: a
    receive thread on a core whose SMT sibling runs someone else's work moves
    bytes ~2x slower (profiles/r2_cores: identical single-stream reads at
    0.066 vs 0.148 CPU-s/GiB on the same box)."""
    import time

    def snap():
        out = {}
        try:
            with open("/proc/stat") as f:
                for line in f:
                    if line.startswith("cpu") and line[3:4].isdigit():
                        p = line.split()
                        v = [int(x) for x in p[1:]]
                        out[int(p[0][3:])] = (sum(v), v[3] + (v[4] if len(v) > 4 else 0))
        except OSError:
            pass
        return out

    a = snap()
    if not a:
        return {}
    time.sleep(sample_s)
    b = snap()
    return {c: 1.0 - (b[c][1] - a[c][1]) / max(1, b[c][0] - a[c][0]) for c in b if c in a}


def _core_key(c: int):
    return (_read(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id"),
            _read(f"/sys/devices/system/cpu/cpu{c}/topology/core_id"))


def quiet_cores(cpus: list[int], busy: dict[int, float]) -> list[list[int]]:
    """Physical cores of `cpus` (each as [cpu, siblings...]) ordered from the
    least to the most busy (both hardware threads counted).  The core of CPU 0
    goes last: it carries the host's housekeeping (timers, IRQ defaults)."""
    cores: dict = {}
    for c in cpus:
        cores.setdefault(_core_key(c), []).append(c)
    def load(core):
        pen = 1.0 if 0 in core else 0.0
        return (pen + sum(busy.get(c, 0.0) for c in core), core[0])
    return [sorted(v) for v in sorted(cores.values(), key=load)]


def quota_budget() -> int:
    """CPUs one rank may keep busy without the container being throttled:
    the CFS quota split over the node's ranks (LOCAL_WORLD_SIZE), 0 = no
    limit.  Running more threads than this at once buys no throughput -- the
    quota caps it -- but every quota-exhausted period stalls all threads for
    the rest of the period: tens of ms of p99 (profiles/r2_streams_ab/w48.txt:
    48 HTTP workers unpinned, 3 of 3 periods throttled, p99 36-46 ms)."""
    q = cpu_quota()
    if q <= 0:
        return 0
    ranks = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
    return max(2, int(q // ranks))


def trim_to_quota(cpus: list[int], busy: dict[int, float] | None = None) -> list[int]:
    """cpus cut to the quota budget, one hardware thread per physical core
    first.  With `busy` (cpu_busy), the least busy cores are kept: on a
    shared host another tenant's work on a kept core, or on its SMT sibling,
    slows every thread scheduled there."""
    b = quota_budget()
    if b <= 0 or len(cpus) <= b:
        return cpus
    if busy:
        cores = quiet_cores(cpus, busy)
        order = [c[0] for c in cores] + [t for c in cores for t in c[1:]]
        return sorted(order[:b])
    return sorted(core_first(cpus)[:b])


def _quiet_sampling() -> bool:
    return os.environ.get("GCSB_QUIET_CORES", "1") != "0"


def plan(device: int, mode: str = "split", slot: int = 0) -> dict:
    """CPU sets for this rank: {"client": [...], "server": [...]}.

    slot: ranks sharing one GPU (GCSB_DIST_BACKEND=gloo rehearsals) pass
    their index so they land on different L3 domains.
    mode: "quota" (no GPU locality: as many cores as the container's CPU
                   quota allows this rank, see quota_budget),
          "pair" (one physical core + SMT sibling for the client's threads,
                  the next core of the same L3 domain for the endpoint's),
          "share" (this rank's fair share of its NUMA node's L3 domains --
                   node L3 domains / GPUs on the node -- shared by client and
                   endpoint threads: all 8 domains on a 1-GPU box, 2 per rank
                   on a full 8-GPU node; best for sliced reads),
          "share_quota" (share, trimmed to the rank's CPU-quota budget),
          "split_quota" (share_quota's cores split by physical core: a
                  quarter for the endpoint's threads, the rest for the
                  client's, so 48 endpoint handlers never queue behind 48
                  client workers for a CPU -- a remote server would not share
                  the client's cores at all),
          "split" (client and endpoint on two L3 domains of the GPU's node),
          "same" (one shared L3 domain), "numa" (whole node), "none".
    """
    if mode == "none":
        return {"client": [], "server": [], "mode": mode}
    if mode == "quota":
        # no GPU locality: the first quota-budget cores this process may use
        mine = trim_to_quota(sorted(os.sched_getaffinity(0)))
        return {"client": mine, "server": mine, "mode": mode, "quota_cpus": quota_budget()}
    cpus, local_ok = _gpu_local(device)
    if mode == "numa":
        return {"client": cpus, "server": cpus, "mode": mode}
    node = gpu_numa_node(device)
    peers = []
    for d in range(_native.gpu_device_count()):
        if gpu_numa_node(d) == node:
            peers.append((_native.gpu_pci_bus_id(d).lower(), d))
    peers.sort()
    k = [d for _, d in peers].index(device) if any(d == device for _, d in peers) else 0
    groups = l3_groups(cpus)
    share = max(1, len(groups) // max(1, len(peers)))
    if not local_ok:
        # no GPU-local CPUs in our cpuset (gpu_local_cpus fell back to all we
        # may use): split those among the node's ranks by local rank instead,
        # so ranks of different NUMA nodes do not pick the same domains
        ranks = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
        k = int(os.environ.get("LOCAL_RANK", "0") or 0) % ranks
        share = max(1, len(groups) // ranks)
    # slot: this rank's index among ranks sharing ONE GPU (shared-GPU
    # rehearsals only; 0 on a node with a GPU per rank) -> the next L3 domains
    base = (k * share + slot) % max(1, len(groups))
    if mode in ("share", "share_quota", "split_quota"):
        # not trimmed to the quota: a handful of busy threads (one stream per
        # read, or 8 sliced streams) did better spread over the share's 64
        # CPUs than packed onto 16 cores (sliced 32-34k vs 40-43k MiB/s,
        # profiles/r2_quota); quota packing pays off with many threads.
        # share_quota: the share trimmed to this rank's quota budget (one
        # hardware thread per physical core first) -- many workers per rank
        # (the reference's 48) without the 8 ranks of a node piling onto the
        # same first cores as plain "quota" would
        mine = [c for g in groups[base:base + share] for c in g] or cpus
        if mode in ("share_quota", "split_quota"):
            mine = trim_to_quota(mine, cpu_busy(0.1) if _quiet_sampling() else None)
        if mode == "split_quota":
            cores: dict = {}
            for c in mine:
                cores.setdefault(_core_key(c), []).append(c)
            cl = [sorted(v) for _, v in sorted(cores.items(), key=lambda kv: min(kv[1]))]
            if len(cl) >= 2:
                nsrv = max(1, len(cl) // 4)
                return {"client": sorted(c for core in cl[nsrv:] for c in core),
                        "server": sorted(c for core in cl[:nsrv] for c in core), "mode": mode, "numa_node": node,
                        "gpu_index_on_node": k, "l3_domains": share}
        return {"client": mine, "server": mine, "mode": mode, "numa_node": node, "gpu_index_on_node": k,
                "l3_domains": share}
    if mode in ("pair", "pair2"):
        # three quiet physical cores of one L3 domain of the rank's share
        # (with their SMT siblings): the client's receive thread, the
        # endpoint's send thread, the device submitter.  The domain and the
        # cores are the least busy ones right now (cpu_busy); one domain keeps
        # the loopback copy in one L3 (profiles/r2_placement)
        doms = groups[base:base + share] if groups else [cpus]
        busy = cpu_busy() if _quiet_sampling() else {}
        if busy:
            best = None
            need = 5 if mode == "pair2" else 3
            for dom in doms:
                q = quiet_cores(dom, busy)
                if len(q) < need:
                    continue
                load = sum(busy.get(c, 0.0) for core in q[:3] for c in core) + (1.0 if 0 in q[0] + q[1] else 0.0)
                if best is None or load < best[0]:
                    best = (load, q)
            if best is not None:
                q = best[1]
                if mode == "pair2":
                    # a second quiet core each for the client and the endpoint
                    # thread: somewhere to go when another tenant's thread
                    # lands on the first (the scheduler moves the busy one)
                    return {"client": sorted(q[0] + q[3]), "server": sorted(q[1] + q[4]), "aux": q[2], "mode": mode,
                            "numa_node": node, "gpu_index_on_node": k, "picked_by": "quiet",
                            "busy": round(best[0], 3)}
                return {"client": q[0], "server": q[1], "aux": q[2], "mode": mode,
                        "numa_node": node, "gpu_index_on_node": k, "picked_by": "quiet",
                        "busy": round(best[0], 3)}
        g = core_first(groups[base] if groups else cpus)
        sib = {c: [d for d in (groups[base] if groups else cpus) if d != c and _same_core(c, d)] for c in g[:2]}
        if len(g) < 2:
            return {"client": g, "server": g, "mode": mode}
        # a third core (when the domain has one) for the per-device submitter
        # thread, so slot hand-offs never run on the receiving core's SMT pair
        aux = [g[2]] + [d for d in (groups[base] if groups else cpus) if d != g[2] and _same_core(g[2], d)] \
            if len(g) > 2 else []
        return {"client": [g[0]] + sib[g[0]], "server": [g[1]] + sib[g[1]], "aux": aux,
                "mode": mode, "numa_node": node, "gpu_index_on_node": k}
    client = groups[base] if groups else cpus
    if mode == "same" and share > 1 and _quiet_sampling():
        # the least busy L3 domain of the share (every thread of the block
        # runs in it: a busy neighbour there costs the whole block)
        busy = cpu_busy(0.1)
        if busy:
            client = min(groups[base:base + share], key=lambda g: (sum(busy.get(c, 0.0) for c in g), g[0]))
    if mode == "same" or share < 2:
        server = client
    else:
        server = groups[(base + 1) % len(groups)]
    return {"client": client, "server": server, "mode": mode, "numa_node": node, "gpu_index_on_node": k}


def isolate_reader(pl: dict, min_cores: int = 3) -> dict:
    """A copy of plan `pl` whose client set gives one physical core to the
    multiplexed connection's reader thread alone: "reader_cpus" is one
    hardware thread of the quietest client core, and "client" (the workers)
    loses that whole core, SMT sibling included.  A gRPC connection carrying
    every worker's stream is bound by its one reader thread's receive copy;
    next to a busy sibling (a worker CRC'ing, or spinning in an event wait)
    that copy runs slower.  Unchanged when the client set has fewer than
    `min_cores` physical cores."""
    client = list(pl.get("client") or [])
    cores = quiet_cores(client, cpu_busy(0.05)) if client else []
    if len(cores) < min_cores:
        return dict(pl)
    core = cores[0]
    out = dict(pl)
    out["reader_cpus"] = [core[0]]
    out["client"] = [c for c in client if c not in core]
    if pl.get("server") == pl.get("client"):  # shared sets: keep the endpoint off the reader's core too
        out["server"] = list(out["client"])
    return out


def isolate_sender(pl: dict, min_cores: int = 4) -> dict:
    """A copy of plan `pl` whose endpoint gets one physical core for its
    gRPC send threads alone ("send_cpus"; ServerConfig::send_cpus): the
    quietest client core other than the reader's, taken out of the client
    and server sets, SMT sibling included.  On one connection the endpoint's
    send thread also runs the loopback receive processing of every byte, so
    it competes with the workers on a shared L3 domain.  Unchanged when the
    client set has fewer than `min_cores` physical cores."""
    client = list(pl.get("client") or [])
    taken = set(pl.get("reader_cpus") or [])
    cores = [c for c in (quiet_cores(client, cpu_busy(0.05)) if client else []) if not taken & set(c)]
    if len(cores) < min_cores - 1:
        return dict(pl)
    core = cores[0]
    out = dict(pl)
    out["send_cpus"] = [core[0]]
    out["client"] = [c for c in client if c not in core]
    out["server"] = [c for c in (pl.get("server") or []) if c not in core] or list(out["client"])
    return out


def visible_gpu_summary() -> list[dict]:
    out = []
    for d in range(_native.gpu_device_count()):
        out.append({"device": d, "bus": _native.gpu_pci_bus_id(d), "numa": gpu_numa_node(d)})
    return out


def list_accelerators() -> list[str]:
    return sorted(os.path.basename(p) for p in glob.glob("/sys/class/drm/card*"))
