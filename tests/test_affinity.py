"""CPU placement planner (parallel/affinity.py) on the host topology."""
import os

import pytest


@pytest.fixture()
def aff(native):
    from custom_go_client_benchmark_amd.parallel import affinity

    return affinity


def test_none_mode_pins_nothing(aff):
    p = aff.plan(0, "none")
    assert p["client"] == [] and p["server"] == []


@pytest.mark.parametrize("mode", ["share", "same", "split", "numa"])
def test_modes_stay_inside_allowed_cpus(aff, mode):
    allowed = set(os.sched_getaffinity(0))
    p = aff.plan(0, mode)
    assert p["client"] and p["server"]
    assert set(p["client"]) <= allowed and set(p["server"]) <= allowed
    if mode in ("share", "same", "numa"):
        assert p["client"] == p["server"]


def test_share_is_union_of_whole_l3_domains(aff):
    cpus = aff.gpu_local_cpus(0)
    groups = aff.l3_groups(cpus)
    p = aff.plan(0, "share")
    got = set(p["client"])
    for g in groups:
        assert set(g) <= got or not (set(g) & got)  # whole domains only


def test_split_uses_disjoint_domains_when_available(aff):
    groups = aff.l3_groups(aff.gpu_local_cpus(0))
    p = aff.plan(0, "split")
    if len(groups) >= 2:
        assert not set(p["client"]) & set(p["server"])
    else:
        assert p["client"] == p["server"]


def test_l3_groups_partition(aff):
    cpus = aff.gpu_local_cpus(0)
    groups = aff.l3_groups(cpus)
    flat = [c for g in groups for c in g]
    assert sorted(flat) == sorted(cpus)


def test_cpu_quota_and_trim(monkeypatch):
    from custom_go_client_benchmark_amd.parallel import affinity as a

    files = {"/sys/fs/cgroup/cpu.max": "1600000 100000"}
    # 4 cores x 2 SMT threads: cpu c and c+4 are siblings
    for c in range(8):
        files[f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id"] = "0"
        files[f"/sys/devices/system/cpu/cpu{c}/topology/core_id"] = str(c % 4)
    monkeypatch.setattr(a, "_read", lambda p: files.get(p))
    assert a.cpu_quota() == 16.0
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert a.quota_budget() == 2
    assert a.core_first([0, 4, 1, 5, 2, 6, 3, 7]) == [0, 1, 2, 3, 4, 5, 6, 7]
    assert a.trim_to_quota([0, 4, 1, 5, 2, 6, 3, 7]) == [0, 1]
    # with a busy map: the two quietest cores (core 1's sibling busy, CPU 0's core last)
    busy = {c: 0.0 for c in range(8)}
    busy[5] = 0.9
    assert a.trim_to_quota(list(range(8)), busy) == [2, 3]
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    assert a.trim_to_quota(list(range(8))) == list(range(8))  # 16-CPU budget > 8 CPUs
    files["/sys/fs/cgroup/cpu.max"] = "max 100000"
    assert a.cpu_quota() == 0.0 and a.quota_budget() == 0


def _fake_topology(monkeypatch, a, ncpu=16, per_l3=8):
    """ncpu CPUs: SMT siblings c and c + ncpu/2, L3 domains of per_l3 CPUs
    (both siblings of a core in the same domain)."""
    half = ncpu // 2
    files = {}
    for c in range(ncpu):
        core = c % half
        files[f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id"] = "0"
        files[f"/sys/devices/system/cpu/cpu{c}/topology/core_id"] = str(core)
        dom = core // (per_l3 // 2)
        lo = dom * (per_l3 // 2)
        files[f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list"] = \
            f"{lo}-{lo + per_l3 // 2 - 1},{lo + half}-{lo + half + per_l3 // 2 - 1}"
    monkeypatch.setattr(a, "_read", lambda p: files.get(p))
    monkeypatch.setattr(a.os, "sched_getaffinity", lambda pid: set(range(ncpu)))


def test_quiet_cores_order_and_cpu0_last(monkeypatch):
    from custom_go_client_benchmark_amd.parallel import affinity as a

    _fake_topology(monkeypatch, a)
    busy = {c: 0.0 for c in range(16)}
    busy[1] = 0.9   # core 1 busy on its first thread
    busy[10] = 0.5  # core 2 busy on its SMT sibling
    q = a.quiet_cores(list(range(8)) + list(range(8, 16)), busy)
    flat = [core[0] for core in q]
    assert flat[-1] == 0            # CPU 0's core goes last (housekeeping)
    assert flat.index(1) > flat.index(3) and flat.index(2) > flat.index(3)
    assert all(len(core) == 2 for core in q)


def test_pair_plan_picks_quiet_disjoint_cores_in_one_domain(monkeypatch):
    from custom_go_client_benchmark_amd.parallel import affinity as a

    _fake_topology(monkeypatch, a)
    busy = {c: 0.0 for c in range(16)}
    for c in (4, 5, 12):  # domain 1 partly busy
        busy[c] = 0.8
    monkeypatch.setattr(a, "cpu_busy", lambda sample_s=0.15: busy)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    monkeypatch.setenv("LOCAL_RANK", "0")
    p = a.plan(0, "pair")
    assert p["picked_by"] == "quiet"
    cl, sv, ax = set(p["client"]), set(p["server"]), set(p["aux"])
    assert not (cl & sv) and not (cl & ax) and not (sv & ax)
    dom0 = {0, 1, 2, 3, 8, 9, 10, 11}
    assert cl | sv | ax <= dom0       # the quiet domain, one L3
    assert 0 not in cl | sv | ax      # CPU 0's core avoided while others are free


def test_plan_without_gpu_locality_splits_by_local_rank(monkeypatch):
    from custom_go_client_benchmark_amd.parallel import affinity as a

    _fake_topology(monkeypatch, a, ncpu=32, per_l3=8)
    monkeypatch.setenv("GCSB_QUIET_CORES", "0")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    seen = []
    for r in range(4):
        monkeypatch.setenv("LOCAL_RANK", str(r))
        seen.append(set(a.plan(0, "share")["client"]))
    for i in range(4):
        for j in range(i + 1, 4):
            assert not (seen[i] & seen[j])  # ranks never share a domain


def test_numa_placement_queries(native):
    """numa_nodes_of / pattern_memfd_numa report where pages live (the bench
    line's `numa` block): touched pages are resident on some node, untouched
    ones are reported absent (last entry)."""
    import numpy as np

    a = np.empty(8 << 20, dtype=np.uint8)
    untouched = native.numa_nodes_of(a.ctypes.data, a.nbytes)
    a[:] = 1
    touched = native.numa_nodes_of(a.ctypes.data, a.nbytes)
    assert len(touched) == 9 and sum(touched) == sum(untouched) > 0
    assert touched[-1] == 0 and sum(touched[:-1]) == sum(touched)
    node = native.current_numa_node()
    assert node >= 0
    srv = native.Server({"port": 0, "cpus": sorted(os.sched_getaffinity(0))[:2]})
    srv.start()
    try:
        memfd = native.pattern_memfd_numa()
        assert memfd and sum(memfd[:-1]) > 0 and memfd[-1] == 0
    finally:
        srv.stop()


def _fake_mi355x_node(monkeypatch, a, quota_cpus=None):
    """A full 8-GPU node as the driver's scaling run sees it: 2 sockets x 64
    cores x SMT2 (CPU c and c + 128 are siblings; socket s holds cores
    64s .. 64s + 63), 8 L3 domains of 8 cores per socket, GPUs 0-3 on NUMA
    node 0 and 4-7 on node 1 (PCI local_cpulist / numa_node per GPU)."""
    files = {}
    for c in range(256):
        core = c % 128
        sock = core // 64
        files[f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id"] = str(sock)
        files[f"/sys/devices/system/cpu/cpu{c}/topology/core_id"] = str(core % 64)
        lo = core // 8 * 8
        files[f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list"] = f"{lo}-{lo + 7},{lo + 128}-{lo + 135}"
    buses = [f"0000:{b:02x}:00.0" for b in (0x05, 0x15, 0x25, 0x35, 0x85, 0x95, 0xa5, 0xb5)]
    for d, bus in enumerate(buses):
        node = d // 4
        files[f"/sys/bus/pci/devices/{bus}/numa_node"] = str(node)
        files[f"/sys/bus/pci/devices/{bus}/local_cpulist"] = \
            f"{64 * node}-{64 * node + 63},{128 + 64 * node}-{128 + 64 * node + 63}"
    files["/sys/fs/cgroup/cpu.max"] = f"{quota_cpus * 100000} 100000" if quota_cpus else "max 100000"
    real = a._native

    class FakeNative:
        parse_cpulist = staticmethod(real.parse_cpulist)

        @staticmethod
        def gpu_device_count():
            return 8

        @staticmethod
        def gpu_pci_bus_id(d):
            return buses[d]

    monkeypatch.setattr(a, "_native", FakeNative)
    monkeypatch.setattr(a, "_read", lambda p: files.get(p))
    monkeypatch.setattr(a.os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")


@pytest.mark.parametrize("mode", ["pair", "share", "same", "split", "share_quota"])
def test_eight_ranks_of_a_node_get_disjoint_gpu_local_cpus(monkeypatch, mode):
    """bench.py --gpus 8 on one node: every rank plans its own placement at
    the same time (pair mode samples /proc/stat separately in each rank).
    The client / endpoint / submitter CPUs of the 8 ranks must not overlap,
    and each rank stays on its GPU's NUMA node; a collision would quietly
    halve a rank's one-stream rate in the driver's first scaling run."""
    import random

    from custom_go_client_benchmark_amd.parallel import affinity as a

    _fake_mi355x_node(monkeypatch, a, quota_cpus=128)
    rng = random.Random(7)
    sets = []
    for r in range(8):
        monkeypatch.setenv("LOCAL_RANK", str(r))
        # each rank sees its own (different) busy sample
        busy = {c: rng.random() * 0.5 for c in range(256)}
        monkeypatch.setattr(a, "cpu_busy", lambda sample_s=0.15, b=busy: b)
        p = a.plan(r, mode)
        assert p["client"] and p["server"], p
        mine = set(p["client"]) | set(p["server"]) | set(p.get("aux") or [])
        node = r // 4
        assert all((c % 128) // 64 == node for c in mine), (r, sorted(mine))
        if mode == "pair":
            assert p["picked_by"] == "quiet" and len({frozenset(p[k]) for k in ("client", "server", "aux")}) == 3
        if mode == "share_quota":
            assert len(p["client"]) <= 16  # 128-CPU quota over 8 ranks
        sets.append(mine)
    for i in range(8):
        for j in range(i + 1, 8):
            assert not (sets[i] & sets[j]), (mode, i, j, sorted(sets[i] & sets[j]))


def test_isolate_reader_gives_the_reader_a_whole_core(monkeypatch):
    """The multiplexed connection's reader gets one hardware thread of the
    quietest client core; neither the workers nor a shared endpoint keep
    either thread of that core."""
    from custom_go_client_benchmark_amd.parallel import affinity as a

    _fake_topology(monkeypatch, a)
    busy = {c: 0.0 for c in range(16)}
    busy[1] = busy[9] = 0.9
    monkeypatch.setattr(a, "cpu_busy", lambda sample_s=0.15: busy)
    pl = {"client": list(range(16)), "server": list(range(16)), "mode": "share_quota"}
    out = a.isolate_reader(pl)
    (r,) = out["reader_cpus"]
    core = {c for c in range(16) if a._same_core(c, r)}
    assert len(core) == 2 and 0 not in core and 1 not in core
    assert not core & set(out["client"]) and not core & set(out["server"])
    assert set(out["client"]) | core == set(range(16))
    assert pl["client"] == list(range(16))  # the input plan is not modified
    # too few cores to spare one: unchanged
    small = {"client": [2, 10], "server": [3, 11]}
    assert a.isolate_reader(small) == small


def test_isolate_sender_takes_another_whole_core(monkeypatch):
    """After isolate_reader, the endpoint's send threads get one hardware
    thread of the next quietest core: not the reader's core, and neither the
    workers nor the endpoint's other threads keep either thread of it."""
    from custom_go_client_benchmark_amd.parallel import affinity as a

    _fake_topology(monkeypatch, a)
    busy = {c: 0.0 for c in range(16)}
    monkeypatch.setattr(a, "cpu_busy", lambda sample_s=0.15: busy)
    pl = {"client": list(range(16)), "server": list(range(16)), "mode": "same"}
    rd = a.isolate_reader(pl)
    out = a.isolate_sender(rd)
    (s,) = out["send_cpus"]
    (r,) = out["reader_cpus"]
    score = {c for c in range(16) if a._same_core(c, s)}
    rcore = {c for c in range(16) if a._same_core(c, r)}
    assert len(score) == 2 and not score & rcore
    assert not score & set(out["client"]) and not score & set(out["server"])
    assert set(out["client"]) | score | rcore == set(range(16))
    assert rd.get("send_cpus") is None  # the input plan is not modified
    # too few cores to spare another one: unchanged
    small = {"client": [2, 10, 3, 11], "server": [2, 10, 3, 11], "reader_cpus": [4]}
    assert a.isolate_sender(small) == small


def test_fd_table_reserved(native):
    import resource

    n = native.reserve_fd_table()
    soft, _ = resource.getrlimit(resource.RLIMIT_NOFILE)
    assert n == 0 or 64 < n <= max(soft, 64)
    assert native.reserve_fd_table() == n  # once per process
