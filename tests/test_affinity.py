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
