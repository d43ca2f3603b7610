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
