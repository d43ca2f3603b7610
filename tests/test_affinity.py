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
