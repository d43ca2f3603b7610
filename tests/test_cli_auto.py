"""The CLI's `-affinity auto` and ring auto-geometry choices
(custom_go_client_benchmark_amd/cli.py auto_affinity / auto_ring), each
pinned to the measurement that picked it."""
import pytest

from custom_go_client_benchmark_amd.cli import auto_affinity, auto_ring


@pytest.mark.parametrize("args,want", [
    (("gpu", "grpc", 1, 1, 1, "read"), "pair"),          # one stream per read: the bench's placement
    (("gpu", "grpc", 8, 1, 1, "read"), "same"),          # several GPU readers: one L3 domain
    (("gpu", "http", 1, 1, 8, "read"), "share"),         # sliced reads spread over the share
    (("discard", "grpc", 48, 1, 1, "read"), "same"),     # 48 streams on one connection (r3_mux_thp/refplace)
    (("discard", "http2", 48, 1, 1, "read"), "same"),
    (("discard", "grpc", 8, 8, 1, "read"), "quota"),     # a connection per worker: no shared reader
    (("discard", "http", 48, 1, 1, "read"), "quota"),    # HTTP workers each receive: the quota's cores
    (("gpu", "grpc", 1, 1, 1, "write"), "pair"),         # upload from HBM: three quiet cores
    (("gpu", "grpc", 1, 1, 8, "write"), "none"),         # composite upload
    (("discard", "grpc", 1, 1, 1, "write"), "none"),
])
def test_auto_affinity(args, want):
    assert auto_affinity(*args) == want


def test_auto_ring_keeps_the_receive_destinations_small():
    assert auto_ring(1, 1) == (1 << 20, 4)     # the headline's ring (r4_main8)
    assert auto_ring(8, 1) == (1 << 20, 2)     # r3_mux_thp/listring
    assert auto_ring(48, 1) == (1 << 20, 2)
    assert auto_ring(1, 8) == (2 << 20, 2)     # r3_ring_thp/sliced
    # every worker's ring together stays within an L3 domain for the
    # config-3 geometry (8 readers)
    b, n = auto_ring(8, 1)
    assert 8 * b * n <= 32 << 20
