"""CDNA4 CRC32C kernels vs the host CRC32C (fp32-reference analogue: exact)."""
import os

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 4095, 4096, 4097, 16383, 16384, 16385, 2 << 20, (2 << 20) + 13,
                               (4 << 20) + 16384 + 7, 64 << 20])
@pytest.mark.parametrize("misalign", [0, 1, 7, 15])
def test_gpu_crc_matches_host(native, gpu_available, n, misalign):
    import torch

    data = os.urandom(n)
    buf = torch.zeros(n + 64, dtype=torch.uint8, device="cuda:0")
    if n:
        buf[misalign : misalign + n] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    torch.cuda.synchronize()
    got = native.gpu_crc32c(0, buf.data_ptr() + misalign, n)
    assert got == native.crc32c(data)


@pytest.mark.parametrize("bank_private", [False, True])
def test_gpu_crc_large_multi_segment(native, gpu_available, bank_private):
    """> 1 GiB through the bulk (non-fused) tile kernels: the bank-private
    slice-by-4 default (CrcLaunchOptions::bank_private) and slice-by-16."""
    import torch

    n = (1 << 30) + 12345  # > 1 GiB: several kernel segments combined on host
    t = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda:0")
    host = t.cpu().numpy().tobytes()
    defaults = native.set_crc_options({})
    try:
        native.set_crc_options({"bank_private": bank_private})
        assert native.gpu_crc32c(0, t.data_ptr(), n) == native.crc32c(host)
    finally:
        native.set_crc_options(defaults)


def test_fill_and_verify_pattern(native, gpu_available):
    import torch

    name = "princer_100M_files/file_7"
    n = (5 << 20) + 3
    t = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    native.gpu_fill_pattern(0, t.data_ptr(), n, name, 1000)
    assert t.cpu().numpy().tobytes() == native.object_bytes(name, 1000, n)
    bad, _ = native.gpu_verify_pattern(0, t.data_ptr(), n, name, 1000)
    assert bad == 0
    t[12345] ^= 0xFF
    bad, first = native.gpu_verify_pattern(0, t.data_ptr(), n, name, 1000)
    assert bad == 1 and first == 12345


@pytest.mark.parametrize("opts", [{"slot_waves": 1}, {"xor_arrival": False}, {"slot_waves": 8},
                                  {"slice8": False}, {"slice8": False, "slot_waves": 1},
                                  {"slice8": False, "xor_arrival": False}, {"slice8": True},
                                  {"bank_private": False}, {"bank_private": True}])
def test_crc_kernel_variants(native, gpu_available, opts):
    """Every CRC kernel variant (gpu/crc32c_gpu.h CrcLaunchOptions) against
    the host CRC32C.  One wave per workgroup on 600 - 1024 tiles puts more
    than 32 workgroups in a counter group, which takes the stored-tile
    epilogue instead of the 64-bit XOR arrival words."""
    import torch

    defaults = native.set_crc_options({})
    try:
        native.set_crc_options(opts)
        for size, mis in [(4096 * 600 + 5, 3), (4 << 20, 0), ((2 << 20) + 13, 7), (17, 1), ((9 << 20) + 5, 0)]:
            data = os.urandom(size)
            buf = torch.zeros(size + 64, dtype=torch.uint8, device="cuda:0")
            buf[mis:mis + size] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
            torch.cuda.synchronize()
            assert native.gpu_crc32c(0, buf.data_ptr() + mis, size) == native.crc32c(data), (opts, size, mis)
    finally:
        native.set_crc_options(defaults)
