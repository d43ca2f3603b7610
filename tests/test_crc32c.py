"""CRC32C host algebra + bit-exact emulation of the GPU kernel algorithm."""
import os
import zlib

import pytest


def test_known_vectors(native):
    assert native.crc32c(b"123456789") == 0xE3069283
    assert native.crc32c(b"") == 0
    assert native.crc32c(b"\x00" * 32) == 0x8A9136AA
    assert native.crc32c(b"\xff" * 32) == 0x62A8AB43


def test_extend_and_combine(native):
    a, b = os.urandom(100001), os.urandom(777)
    ca, cb = native.crc32c(a), native.crc32c(b)
    assert native.crc32c_extend(ca, b) == native.crc32c(a + b)
    assert native.crc32c_combine(ca, cb, len(b)) == native.crc32c(a + b)


def test_raw_fixup_identity(native):
    for n in [0, 1, 7, 4096, 123457]:
        d = os.urandom(n)
        assert native.crc32c_raw(d) ^ native.crc32c_fixup(n) == native.crc32c(d)


def test_large_buffer_interleaved_path(native):
    # > 3 * 8 KiB exercises the 3-stream interleave + shift-table recombine
    d = os.urandom((1 << 20) + 12345)
    c = 0
    for i in range(0, len(d), 1000):
        c = native.crc32c_extend(c, d[i : i + 1000])
    assert native.crc32c(d) == c


@pytest.mark.parametrize("misalign", [0, 1, 3, 8, 15])
@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 255, 256, 257, 4095, 4096, 4097, 16383, 16384, 16385, 16400,
                               65536 + 5, (1 << 20) + 3])
@pytest.mark.parametrize("geom", [(14, 8), (12, 1), (14, 1), (12, 8), (12, 0)])
def test_gpu_algorithm_emulation(native, misalign, n, geom):
    """Kernel math on the CPU: 16 KiB / 4 KiB tiles x fused (1 wave per
    segment) / separate (8 waves per segment) fold / slot kernel (GF(2) lane
    and tile matrices, fold_waves=0), parallel 1..16 B tail."""
    tl, fw = geom
    d = os.urandom(n)
    want = native.crc32c(d)
    raw, crc, status = native.emulate_gpu_crc32c(d, misalign, want, True, tl, fw)
    assert crc == want and status == 1
    assert raw == native.crc32c_raw(d)
    _, _, bad = native.emulate_gpu_crc32c(d, misalign, want ^ 1, True, tl, fw)
    assert bad == 2


@pytest.mark.parametrize("geom", [(14, 8), (12, 1), (14, 1)])
def test_emulation_multi_megabyte_tile_fold(native, geom):
    # more tiles than fold threads exercises the strided Horner step
    d = os.urandom(9 * (1 << 20) + 999)
    raw, crc, _ = native.emulate_gpu_crc32c(d, 5, 0, False, *geom)
    assert crc == native.crc32c(d)


@pytest.mark.parametrize("n,misalign", [((4 << 20) - 5, 3), (4 << 20, 0), ((4 << 20) + 16, 0)])
def test_emulation_slot_kernel_longest_segment(native, n, misalign):
    """The slot kernel's tile matrices cover segments of up to 1024 tiles
    (4 MiB + up to 16 tail bytes); one more tile is outside its domain."""
    d = os.urandom(n)
    raw, crc, status = native.emulate_gpu_crc32c(d, misalign, native.crc32c(d), True, 12, 0)
    assert crc == native.crc32c(d) and status == 1
    _, _, st = native.emulate_gpu_crc32c(d + b"x" * 4096, 3, 0, True, 12, 0)
    assert st == 3


def test_slot_matrices_match_shift_tables(native):
    """lane_k / tile_k columns are the GF(2) shifts the tree and fold tables
    apply: shift(v, n) == XOR of the columns of v's set bits."""
    import random
    for nbytes in (64, 64 * 63, 4096, 4096 * 1023):
        v = random.getrandbits(32)
        cols = [native.crc32c_shift(1 << i, nbytes) for i in range(32)]
        acc = 0
        for i in range(32):
            if v >> i & 1:
                acc ^= cols[i]
        assert acc == native.crc32c_shift(v, nbytes)


def test_goog_hash_parsing(native):
    has, crc, md5 = native.parse_goog_hash("crc32c=4waSgw==,md5=XUFAKrxLKna5cZ2REBfFkg==")
    assert has and crc == 0xE3069283
    assert len(md5) == 16
