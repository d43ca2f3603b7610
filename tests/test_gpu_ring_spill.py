"""The per-sink ring's two round-4 receive paths, pinned down byte-exact
(ADVICE r4): the contiguous-ring spill (a receive window runs on into the
next free slot and commit() splits it at the slot end) and slot reuse on the
CRC kernel's host-visible status.  64 KiB slots with odd-sized gRPC messages
put message boundaries, slot ends and resume offsets at every relative
position; ring_span on and off must land the same bytes and verify the same
chunks."""
import pytest

pytestmark = pytest.mark.gpu

B = "princer-working-dirs"
P = "spill/file_"
SIZE = (5 << 20) + 12345


def _read(native, srv, span, faults=None):
    import torch

    if faults:
        srv.set_faults(faults)
    c = native.Client({"protocol": "grpc", "endpoint": srv.url, "retry_initial_s": 0.01})
    t = torch.empty(SIZE, dtype=torch.uint8, device="cuda:0")
    sink = native.GpuSink({"device": 0, "ring_slot_bytes": 64 << 10, "ring_slots": 4, "ring_span": span})
    sink.set_external_destination(t.data_ptr(), t.numel())
    r = c.read_gpu(B, P + "0", sink)
    torch.cuda.synchronize()
    bad, first = native.gpu_verify_pattern(0, t.data_ptr(), SIZE, P + "0", 0)
    return r, sink.stats(), bad, first, native.gpu_crc32c(0, t.data_ptr(), SIZE)


@pytest.fixture()
def odd_server(native):
    # 99,991-byte messages: never a multiple of the 64 KiB slot
    srv = native.Server({"port": 0, "grpc_chunk": 99991})
    srv.start()
    srv.add_synthetic(B, P, "", 0, 1, SIZE)
    yield srv
    srv.stop()


def test_spill_with_odd_messages_matches_no_span(native, odd_server, gpu_available):
    want = odd_server.object_info(B, P + "0")["crc32c"]
    out = {}
    for span in (True, False):
        r, st, bad, first, crc = _read(native, odd_server, span)
        assert r["bytes"] == SIZE and r["verified"] and not r["crc_mismatch"], (span, r)
        assert bad == 0, (span, first)
        assert crc == want
        out[span] = st
    # every gRPC message checked, on the GPU epilogue or by the host fold
    msgs = (SIZE + 99990) // 99991
    for span, st in out.items():
        assert st["chunks_verified_gpu"] + st["chunks_verified_host"] == msgs, (span, st)
        assert st["objects_verified"] == 1
    # reuse on the kernel's host-visible status happened (no HIP wait per slot)
    assert out[True]["flag_reuses"] + out[True]["slot_waits"] > 0


@pytest.mark.parametrize("at", [64 << 10, (64 << 10) * 7, (64 << 10) * 7 + 1, 99991 * 3, 99991 * 3 - 1,
                                (64 << 10) * 33 - 1])
def test_resume_mid_spill_byte_exact(native, odd_server, gpu_available, at):
    """A disconnect at a slot end, one byte either side of it, and at a
    message boundary: the retry resumes at read_offset and the object still
    lands byte-exact with its CRC32C verified, with and without spill."""
    for span in (True, False):
        r, st, bad, first, crc = _read(native, odd_server, span,
                                       faults={"disconnect_at": at, "disconnect_count": 1})
        assert r["bytes"] == SIZE and not r["crc_mismatch"] and r["verified"], (span, at, r)
        assert r["attempts"] >= 2, (span, at, r)
        assert bad == 0, (span, at, first)
        assert crc == odd_server.object_info(B, P + "0")["crc32c"]
