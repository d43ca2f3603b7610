"""The endpoint's zero-copy send paths (Server config send_source): synthetic object
bodies leave by vmsplice from the pattern's THP copy (default) or by sendfile
from its memfd.  Both must put the same bytes on the wire, over HTTP/1.1,
gRPC and HTTP/2, with faults still cutting in at the right byte
(profiles/r3_splice)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys
sys.path.insert(0, %(root)r)
import custom_go_client_benchmark_amd as pkg
n = pkg._native
B, P = "b", "princer_100M_files/file_"
srv = n.Server({"port": 0, "send_source": %(mode)r})
srv.start()
size = (5 << 20) + 4097
srv.add_synthetic(B, P, "", 0, 2, size)
want = n.object_bytes(P + "1", 0, size)
for proto in ("http", "grpc", "http2"):
    c = n.Client({"protocol": proto, "endpoint": srv.url, "retry_initial_s": 0.001})
    assert c.read_bytes(B, P + "1") == want, proto
    assert c.read(B, P + "1")["verified"], proto
    off, lim = (1 << 20) + 3, (2 << 20) + 5
    assert c.read_bytes(B, P + "1", off, lim) == want[off:off + lim], proto
srv.set_faults({"corrupt_at": (3 << 20) + 11, "corrupt_count": 1})
r = n.Client({"protocol": "grpc", "endpoint": srv.url}).read(B, P + "0")
assert r["crc_mismatch"], r
srv.stop()
print("nodes", n.pattern_memfd_numa())
"""


@pytest.mark.parametrize("mode", ["vmsplice", "sendfile"])
def test_send_paths_put_the_same_bytes_on_the_wire(mode):
    env = dict(os.environ, GCSB_NO_TORCH="1")
    r = subprocess.run([sys.executable, "-c", SCRIPT % {"root": ROOT, "mode": mode}], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    # the send source exists and its pages were counted (THP copy or memfd)
    assert "nodes" in r.stdout and r.stdout.strip() != "nodes []", r.stdout
