"""Synthetic GCS endpoint management (no network on the benchmark boxes).

  start_inprocess(...)  native server threads inside this process
  start_subprocess(...) the standalone `bin/fakegcs` binary (HTTP/1.1 + h2c
                        gRPC on one port), e.g. one per rank or shared
  storage_v2_pb         Python protobuf classes for interop tests
"""
from __future__ import annotations

import os
import signal
import subprocess
import tempfile
import time
from dataclasses import dataclass

from .. import _native

BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bin", "fakegcs")


@dataclass
class Endpoint:
    url: str
    kind: str
    handle: object = None

    def stop(self):
        if self.kind == "inprocess":
            self.handle.stop()
        elif self.kind == "subprocess" and self.handle.poll() is None:
            self.handle.send_signal(signal.SIGTERM)
            try:
                self.handle.wait(timeout=10)
            except subprocess.TimeoutExpired:
                self.handle.kill()
                self.handle.wait()


def start_inprocess(bucket: str, prefix: str, suffix: str, first: int, count: int, size: int, md5: bool = False,
                    cpus=None, require_auth: bool = False, grpc_chunk: int = 2 << 20,
                    retain_uploads: bool = True, send_cpus=None) -> Endpoint:
    srv = _native.Server({"port": 0, "md5": md5, "cpus": list(cpus or []), "require_auth": require_auth,
                          "grpc_chunk": grpc_chunk, "retain_uploads": retain_uploads,
                          "send_cpus": list(send_cpus or [])})
    srv.start()
    if count > 0:
        srv.add_synthetic(bucket, prefix, suffix, first, count, size)
    return Endpoint(srv.url, "inprocess", srv)


def start_subprocess(bucket: str, prefix: str, suffix: str, first: int, count: int, size: int, md5: bool = True,
                     extra_args: list | None = None, timeout_s: float = 120.0) -> Endpoint:
    if not os.path.exists(BIN):
        raise FileNotFoundError(f"{BIN} not built (run `make`)")
    fd, port_file = tempfile.mkstemp(prefix="fakegcs-port-")
    os.close(fd)
    os.unlink(port_file)
    args = [BIN, "-port", "0", "-port-file", port_file, "-bucket", bucket, "-object-prefix", prefix,
            "-object-suffix", suffix, "-first-object", str(first), "-objects", str(count), "-object-size", str(size),
            f"-md5={'true' if md5 else 'false'}"] + list(extra_args or [])
    proc = subprocess.Popen(args, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    deadline = time.time() + timeout_s
    while time.time() < deadline:
        if os.path.exists(port_file):
            with open(port_file) as f:
                port = int(f.read().strip())
            os.unlink(port_file)
            return Endpoint(f"http://127.0.0.1:{port}", "subprocess", proc)
        if proc.poll() is not None:
            raise RuntimeError(f"fakegcs exited early: {proc.stderr.read().decode(errors='replace')}")
        time.sleep(0.02)
    proc.kill()
    raise TimeoutError("fakegcs did not start")
