"""TLS transports: https (HTTP/1.1, ALPN http/1.1) and gRPC over TLS (ALPN h2)
against the synthetic server with a throw-away self-signed certificate;
certificate + host-name verification on by default."""
import os
import shutil
import subprocess

import pytest

B = "princer-working-dirs"
P = "princer_100M_files/file_"

pytestmark = pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI not available")


@pytest.fixture(scope="module")
def cert(tmp_path_factory):
    d = tmp_path_factory.mktemp("tls")
    key, crt = d / "key.pem", d / "cert.pem"
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(key), "-out",
                    str(crt), "-days", "1", "-subj", "/CN=localhost",
                    "-addext", "subjectAltName=DNS:localhost,IP:127.0.0.1"],
                   check=True, capture_output=True, timeout=60)
    return str(crt), str(key)


@pytest.fixture()
def tls_server(native, cert):
    crt, key = cert
    srv = native.Server({"port": 0, "tls_cert_file": crt, "tls_key_file": key})
    srv.start()
    srv.add_synthetic(B, P, "", 0, 1, (3 << 20) + 7)
    yield srv
    srv.stop()


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_read_over_tls_verified(native, tls_server, cert, proto):
    assert tls_server.url.startswith("https://")
    ep = tls_server.url.replace("127.0.0.1", "localhost")
    c = native.Client({"protocol": proto, "endpoint": ep, "tls_ca_file": cert[0]})
    r = c.read(B, P + "0")
    assert r["verified"] and r["bytes"] == (3 << 20) + 7
    data = os.urandom(700 << 10)
    m = c.write_bytes(B, "tls/up", data, True, 256 << 10)
    assert m["crc32c"] == native.crc32c(data)
    assert c.read_bytes(B, "tls/up") == data


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_untrusted_certificate_is_rejected(native, tls_server, proto):
    c = native.Client({"protocol": proto, "endpoint": tls_server.url, "retry_max_attempts": 1})
    with pytest.raises(native.StorageError, match="TLS handshake"):
        c.read(B, P + "0")


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_insecure_mode_skips_verification(native, tls_server, proto):
    c = native.Client({"protocol": proto, "endpoint": tls_server.url, "tls_verify": False})
    assert c.read(B, P + "0")["verified"]


def test_host_name_mismatch_is_rejected(native, cert):
    crt, key = cert
    srv = native.Server({"port": 0, "tls_cert_file": crt, "tls_key_file": key})
    srv.start()
    try:
        srv.add_synthetic(B, P, "", 0, 1, 4096)
        # the certificate names localhost / 127.0.0.1; 127.0.0.2 is not in it
        ep = srv.url.replace("127.0.0.1", "127.0.0.2")
        c = native.Client({"protocol": "http", "endpoint": ep, "tls_ca_file": crt, "retry_max_attempts": 1})
        with pytest.raises(native.StorageError):
            c.read(B, P + "0")
    finally:
        srv.stop()


def test_sliced_read_over_tls(native, tls_server, cert):
    r = native.Runner({"protocol": "grpc", "endpoint": tls_server.url, "tls_ca_file": cert[0], "bucket": B,
                       "object_prefix": P, "workers": 1, "reads_per_worker": 2, "slices": 3,
                       "slice_min_bytes": 1 << 20, "keep_records": False})
    r.start()
    r.wait()
    s = r.summary()
    assert s["errors"] == 0 and s["verified"] == 2, s["first_error"]


def test_cli_against_tls_fakegcs_subprocess(native, cert, tmp_path):
    import sys

    from custom_go_client_benchmark_amd import server as fs

    crt, key = cert
    ep = fs.start_subprocess(B, P, "", 0, 2, 1 << 20, extra_args=["-tls-cert", crt, "-tls-key", key])
    try:
        url = ep.url.replace("http://", "https://").replace("127.0.0.1", "localhost")
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        for proto in ("http", "grpc"):
            r = subprocess.run([sys.executable, "-m", "custom_go_client_benchmark_amd", "-endpoint", url,
                                "-client-protocol", proto, "-worker", "2", "-read-call-per-worker", "3",
                                "-tls-ca-file", crt], capture_output=True, text=True, timeout=120, cwd=root)
            assert r.returncode == 0, r.stderr[-2000:]
            assert len([l for l in r.stdout.splitlines() if l.endswith("ms")]) == 6
    finally:
        ep.stop()


def test_grpc_tls_many_streams_one_connection(native, tls_server, cert):
    """HTTP/2 over TLS: one reader thread and many writer threads share one
    SSL object (regression: concurrent SSL_read/SSL_write crashed)."""
    r = native.Runner({"protocol": "grpc", "endpoint": tls_server.url, "tls_ca_file": cert[0], "bucket": B,
                       "object_prefix": P, "workers": 8, "reads_per_worker": 6, "grpc_conn_pool_size": 1,
                       "keep_records": False, "object_names": [P + "0"]})
    r.start()
    r.wait()
    s = r.summary()
    assert s["errors"] == 0 and s["verified"] == 48, s["first_error"]
