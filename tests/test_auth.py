"""OAuth2 token sources (reference auth.go:28-76) against the fake server's
/token and metadata endpoints: service-account JWT (RS256, signature verified
by the server), authorized_user refresh grant, GCE metadata server, ADC chain."""
import base64
import json
import os

import pytest

B = "princer-working-dirs"
P = "princer_100M_files/file_"


@pytest.fixture()
def keypair(native):
    return native.rsa_generate()


@pytest.fixture()
def auth_server(native, keypair):
    srv = native.Server({"port": 0, "require_auth": True, "jwt_public_key_pem": keypair[1]})
    srv.start()
    srv.add_synthetic(B, P, "", 0, 1, 65536)
    yield srv
    srv.stop()


def _key_file(tmp_path, pem, token_uri):
    key = {"type": "service_account", "project_id": "gcs-fuse-test", "private_key_id": "kid-1",
           "private_key": pem, "client_email": "bench@gcs-fuse-test.iam.gserviceaccount.com",
           "token_uri": token_uri}
    p = tmp_path / "key.json"
    p.write_text(json.dumps(key))
    return str(p)


def test_jwt_assertion_shape(native, keypair, tmp_path):
    kf = _key_file(tmp_path, keypair[0], "http://127.0.0.1:1/token")
    a = native.service_account_assertion(open(kf).read(), "", 1700000000)
    h, c, s = a.split(".")
    pad = lambda x: x + "=" * (-len(x) % 4)  # noqa: E731
    header = json.loads(base64.urlsafe_b64decode(pad(h)))
    claims = json.loads(base64.urlsafe_b64decode(pad(c)))
    assert header == {"alg": "RS256", "typ": "JWT", "kid": "kid-1"}
    assert claims["scope"] == "https://www.googleapis.com/auth/devstorage.full_control"
    assert claims["exp"] - claims["iat"] == 3600 and claims["aud"] == "http://127.0.0.1:1/token"
    assert len(base64.urlsafe_b64decode(pad(s))) == 256  # RSA-2048 signature


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_service_account_key_file(native, auth_server, keypair, tmp_path, proto):
    kf = _key_file(tmp_path, keypair[0], auth_server.url + "/token")
    c = native.Client({"protocol": proto, "endpoint": auth_server.url, "auth": "key_file", "key_file": kf})
    assert c.read(B, P + "0")["verified"]


def test_wrong_key_rejected_by_token_endpoint(native, auth_server, tmp_path):
    other_priv, _ = native.rsa_generate()
    kf = _key_file(tmp_path, other_priv, auth_server.url + "/token")
    with pytest.raises(native.StorageError, match="Invalid JWT Signature"):
        native.Client({"protocol": "http", "endpoint": auth_server.url, "auth": "key_file", "key_file": kf}).read(
            B, P + "0")


def test_adc_chain_metadata_server(native, auth_server, tmp_path, monkeypatch):
    monkeypatch.delenv("GOOGLE_APPLICATION_CREDENTIALS", raising=False)
    monkeypatch.setenv("HOME", str(tmp_path))  # no gcloud ADC file
    monkeypatch.setenv("GCE_METADATA_HOST", auth_server.url.replace("http://", ""))
    kind, tok = native.get_access_token("", "")
    assert kind == "metadata" and tok.startswith("ya29.fake-")
    c = native.Client({"protocol": "grpc", "endpoint": auth_server.url, "auth": "adc"})
    assert c.read(B, P + "0")["verified"]


def test_adc_chain_authorized_user_file(native, auth_server, tmp_path, monkeypatch):
    f = tmp_path / "adc.json"
    f.write_text(json.dumps({"type": "authorized_user", "client_id": "cid", "client_secret": "sec",
                             "refresh_token": "rt"}))
    monkeypatch.setenv("GOOGLE_APPLICATION_CREDENTIALS", str(f))
    kind, tok = native.get_access_token("", auth_server.url + "/token")
    assert kind == "authorized_user" and tok.startswith("ya29.fake-")


def test_missing_key_file_error_names_method(native):
    with pytest.raises(native.StorageError, match="newTokenSourceFromPath"):
        native.get_access_token("/nonexistent/key.json", "")
