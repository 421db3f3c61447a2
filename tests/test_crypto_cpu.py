"""RSA signatures (dalle_amd.parallel.crypto) against OpenSSL / OpenSSH, and owner-signed DHT records
(hivemind RSASignatureValidator semantics)."""
import os
import re
import shutil
import subprocess
import time

import pytest

from dalle_amd.parallel.crypto import RSAPrivateKey, RSAPublicKey
from dalle_amd.parallel.validation import RSASignatureValidator

openssl = shutil.which("openssl")


def _openssl_key(tmp_path):
    pem = tmp_path / "k.pem"
    subprocess.run([openssl, "genrsa", "-out", str(pem), "2048"], check=True, capture_output=True)
    text = subprocess.run([openssl, "rsa", "-in", str(pem), "-text", "-noout"], check=True, capture_output=True,
                          text=True).stdout

    def field(name):
        m = re.search(name + r":\s*\n((?:\s+[0-9a-f:]+\n)+)", text)
        return int(m.group(1).replace(":", "").replace(" ", "").replace("\n", ""), 16)

    e = int(re.search(r"publicExponent: (\d+)", text).group(1))
    key = RSAPrivateKey(field("modulus"), e, field("privateExponent"), field("prime1"), field("prime2"))
    return pem, key


@pytest.mark.skipif(openssl is None, reason="openssl CLI not available")
def test_signature_matches_openssl(tmp_path):
    pem, key = _openssl_key(tmp_path)
    data = os.urandom(1000)
    (tmp_path / "d.bin").write_bytes(data)
    ref = subprocess.run([openssl, "dgst", "-sha256", "-sign", str(pem), str(tmp_path / "d.bin")], check=True,
                         capture_output=True).stdout
    assert key.sign(data) == ref  # PKCS#1 v1.5 is deterministic: byte-identical signatures
    pub = key.get_public_key()
    assert pub.verify(data, ref)
    assert not pub.verify(data + b"x", ref)
    assert not pub.verify(data, ref[:-1] + bytes([ref[-1] ^ 1]))


@pytest.mark.skipif(shutil.which("ssh-keygen") is None or openssl is None, reason="ssh-keygen not available")
def test_public_key_is_openssh_format(tmp_path):
    pem, key = _openssl_key(tmp_path)
    os.chmod(pem, 0o600)
    ref = subprocess.run(["ssh-keygen", "-y", "-f", str(pem)], check=True, capture_output=True).stdout.split()
    ours = key.get_public_key().to_bytes().split()
    assert ours[:2] == ref[:2]
    assert RSAPublicKey.from_bytes(b" ".join(ref[:2])) == key.get_public_key()


def test_keygen_roundtrip_and_persistence(tmp_path):
    k = RSAPrivateKey.generate(1024)
    assert k.n.bit_length() == 1024
    sig = k.sign(b"payload")
    assert k.get_public_key().verify(b"payload", sig)
    path = str(tmp_path / "id.json")
    k.save(path)
    assert oct(os.stat(path).st_mode & 0o777) == "0o600"
    assert RSAPrivateKey.load(path).sign(b"payload") == sig


def test_signed_records_through_the_dht():
    from dalle_amd.parallel.dht import DHT, get_dht_time

    alice = RSASignatureValidator(RSAPrivateKey.generate(1024))
    mallory = RSASignatureValidator(RSAPrivateKey.generate(1024))
    host = DHT(start=True, host_maddrs=["/ip4/127.0.0.1/tcp/0"], record_validators=[alice])
    try:
        maddr = host.get_visible_maddrs()[0]
        peer = DHT(start=True, initial_peers=[maddr], record_validators=[mallory])
        exp = get_dht_time() + 60
        assert host.store("run_metrics", subkey=alice.local_public_key, value={"loss": 1.5}, expiration_time=exp)
        got = peer.get("run_metrics")
        assert got.value[alice.local_public_key].value == {"loss": 1.5}
        # mallory writes under her OWN marker: signed by her, accepted
        assert peer.store("run_metrics", subkey=mallory.local_public_key, value={"loss": 9.0}, expiration_time=exp)
        # a record claiming alice's identity without alice's signature is dropped by every reader
        import msgpack

        forged = msgpack.packb({"loss": 0.0}, use_bin_type=True) + b"[signature:AAAA]"
        peer._client.store("run_metrics2", alice.local_public_key, forged, exp, b"someone")
        assert host.get("run_metrics2") is None
        vals = {k: v.value for k, v in host.get("run_metrics").value.items()}
        assert vals == {alice.local_public_key: {"loss": 1.5}, mallory.local_public_key: {"loss": 9.0}}
        # unprotected keys are unaffected
        assert peer.store("plain", value=3, expiration_time=exp)
        assert host.get("plain").value == 3
        peer.shutdown()
    finally:
        host.shutdown()


def test_validator_rejects_tampering():
    v = RSASignatureValidator(RSAPrivateKey.generate(1024))
    exp = time.time() + 10
    signed = v.sign_value("k", v.local_public_key, b"\x01\x02", exp)
    assert v.validate_signed("k", v.local_public_key, signed, exp)
    assert v.strip_value(signed) == b"\x01\x02"
    assert not v.validate_signed("k", v.local_public_key, signed, exp + 1)  # expiration is signed too
    assert not v.validate_signed("k2", v.local_public_key, signed, exp)
    assert not v.validate_signed("k", v.local_public_key, b"\x01\x02", exp)  # unsigned
    assert v.validate_signed("k", b"nobody", b"\x01\x02", exp)  # not owner-protected


def test_access_tokens(tmp_path, monkeypatch):
    from huggingface_auth import HuggingFaceAuthorizer, LocalAuthority

    monkeypatch.delenv("DALLE_AMD_AUTH_SERVER", raising=False)
    key_path = str(tmp_path / "authority.json")
    a1 = HuggingFaceAuthorizer("org", "model", "alice:tok", local_public_key=b"pk-a", authority=LocalAuthority(key_path))
    tok = a1.get_token()
    assert tok.username == "alice" and a1.is_token_valid(tok)
    # a second peer of the node shares the authority key file: it accepts alice's token
    a2 = HuggingFaceAuthorizer("org", "model", "bob:tok", local_public_key=b"pk-b", authority=LocalAuthority(key_path))
    assert a2.is_token_valid(tok)
    # forged fields or a foreign authority fail
    import dataclasses

    assert not a2.is_token_valid(dataclasses.replace(tok, username="mallory"))
    assert not a2.is_token_valid(dataclasses.replace(tok, public_key=b"pk-m"))
    other = LocalAuthority(private_key=RSAPrivateKey.generate(1024))
    assert not a2.is_token_valid(other.issue("alice", b"pk-a"))
    assert not a2.is_token_valid(dataclasses.replace(tok, expiration_time=time.time() - 1))
