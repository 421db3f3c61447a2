"""RSA keys and signatures for record ownership and access tokens.

hivemind signs owner-protected DHT records and authority-issued access tokens with RSA through the
``cryptography`` package (OpenSSL). That package is not in this image, so this module implements the
two primitives the protocol needs on Python's native big integers (``pow`` with a modulus is C):

* key generation: two random primes (trial division + 40-round Miller-Rabin), e = 65537;
* RSASSA-PKCS1-v1_5 signatures over SHA-256 (RFC 8017 §8.2), deterministic;
* public keys serialised in the OpenSSH wire format (``ssh-rsa <base64>``), which is what hivemind's
  ``RSAPublicKey.to_bytes()`` emits, and private keys in a small JSON file for ``identity_path``.
"""
from __future__ import annotations

import base64
import hashlib
import json
import os
import secrets
import struct
import threading
from typing import Optional, Tuple

_SMALL_PRIMES = [p for p in range(3, 2000, 2) if all(p % q for q in range(3, int(p ** 0.5) + 1, 2))]
# DER prefix of DigestInfo(SHA-256) (RFC 8017 §9.2 note 1)
_SHA256_PREFIX = bytes.fromhex("3031300d060960864801650304020105000420")


def _is_probable_prime(n: int, rounds: int = 40) -> bool:
    if n < 2:
        return False
    for p in _SMALL_PRIMES:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for _ in range(rounds):
        a = secrets.randbelow(n - 3) + 2
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = pow(x, 2, n)
            if x == n - 1:
                break
        else:
            return False
    return True


def _random_prime(bits: int) -> int:
    while True:
        # top two bits set (so p*q has exactly 2*bits bits), odd
        c = secrets.randbits(bits) | (3 << (bits - 2)) | 1
        if _is_probable_prime(c):
            return c


def _i2b(x: int, length: int) -> bytes:
    return x.to_bytes(length, "big")


def _ssh_string(b: bytes) -> bytes:
    return struct.pack(">I", len(b)) + b


def _ssh_mpint(x: int) -> bytes:
    raw = x.to_bytes((x.bit_length() + 8) // 8, "big")  # leading zero byte keeps it positive
    return _ssh_string(raw)


def _read_ssh(buf: bytes, off: int) -> Tuple[bytes, int]:
    (n,) = struct.unpack(">I", buf[off:off + 4])
    return buf[off + 4:off + 4 + n], off + 4 + n


class RSAPublicKey:
    def __init__(self, n: int, e: int = 65537):
        self.n, self.e = n, e

    @property
    def size_bytes(self) -> int:
        return (self.n.bit_length() + 7) // 8

    def verify(self, data: bytes, signature: bytes) -> bool:
        k = self.size_bytes
        if len(signature) != k:
            return False
        s = int.from_bytes(signature, "big")
        if s >= self.n:
            return False
        return _i2b(pow(s, self.e, self.n), k) == _emsa_pkcs1_v15(data, k)

    def to_bytes(self) -> bytes:
        blob = _ssh_string(b"ssh-rsa") + _ssh_mpint(self.e) + _ssh_mpint(self.n)
        return b"ssh-rsa " + base64.b64encode(blob)

    @classmethod
    def from_bytes(cls, data: bytes) -> "RSAPublicKey":
        kind, b64 = data.split(b" ", 1)
        if kind != b"ssh-rsa":
            raise ValueError("not an ssh-rsa public key")
        blob = base64.b64decode(b64, validate=True)
        name, off = _read_ssh(blob, 0)
        e, off = _read_ssh(blob, off)
        n, off = _read_ssh(blob, off)
        if name != b"ssh-rsa" or off != len(blob):
            raise ValueError("malformed ssh-rsa public key")
        return cls(int.from_bytes(n, "big"), int.from_bytes(e, "big"))

    def __eq__(self, other):
        return isinstance(other, RSAPublicKey) and (self.n, self.e) == (other.n, other.e)

    def __hash__(self):
        return hash((self.n, self.e))


def _emsa_pkcs1_v15(data: bytes, k: int) -> bytes:
    t = _SHA256_PREFIX + hashlib.sha256(data).digest()
    if k < len(t) + 11:
        raise ValueError("RSA modulus too short for SHA-256 PKCS#1 v1.5")
    return b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t


class RSAPrivateKey:
    _process_wide: Optional["RSAPrivateKey"] = None
    _lock = threading.Lock()

    def __init__(self, n: int, e: int, d: int, p: int, q: int):
        self.n, self.e, self.d, self.p, self.q = n, e, d, p, q
        # CRT parameters: a signature costs two half-size exponentiations
        self._dp, self._dq, self._qinv = d % (p - 1), d % (q - 1), pow(q, -1, p)

    @classmethod
    def generate(cls, bits: int = 2048, e: int = 65537) -> "RSAPrivateKey":
        while True:
            p, q = _random_prime(bits // 2), _random_prime(bits - bits // 2)
            if p == q:
                continue
            phi = (p - 1) * (q - 1)
            try:
                d = pow(e, -1, phi)
            except ValueError:  # e not invertible (gcd(e, phi) > 1): draw again
                continue
            return cls(p * q, e, d, max(p, q), min(p, q))

    @classmethod
    def process_wide(cls) -> "RSAPrivateKey":
        with cls._lock:
            if cls._process_wide is None:
                cls._process_wide = cls.generate()
            return cls._process_wide

    def get_public_key(self) -> RSAPublicKey:
        return RSAPublicKey(self.n, self.e)

    def sign(self, data: bytes) -> bytes:
        k = (self.n.bit_length() + 7) // 8
        m = int.from_bytes(_emsa_pkcs1_v15(data, k), "big")
        m1, m2 = pow(m, self._dp, self.p), pow(m, self._dq, self.q)
        h = (self._qinv * (m1 - m2)) % self.p
        return _i2b(m2 + h * self.q, k)

    # -- persistence (identity files) ------------------------------------------------------------
    def save(self, path: str):
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        with os.fdopen(fd, "w") as f:
            json.dump({"n": hex(self.n), "e": self.e, "d": hex(self.d), "p": hex(self.p), "q": hex(self.q)}, f)

    @classmethod
    def load(cls, path: str) -> "RSAPrivateKey":
        with open(path) as f:
            o = json.load(f)
        return cls(int(o["n"], 16), int(o["e"]), int(o["d"], 16), int(o["p"], 16), int(o["q"], 16))

    @classmethod
    def load_or_create(cls, path: Optional[str]) -> "RSAPrivateKey":
        if path is None:
            return cls.process_wide()
        if os.path.exists(path):
            return cls.load(path)
        key = cls.generate()
        key.save(path)
        return key
