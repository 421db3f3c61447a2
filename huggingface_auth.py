"""Peer authorisation (reference ``huggingface_auth.py:1-193``).

The reference asks a Hugging Face-hosted authority (``PUT {auth}/api/experiments/join`` with the
user's HF token) for an authority-signed access token (username, peer public key, expiry), retried
with exponential backoff, refreshed one minute before expiry, and validated by signature + expiry.

Same protocol here, with two authorities:
* a remote one when ``DALLE_AMD_AUTH_SERVER`` is set (HTTPS via ``requests``); its response carries
  the token and the authority's RSA public key (``auth_server_public_key``);
* an offline local authority whose RSA key lives in ``DALLE_AMD_AUTH_KEY`` (created on first use,
  mode 0600) so the peers of one node can issue / verify tokens without network access.
Tokens are RSASSA-PKCS1-v1_5 / SHA-256 signatures by the authority (``dalle_amd.parallel.crypto``),
verified with the authority's public key plus the expiry.
"""
import base64
import getpass
import json
import os
import time
from dataclasses import dataclass
from typing import Optional

from dalle_amd.utils.logging import get_logger

logger = get_logger(__name__)


def call_with_retries(func, n_retries: int = 10, initial_delay: float = 1.0):
    """``func()`` with exponential backoff (initial_delay * 2^attempt seconds between attempts); the
    last attempt's exception propagates."""
    attempt = 0
    while True:
        try:
            return func()
        except Exception as err:  # noqa: BLE001 - any transport / server error is retried
            attempt += 1
            if attempt >= n_retries:
                raise
            wait = initial_delay * 2 ** (attempt - 1)
            name = getattr(func, "__name__", repr(func))
            logger.warning(f"{name} failed ({err!r}); attempt {attempt + 1}/{n_retries} in {wait:.1f} s")
            time.sleep(wait)


@dataclass
class AccessToken:
    username: str
    public_key: bytes
    expiration_time: float
    signature: bytes = b""

    def payload(self) -> bytes:
        return json.dumps([self.username, base64.b64encode(self.public_key).decode(), self.expiration_time]).encode()


class LocalAuthority:
    """Offline token authority: an RSA key shared by the peers of one node through a key file."""

    def __init__(self, key_path: Optional[str] = None, private_key=None):
        from dalle_amd.parallel.crypto import RSAPrivateKey

        self._key = private_key or RSAPrivateKey.load_or_create(key_path or os.environ.get("DALLE_AMD_AUTH_KEY"))

    @property
    def public_key(self):
        return self._key.get_public_key()

    def issue(self, username: str, public_key: bytes, lifetime: float = 3600.0) -> AccessToken:
        tok = AccessToken(username, public_key, time.time() + lifetime)
        tok.signature = self._key.sign(tok.payload())
        return tok

    def verify(self, tok: AccessToken) -> bool:
        return verify_access_token(tok, self.public_key)


def verify_access_token(tok: AccessToken, authority_public_key) -> bool:
    """Authority signature over (username, peer public key, expiry) and not yet expired."""
    try:
        return authority_public_key.verify(tok.payload(), tok.signature) and tok.expiration_time > time.time()
    except Exception:  # noqa: BLE001  (malformed token)
        return False


class HuggingFaceAuthorizer:
    _AUTHORITY_REFRESH = 60.0  # refresh one minute before expiry (huggingface_auth.py)

    def __init__(self, organization_name: str, model_name: str, hf_user_access_token: str, local_public_key: bytes = b"",
                 authority: Optional[LocalAuthority] = None):
        self.organization_name, self.model_name = organization_name, model_name
        self.hf_user_access_token = hf_user_access_token
        self.local_public_key = local_public_key
        self.authority = authority
        self._authority_public_key = None
        self.username: Optional[str] = None
        self.coordinator_ip, self.coordinator_port = None, None
        self._token: Optional[AccessToken] = None

    def get_token(self) -> AccessToken:
        if self._token is None or self._token.expiration_time - time.time() < self._AUTHORITY_REFRESH:
            call_with_retries(self.join_experiment)
        return self._token

    def join_experiment(self):
        server = os.environ.get("DALLE_AMD_AUTH_SERVER")
        if server:
            import requests

            r = requests.put(f"{server}/api/experiments/join", params={"experiment_id": f"{self.organization_name}/{self.model_name}"},
                             headers={"Authorization": f"Bearer {self.hf_user_access_token}"},
                             json={"experiment_join_input": {"peer_public_key": base64.b64encode(self.local_public_key).decode()}},
                             timeout=30)
            r.raise_for_status()
            resp = r.json()
            tok = resp["hivemind_access"]
            self.username = tok["username"]
            self._token = AccessToken(tok["username"], base64.b64decode(tok["peer_public_key"]), float(tok["expiration_time"]),
                                      base64.b64decode(tok["signature"]))
            self.coordinator_ip, self.coordinator_port = resp.get("coordinator_ip"), resp.get("coordinator_port")
            from dalle_amd.parallel.crypto import RSAPublicKey

            self._authority_public_key = RSAPublicKey.from_bytes(base64.b64decode(resp["auth_server_public_key"]))
        else:
            if self.authority is None:
                self.authority = LocalAuthority()
            self.username = self.hf_user_access_token.split(":")[0] if ":" in self.hf_user_access_token else getpass.getuser()
            self._token = self.authority.issue(self.username, self.local_public_key)
            self._authority_public_key = self.authority.public_key
        logger.info(f"Access for user {self.username} has been granted until {time.ctime(self._token.expiration_time)}")

    def is_token_valid(self, tok: AccessToken) -> bool:
        if self._authority_public_key is None:
            self.get_token()
        return verify_access_token(tok, self._authority_public_key)

    def does_token_need_refreshing(self, tok: AccessToken) -> bool:
        return tok.expiration_time - time.time() < self._AUTHORITY_REFRESH


def authorize_with_huggingface() -> HuggingFaceAuthorizer:
    while True:
        organization_name = os.getenv("HF_ORGANIZATION_NAME") or input("HuggingFace organization name: ")
        model_name = os.getenv("HF_MODEL_NAME") or input("HuggingFace model name: ")
        hf_user_access_token = os.getenv("HF_USER_ACCESS_TOKEN") or getpass.getpass("HuggingFace access token: ")
        authorizer = HuggingFaceAuthorizer(organization_name, model_name, hf_user_access_token)
        try:
            authorizer.join_experiment()
            return authorizer
        except Exception as e:  # noqa: BLE001
            logger.error(f"Authorization failed: {e!r}")
            if os.getenv("HF_USER_ACCESS_TOKEN"):
                raise
