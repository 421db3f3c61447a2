"""Peer authorisation (reference ``huggingface_auth.py:1-193``).

The reference asks a Hugging Face-hosted authority (``PUT {auth}/api/experiments/join`` with the
user's HF token) for an authority-signed access token (username, peer public key, expiry), retried
with exponential backoff, refreshed one minute before expiry, and validated by signature + expiry.

Same protocol here, with two authorities:
* a remote one when ``DALLE_AMD_AUTH_SERVER`` is set (HTTPS via ``requests``);
* an offline local authority (HMAC-SHA256 with a shared secret from ``DALLE_AMD_AUTH_SECRET``) so
  the peers of one node can still issue / verify tokens without network access.
"""
import base64
import getpass
import hashlib
import hmac
import json
import os
import time
from dataclasses import dataclass
from typing import Optional

from dalle_amd.utils.logging import get_logger

logger = get_logger(__name__)


def call_with_retries(func, n_retries: int = 10, initial_delay: float = 1.0):
    for i in range(n_retries):
        try:
            return func()
        except Exception as e:  # noqa: BLE001
            if i == n_retries - 1:
                raise
            delay = initial_delay * (2 ** i)
            logger.warning(f"Failed to call `{getattr(func, '__name__', func)}` with exception: {e!r}. Retrying in {delay:.1f} sec")
            time.sleep(delay)


@dataclass
class AccessToken:
    username: str
    public_key: bytes
    expiration_time: float
    signature: bytes = b""

    def payload(self) -> bytes:
        return json.dumps([self.username, base64.b64encode(self.public_key).decode(), self.expiration_time]).encode()


class LocalAuthority:
    def __init__(self, secret: Optional[bytes] = None):
        self.secret = secret or os.environ.get("DALLE_AMD_AUTH_SECRET", "dalle-amd-local").encode()

    def issue(self, username: str, public_key: bytes, lifetime: float = 3600.0) -> AccessToken:
        tok = AccessToken(username, public_key, time.time() + lifetime)
        tok.signature = hmac.new(self.secret, tok.payload(), hashlib.sha256).digest()
        return tok

    def verify(self, tok: AccessToken) -> bool:
        good = hmac.new(self.secret, tok.payload(), hashlib.sha256).digest()
        return hmac.compare_digest(good, tok.signature) and tok.expiration_time > time.time()


class HuggingFaceAuthorizer:
    _AUTHORITY_REFRESH = 60.0  # refresh one minute before expiry (huggingface_auth.py)

    def __init__(self, organization_name: str, model_name: str, hf_user_access_token: str, local_public_key: bytes = b"",
                 authority: Optional[LocalAuthority] = None):
        self.organization_name, self.model_name = organization_name, model_name
        self.hf_user_access_token = hf_user_access_token
        self.local_public_key = local_public_key
        self.authority = authority or LocalAuthority()
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
        else:
            self.username = self.hf_user_access_token.split(":")[0] if ":" in self.hf_user_access_token else getpass.getuser()
            self._token = self.authority.issue(self.username, self.local_public_key)
        logger.info(f"Access for user {self.username} has been granted until {time.ctime(self._token.expiration_time)}")

    def is_token_valid(self, tok: AccessToken) -> bool:
        return self.authority.verify(tok)

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
