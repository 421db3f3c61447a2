"""DHT facade over the native key/value store (``dalle_amd._kvstore``, csrc/store/kvstore.cpp).

Replaces ``hivemind.DHT`` + the Go libp2p daemon for a single node. The API the
reference consumes is kept (``task.py:104-119``, ``callback.py:80-86``, ``run_aux_peer.py:107``):

* ``DHT(start, initial_peers, client_mode, host_maddrs, announce_maddrs, use_ipfs,
  record_validators, identity_path, authorizer)``
* ``store(key, subkey, value, expiration_time, return_future=False)``
* ``get(key, latest=True) -> ValueWithExpiration(value={subkey: ValueWithExpiration(value, exp)})``
* ``peer_id``, ``get_visible_maddrs()``, ``shutdown()``

The first peer (no ``initial_peers``) hosts the store inside its own process (a native server
thread); everybody else connects to a multiaddr such as ``/ip4/127.0.0.1/tcp/31337``. Values are
msgpack-serialised; record validators run on every store (schema + owner-signed subkeys).

Losing the hosting peer is not fatal to a client: the store only carries metrics and auxiliary-peer
snapshots (training progress and recovery use the torchrun agent's c10d store), so once the native
client's own reconnect attempt fails, ``store`` returns False, ``get`` None, ``keys`` [] and
``wait_for`` 0, ``degraded`` is set, and every ``reconnect_period`` seconds the next call tries the
address again (a restarted host peer re-binds the same port).
"""
from __future__ import annotations

import concurrent.futures
import os
import re
import secrets
import socket
import time
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence

import msgpack

from ..utils.logging import get_logger

logger = get_logger(__name__)

_MADDR = re.compile(r"^/ip4/(?P<host>[0-9.]+)/tcp/(?P<port>\d+)(?:/p2p/(?P<peer>[A-Za-z0-9]+))?$")


def get_dht_time() -> float:
    """Wall-clock used for record expirations (``hivemind.get_dht_time``)."""
    return time.time()


@dataclass
class ValueWithExpiration:
    value: Any
    expiration_time: float

    def __iter__(self):
        return iter((self.value, self.expiration_time))


def parse_maddr(maddr: str):
    m = _MADDR.match(str(maddr).strip())
    if not m:
        raise ValueError(f"unsupported multiaddr {maddr!r}; expected /ip4/<host>/tcp/<port>[/p2p/<id>]")
    return m.group("host"), int(m.group("port")), m.group("peer")


def _load_kv():
    from ..ops.ext import load_extension  # noqa: F401  (torch loaded first for the shared libs)
    import importlib

    return importlib.import_module("dalle_amd._kvstore")


class DHT:
    def __init__(self, start: bool = True, initial_peers: Sequence[str] = (), client_mode: bool = False,
                 host_maddrs: Sequence[str] = ("/ip4/127.0.0.1/tcp/0",), announce_maddrs: Sequence[str] = (),
                 use_ipfs: bool = False, record_validators: Sequence[Any] = (), identity_path: Optional[str] = None,
                 authorizer: Any = None, connect_timeout: float = 30.0, **kwargs):
        self.client_mode = client_mode
        self.record_validators = list(record_validators)
        self.authorizer = authorizer
        self.use_ipfs = use_ipfs
        self.announce_maddrs = list(announce_maddrs)
        self.peer_id = self._load_identity(identity_path)
        self._server = None
        self._client = None
        self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=2, thread_name_prefix="dht")
        self._host_maddrs = list(host_maddrs)
        self._initial_peers = list(initial_peers)
        self._connect_timeout = connect_timeout
        self.owner = bytes(self.peer_id, "utf8")
        self.degraded = False        # the hosting peer is unreachable (client side only)
        self.reconnect_period = 10.0
        self._next_reconnect = 0.0
        for v in self.record_validators:
            if hasattr(v, "local_public_key"):
                self.owner = v.local_public_key
        if start:
            self.run_in_background()

    @staticmethod
    def _load_identity(path: Optional[str]) -> str:
        if path is None:
            return "Qm" + secrets.token_hex(16)
        if os.path.exists(path):
            with open(path) as f:
                return f.read().strip()
        ident = "Qm" + secrets.token_hex(16)
        with open(path, "w") as f:
            f.write(ident)
        return ident

    # ------------------------------------------------------------------------------------------
    def run_in_background(self, await_ready: bool = True):
        kv = _load_kv()
        if self._initial_peers:
            last_err = None
            for maddr in self._initial_peers:
                host, port, _ = parse_maddr(maddr)
                try:
                    self._client = kv.KVClient(host, port, self._connect_timeout)
                    self._addr = (host, port)
                    break
                except RuntimeError as e:  # try the next bootstrap peer
                    last_err = e
            if self._client is None:
                raise RuntimeError(f"could not reach any initial peer {self._initial_peers}: {last_err}")
        else:
            if self.client_mode:
                raise ValueError("a client-mode peer needs initial_peers to connect to")
            host, port, _ = parse_maddr(self._host_maddrs[0] if self._host_maddrs else "/ip4/127.0.0.1/tcp/0")
            bind = host
            self._server = kv.KVServer(bind, port)
            connect_host = "127.0.0.1" if host == "0.0.0.0" else host
            self._addr = (connect_host, self._server.port)
            self._client = kv.KVClient(connect_host, self._server.port, self._connect_timeout)
        return self

    def is_alive(self) -> bool:
        try:
            return bool(self._client and self._client.ping())
        except RuntimeError:
            return False

    def get_visible_maddrs(self, latest: bool = False) -> List[str]:
        host, port = self._addr
        if host in ("0.0.0.0", "127.0.0.1") and self.announce_maddrs:
            return list(self.announce_maddrs)
        return [f"/ip4/{host}/tcp/{port}/p2p/{self.peer_id}"]

    # ------------------------------------------------------------------------------------------
    def _validate(self, key: str, subkey, value) -> bool:
        for v in self.record_validators:
            if hasattr(v, "validate") and not v.validate(key, subkey, value):
                return False
        return True

    def _call(self, op: str, *args, default=None):
        """One native client call; a lost hosting peer degrades a CLIENT to no-op answers (module doc)."""
        if self.degraded and self._server is None:
            now = time.monotonic()
            if now < self._next_reconnect:
                return default
            self._next_reconnect = now + self.reconnect_period
        try:
            out = getattr(self._client, op)(*args)
        except RuntimeError as e:
            if self._server is not None:  # our own in-process server: a real error
                raise
            if not self.degraded:
                logger.warning(f"DHT host {self._addr[0]}:{self._addr[1]} unreachable ({e}); metrics / snapshot "
                               f"records are dropped until it is back (retry every {self.reconnect_period:.0f}s)")
            self.degraded = True
            self._next_reconnect = time.monotonic() + self.reconnect_period
            return default
        if self.degraded:
            logger.info("DHT host reachable again")
            self.degraded = False
        return out

    def _store(self, key, subkey, value, expiration_time) -> bool:
        if not self._validate(key, subkey, value):
            logger.warning(f"record for key {key!r} rejected by validators")
            return False
        sub = b"" if subkey is None else (subkey if isinstance(subkey, bytes) else str(subkey).encode())
        payload = msgpack.packb(value, use_bin_type=True)
        for v in self.record_validators:  # owner-protected records get signed (RSASignatureValidator)
            if hasattr(v, "sign_value"):
                payload = v.sign_value(str(key), subkey, payload, float(expiration_time))
        owner = self.owner if subkey is not None else b""
        return bool(self._call("store", str(key), sub, payload, float(expiration_time), owner, default=False))

    def _decode(self, key: str, sub, payload: bytes, exp: float):
        """Signature check + strip of one stored record; None when a validator rejects it."""
        for v in self.record_validators:
            if hasattr(v, "validate_signed"):
                if not v.validate_signed(key, None if sub == b"" else sub, payload, exp):
                    logger.warning(f"dropping record {key!r}/{sub[:24]!r}: bad or missing owner signature")
                    return None
                payload = v.strip_value(payload)
        return msgpack.unpackb(payload, raw=False)

    def store(self, key: str, value: Any, expiration_time: float, subkey: Any = None, return_future: bool = False, **kw):
        if return_future:
            return self._pool.submit(self._store, key, subkey, value, expiration_time)
        return self._store(key, subkey, value, expiration_time)

    def get(self, key: str, latest: bool = True, return_future: bool = False, **kw) -> Optional[ValueWithExpiration]:
        if return_future:
            return self._pool.submit(self.get, key, latest)
        items = self._call("get", str(key), default=None)
        if not items:
            return None
        key = str(key)
        if len(items) == 1 and items[0][0] == b"":
            _, payload, exp = items[0]
            val = self._decode(key, b"", payload, exp)
            return None if val is None else ValueWithExpiration(val, exp)
        out: Dict[Any, ValueWithExpiration] = {}
        best = 0.0
        for sub, payload, exp in items:
            val = self._decode(key, sub, payload, exp)
            if val is None:
                continue
            out[sub] = ValueWithExpiration(val, exp)
            best = max(best, exp)
        return ValueWithExpiration(out, best) if out else None

    def delete(self, key: str):
        self._call("delete", str(key))

    def keys(self, prefix: str = "") -> List[str]:
        return list(self._call("keys", prefix, default=[]))

    def wait_for(self, key: str, count: int, timeout: float) -> int:
        """Block until ``key`` has ``count`` live subkeys (server-side wait); returns the live count."""
        return int(self._call("wait", str(key), int(count), float(timeout), default=0))

    def shutdown(self):
        self._pool.shutdown(wait=False)
        if self._server is not None:
            self._server.stop()
            self._server = None

    def __del__(self):
        try:
            self.shutdown()
        except Exception:
            pass


def choose_ip_address(maddrs, prefer_global: bool = True) -> str:
    """Pick an IPv4 address from multiaddrs (``hivemind.choose_ip_address``)."""
    hosts = []
    for m in maddrs:
        try:
            hosts.append(parse_maddr(str(m))[0])
        except ValueError:
            continue
    for h in hosts:
        if h not in ("127.0.0.1", "0.0.0.0"):
            return h
    if hosts:
        return hosts[0]
    return socket.gethostbyname("localhost")
