"""The metrics key/value store as a process of its own (round-4 review item 5; reference run_aux_peer.py:107).

On the default torchrun path the store used to live inside the rank-0 trainer, so the auxiliary peer's
view of ``{prefix}_metrics`` went dark for the rest of the run once rank 0 died, although the other
trainers kept training. Here rank 0 only *spawns* the store: a detached child process (own session, so the
torchrun agent's teardown of a dead worker does not take it along) that serves the native
``dalle_amd._kvstore`` server and exits when the process it watches -- the torchrun agent, which outlives
every worker -- is gone. A restarted rank 0 finds the port taken and simply connects.

    python -m dalle_amd.parallel.dht_host --host 127.0.0.1 --port 29501 --watch-pid <agent pid>
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import time
from typing import Optional


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    return True


def _reachable(host: str, port: int, timeout: float) -> bool:
    from .dht import _load_kv

    try:
        c = _load_kv().KVClient(host, port, timeout)
        return bool(c.ping())
    except RuntimeError:
        return False


def spawn_host(host: str, port: int, watch_pid: Optional[int] = None, timeout: float = 30.0,
               log_path: Optional[str] = None) -> Optional[subprocess.Popen]:
    """Start the store process (unless one already answers on ``host:port``) and wait until it serves.
    Returns the Popen handle of a process this call started, None when a running one was found."""
    connect = "127.0.0.1" if host in ("0.0.0.0", "localhost") else host
    if _reachable(connect, port, 1.0):
        return None
    watch = int(watch_pid if watch_pid is not None else os.getpid())
    out = open(log_path, "ab") if log_path else subprocess.DEVNULL
    proc = subprocess.Popen([sys.executable, "-m", "dalle_amd.parallel.dht_host", "--host", host, "--port", str(port),
                             "--watch-pid", str(watch)], stdin=subprocess.DEVNULL, stdout=out, stderr=out,
                            start_new_session=True, close_fds=True,
                            env={**os.environ, "PYTHONPATH": os.pathsep.join(p for p in sys.path if p)})
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if _reachable(connect, port, 1.0):
            return proc
        if proc.poll() is not None:  # lost a bind race to another host process: use that one
            if _reachable(connect, port, 2.0):
                return None
            raise RuntimeError(f"DHT host process exited with {proc.returncode} before serving {host}:{port}")
        time.sleep(0.05)
    proc.kill()
    raise RuntimeError(f"DHT host process did not serve {host}:{port} within {timeout:.0f}s")


def default_watch_pid() -> int:
    """``DALLE_AMD_DHT_WATCH_PID``, else the torchrun agent (the workers' parent: it outlives every worker)
    under torchrun, else this process."""
    if os.environ.get("DALLE_AMD_DHT_WATCH_PID"):
        return int(os.environ["DALLE_AMD_DHT_WATCH_PID"])
    return os.getppid() if os.environ.get("TORCHELASTIC_RUN_ID") else os.getpid()


def torchrun_endpoints(rank: int):
    """(initial_peers, host_maddrs) of a torchrun worker with no external store: the store serves next to
    the rendezvous port (MASTER_PORT + 1). By default rank 0 starts it as a process of its own and every rank,
    rank 0 included, is its client; DALLE_AMD_DHT_HOST=inproc has rank 0 serve it from a thread instead."""
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    addr = addr if addr != "localhost" else "127.0.0.1"
    port = int(os.environ.get("MASTER_PORT", "29500")) + 1
    maddr = f"/ip4/{addr}/tcp/{port}"
    if os.environ.get("DALLE_AMD_DHT_HOST", "process") == "inproc":
        return ([], [maddr]) if rank == 0 else ([maddr], [])
    if rank == 0:
        spawn_host(addr, port, watch_pid=default_watch_pid())
    return [maddr], []


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--watch-pid", type=int, required=True)
    ap.add_argument("--poll", type=float, default=0.5)
    a = ap.parse_args(argv)
    from .dht import _load_kv

    try:
        server = _load_kv().KVServer(a.host, a.port)
    except RuntimeError as e:  # port taken: another host process serves it
        print(f"dht_host: {e}", flush=True)
        return 1
    print(f"dht_host: serving {a.host}:{server.port}, watching pid {a.watch_pid}", flush=True)
    try:
        while _alive(a.watch_pid):
            time.sleep(a.poll)
    finally:
        server.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
