"""Local swarm manager: the single-node counterpart of the reference's Azure scale-set manager
(``manage_scaleset.py``).

The reference provisions a spot-VM scale set where every VM runs one training peer (cloud-init: env +
``run_trainer.py`` pointed at the initial peers) plus a coordinator VM running ``run_aux_peer.py``;
spot evictions deallocate VMs and the scale set brings them back. On an MI355X node the same fleet is
processes: one aux peer hosting the key-value store (the DHT replacement) and the elastic coordinator,
and one trainer peer per GPU (``HIP_VISIBLE_DEVICES`` pinned), each an independent process that forms
its RCCL/gloo communicator through the coordinator (``dalle_amd.parallel.elastic``). The supervisor
restarts peers that die -- the analogue of the scale set re-allocating an evicted spot VM -- and the
``--chaos`` option evicts a random trainer periodically to exercise the recovery path.

CLI::

    python -m dalle_amd.utils.swarm up --trainers 8 --log-dir swarm_logs -- --model_preset bench24 ...
    python -m dalle_amd.utils.swarm status --log-dir swarm_logs
    python -m dalle_amd.utils.swarm down --log-dir swarm_logs
"""
from __future__ import annotations

import argparse
import json
import os
import random
import signal
import socket
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@dataclass
class Peer:
    name: str
    cmd: List[str]
    env: Dict[str, str]
    log_path: str
    proc: Optional[subprocess.Popen] = None
    restarts: int = 0
    log_file: Optional[object] = None

    def start(self):
        self.log_file = open(self.log_path, "ab")
        self.proc = subprocess.Popen(self.cmd, env=self.env, stdout=self.log_file, stderr=subprocess.STDOUT,
                                     start_new_session=True, cwd=ROOT)

    def alive(self) -> bool:
        return self.proc is not None and self.proc.poll() is None

    def stop(self, sig=signal.SIGTERM, wait: float = 10.0):
        if self.proc is None:
            return
        if self.proc.poll() is None:
            try:
                os.killpg(self.proc.pid, sig)  # the peer's own process group (start_new_session)
            except ProcessLookupError:
                pass
            try:
                self.proc.wait(wait)
            except subprocess.TimeoutExpired:
                os.killpg(self.proc.pid, signal.SIGKILL)
                self.proc.wait(wait)
        if self.log_file is not None:
            self.log_file.close()
            self.log_file = None


@dataclass
class LocalSwarm:
    num_trainers: int
    peer_args: List[str] = field(default_factory=list)
    trainer_args: List[str] = field(default_factory=list)
    aux_args: List[str] = field(default_factory=list)
    log_dir: str = "swarm_logs"
    devices: Optional[List[int]] = None  # GPU per trainer (None: CPU peers)
    dht_port: int = 0
    coordinator_port: int = 0
    peers: List[Peer] = field(default_factory=list)

    def __post_init__(self):
        os.makedirs(self.log_dir, exist_ok=True)
        self.dht_port = self.dht_port or free_port()
        self.coordinator_port = self.coordinator_port or free_port()

    # -- fleet definition ------------------------------------------------------------------------------
    def _env(self, device: Optional[int]) -> Dict[str, str]:
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
            env.pop(k, None)  # each peer is its own job; the communicator comes from the coordinator
        if device is not None:
            env["HIP_VISIBLE_DEVICES"] = str(device)
        return env

    def aux_peer(self) -> Peer:
        cmd = [sys.executable, os.path.join(ROOT, "run_aux_peer.py"), *self.peer_args,
               "--host_maddrs", f"/ip4/127.0.0.1/tcp/{self.dht_port}",
               "--elastic_coordinator", f"127.0.0.1:{self.coordinator_port}", "--host_elastic_coordinator", "True",
               *self.aux_args]
        if "--local_path" not in self.aux_args:  # checkpoints next to the logs, not in the source tree
            cmd += ["--local_path", os.path.join(self.log_dir, "Repo")]
        return Peer("aux", cmd, self._env(None), os.path.join(self.log_dir, "aux.log"))

    def trainer(self, i: int) -> Peer:
        dev = self.devices[i % len(self.devices)] if self.devices else None
        cmd = [sys.executable, os.path.join(ROOT, "run_trainer.py"), *self.peer_args,
               "--initial_peers", f"/ip4/127.0.0.1/tcp/{self.dht_port}",
               "--elastic_coordinator", f"127.0.0.1:{self.coordinator_port}", *self.trainer_args]
        return Peer(f"trainer{i}", cmd, self._env(dev), os.path.join(self.log_dir, f"trainer{i}.log"))

    # -- lifecycle -------------------------------------------------------------------------------------
    def up(self, aux_startup: float = 3.0):
        aux = self.aux_peer()
        aux.start()
        self.peers = [aux]
        time.sleep(aux_startup)  # the key-value store and the coordinator must be listening first
        for i in range(self.num_trainers):
            p = self.trainer(i)
            p.start()
            self.peers.append(p)
        self._write_state()

    def status(self) -> Dict[str, dict]:
        return {p.name: {"pid": p.proc.pid if p.proc else None, "alive": p.alive(), "restarts": p.restarts,
                         "returncode": None if p.alive() or p.proc is None else p.proc.returncode} for p in self.peers}

    def supervise(self, duration: float, poll: float = 1.0, restart: bool = True, chaos_interval: Optional[float] = None,
                  seed: int = 0, on_event=None):
        """Restart dead trainers (spot re-allocation); optionally evict a random trainer every
        ``chaos_interval`` seconds. Returns the list of events."""
        rng = random.Random(seed)
        events = []
        t0 = last_chaos = time.time()
        while time.time() - t0 < duration:
            time.sleep(poll)
            now = time.time()
            if chaos_interval and now - last_chaos >= chaos_interval:
                victims = [p for p in self.peers[1:] if p.alive()]
                if victims:
                    v = rng.choice(victims)
                    v.stop(signal.SIGKILL)
                    events.append({"t": now - t0, "event": "evict", "peer": v.name})
                    if on_event:
                        on_event(events[-1])
                last_chaos = now
            for p in self.peers[1:]:
                if not p.alive() and restart:
                    rc = p.proc.returncode if p.proc else None
                    if rc == 0:
                        continue  # finished its max_steps: not a failure
                    p.stop()
                    p.restarts += 1
                    p.start()
                    events.append({"t": now - t0, "event": "restart", "peer": p.name, "returncode": rc})
                    if on_event:
                        on_event(events[-1])
            self._write_state()
        return events

    def down(self):
        for p in reversed(self.peers):
            p.stop()
        self._write_state()

    def _write_state(self):
        with open(os.path.join(self.log_dir, "swarm.json"), "w") as f:
            json.dump({"dht_port": self.dht_port, "coordinator_port": self.coordinator_port, "peers": self.status()}, f,
                      indent=1)


def _cli(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("action", choices=["up", "status", "down"])
    ap.add_argument("--trainers", type=int, default=2)
    ap.add_argument("--gpus", type=str, default="", help="comma-separated GPU ids, one per trainer (default: CPU)")
    ap.add_argument("--log-dir", default="swarm_logs")
    ap.add_argument("--duration", type=float, default=3600.0, help="supervise for this long, then tear down")
    ap.add_argument("--chaos", type=float, default=0.0, help="evict a random trainer every N seconds")
    ap.add_argument("rest", nargs=argparse.REMAINDER, help="-- then arguments for every peer")
    a = ap.parse_args(argv)
    state_file = os.path.join(a.log_dir, "swarm.json")
    if a.action == "status":
        print(open(state_file).read() if os.path.exists(state_file) else "no swarm")
        return 0
    if a.action == "down":
        if os.path.exists(state_file):
            for name, st in json.load(open(state_file))["peers"].items():
                if st.get("alive") and st.get("pid"):
                    try:
                        os.killpg(st["pid"], signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        return 0
    rest = a.rest[1:] if a.rest[:1] == ["--"] else a.rest
    sw = LocalSwarm(a.trainers, peer_args=rest, log_dir=a.log_dir,
                    devices=[int(x) for x in a.gpus.split(",")] if a.gpus else None)
    sw.up()
    try:
        sw.supervise(a.duration, chaos_interval=a.chaos or None, on_event=lambda ev: print(json.dumps(ev), flush=True))
    finally:
        sw.down()
    return 0


if __name__ == "__main__":
    sys.exit(_cli())
