"""The metrics / snapshot store (``dalle_amd/parallel/dht.py``): losing the hosting peer degrades the
clients to no-op answers instead of raising into the training loop, and they reconnect when a host
is back on the same address (the rank-0-hosted store must not be fatal)."""
import time

from dalle_amd.parallel.dht import DHT, get_dht_time


def test_client_survives_lost_host_and_reconnects():
    host = DHT(host_maddrs=["/ip4/127.0.0.1/tcp/0"])
    port = host._addr[1]
    client = DHT(initial_peers=[f"/ip4/127.0.0.1/tcp/{port}"], connect_timeout=5.0)
    client.reconnect_period = 0.0
    assert client.store("k", {"a": 1}, get_dht_time() + 60, subkey="s")
    assert client.get("k").value[b"s"].value == {"a": 1}

    host.shutdown()  # the hosting peer dies
    time.sleep(0.2)
    assert client.store("k", {"a": 2}, get_dht_time() + 60, subkey="s") is False
    assert client.degraded
    assert client.get("k") is None and client.keys() == [] and client.wait_for("k", 1, 0.1) == 0

    host2 = DHT(host_maddrs=[f"/ip4/127.0.0.1/tcp/{port}"])  # a restarted host re-binds the port
    try:
        assert client.store("k", {"a": 3}, get_dht_time() + 60, subkey="s")
        assert not client.degraded
        assert host2.get("k").value[b"s"].value == {"a": 3}
    finally:
        host2.shutdown()


def test_metrics_outlive_a_killed_rank0(tmp_path):
    """Default torchrun path (dalle_amd/parallel/dht_host.py): rank 0 starts the store as a process of its
    own, watched against the torchrun agent -- a SIGKILLed rank 0 no longer takes the metrics with it, the
    auxiliary peer still reads ``{prefix}_metrics`` (reference run_aux_peer.py:107), and the store exits
    with the agent."""
    import os
    import signal
    import socket
    import subprocess
    import sys

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    agent = subprocess.Popen(["sleep", "300"])  # stands in for the torchrun agent
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port - 1), WORLD_SIZE="2", RANK="0",
               DALLE_AMD_DHT_WATCH_PID=str(agent.pid))
    env.pop("DALLE_AMD_DHT_HOST", None)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import time; from dalle_amd.parallel.dht import DHT, get_dht_time; "
            "from dalle_amd.parallel.dht_host import torchrun_endpoints; "
            "peers, hm = torchrun_endpoints(0); d = DHT(initial_peers=peers); "
            "assert d.store('run_metrics', {'loss': 1.5}, get_dht_time() + 600, subkey='rank0'); "
            "print('stored', flush=True); time.sleep(600)")
    rank0 = subprocess.Popen([sys.executable, "-c", code], env=env, cwd=root, stdout=subprocess.PIPE, text=True)
    try:
        assert rank0.stdout.readline().strip() == "stored"
        rank0.send_signal(signal.SIGKILL)  # rank 0 dies
        rank0.wait(10)
        maddr = f"/ip4/127.0.0.1/tcp/{port}"
        rank1 = DHT(initial_peers=[maddr], connect_timeout=5.0)
        assert rank1.store("run_metrics", {"loss": 2.5}, get_dht_time() + 600, subkey="rank1")
        aux = DHT(initial_peers=[maddr], connect_timeout=5.0)
        got = aux.get("run_metrics").value
        assert {k: v.value["loss"] for k, v in got.items()} == {b"rank0": 1.5, b"rank1": 2.5}
        assert not aux.degraded
    finally:
        if rank0.poll() is None:
            rank0.kill()
        agent.kill()
        agent.wait()
    # the store follows the agent out
    aux.reconnect_period = 0.0
    deadline = time.time() + 15
    while time.time() < deadline and aux.get("run_metrics") is not None:
        time.sleep(0.5)
    assert aux.get("run_metrics") is None and aux.degraded
