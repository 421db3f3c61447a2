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
