"""The reference's multi-process CLI (distributed.py:14-20, :156-184: ``--mode
slave`` and ``--mode master`` in separate processes talking through RabbitMQ) over
the socket broker (broker.SocketBroker): the broker runs in this process, master and
slave are separate Python processes.  CPU tests: the nodes' arithmetic is the
float64 oracle (tests/socket_node.py --oracle), so these pin the transport and the
protocol against the golden run of the reference itself
(tests/golden/spiked_d128_k2_m5_ragged.npz: arrival order, JSON schema, results)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from distributed_eigenspaces_amd import broker as br
from oracle import ref_cpu
from tests.conftest import ROOT, load_golden

NODE = os.path.join(ROOT, "tests", "socket_node.py")


def _run_pair(tmp_path, golden, extra, timeout=120, nslaves=1):
    g = load_golden(golden)
    path = os.path.join(tmp_path, "X.npy")
    np.save(path, g["X"])
    b = br.SocketBroker("127.0.0.1", 0).start()
    out = os.path.join(tmp_path, "master.npz")
    env = dict(os.environ, PYTHONPATH=ROOT)
    slaves = [subprocess.Popen([sys.executable, NODE, "slave", b.address, path] + extra, env=env)
              for _ in range(nslaves)]
    try:
        rc = subprocess.run([sys.executable, NODE, "master", b.address, path, str(int(g["k"])),
                             str(int(g["m"])), out] + extra, env=env, timeout=timeout).returncode
        assert rc == 0
    finally:
        b.shutdown()
        for s in slaves:
            try:
                s.wait(timeout=30)
            except subprocess.TimeoutExpired:
                s.kill()
    return g, np.load(out), b


def test_two_process_protocol_matches_reference_run(tmp_path):
    g, r, b = _run_pair(tmp_path, "spiked_d128_k2_m5_ragged", ["--oracle"])
    # arrival order at the master == the reference's (LIFO dispatch, FIFO slave)
    np.testing.assert_array_equal(r["ranges"], g["ranges"])
    for i in range(len(g["ranges"])):
        assert ref_cpu.projector_distance(r["worker_V"][i], g["worker_V"][i]) <= 1e-6  # projector_distance floor: sqrt of float64 rounding
    assert ref_cpu.projector_distance(r["server_V"], g["server_V"]) <= 1e-6  # projector_distance floor: sqrt of float64 rounding
    np.testing.assert_allclose(r["server_evals"], g["server_evals"], rtol=1e-12)
    # request schema on the wire: {"rank": k, "batch": [lo, hi]}
    import json
    reqs = [json.loads(body) for q, body in b.delivered if q == "slaves"]
    assert all(set(x) == {"rank", "batch"} and x["rank"] == int(g["k"]) for x in reqs)
    np.testing.assert_array_equal([x["batch"] for x in reqs], g["request_ranges"])


def test_competing_slave_processes(tmp_path):
    """Three slave processes on one queue (RabbitMQ round-robin): every shard once."""
    g, r, _ = _run_pair(tmp_path, "spiked_d64_k4_m8", ["--oracle"], nslaves=3)
    assert sorted(map(tuple, r["ranges"])) == sorted(map(tuple, g["ranges"]))
    by = {tuple(x): i for i, x in enumerate(g["ranges"])}
    for rg, V in zip(r["ranges"], r["worker_V"]):
        assert ref_cpu.projector_distance(V, g["worker_V"][by[tuple(rg)]]) <= 1e-6  # projector_distance floor: sqrt of float64 rounding
    assert ref_cpu.projector_distance(r["server_V"], g["server_V"]) <= 1e-6  # projector_distance floor: sqrt of float64 rounding


def test_unacked_messages_are_requeued():
    """A consumer that disconnects before acking: its message goes to the next one."""
    b = br.SocketBroker("127.0.0.1", 0).start()
    try:
        c1 = br.connect(b.address).channel()
        c1.queue_declare("q")
        got = []
        c1.basic_consume("q", lambda ch, m, p, body: got.append(body))
        pub = br.connect(b.address).channel()
        pub.basic_publish("", "q", "hello")
        msg = br._recv(c1.conn.sock)  # delivered, never acked
        assert msg["body"] == "hello"
        c1.conn.close()
        c2 = br.connect(b.address).channel()
        seen = []

        def cb(ch, m, p, body):
            seen.append(body.decode())
            ch.basic_ack(m.delivery_tag)
            ch.stop_consuming()
        c2.basic_consume("q", cb)
        c2.start_consuming()
        assert seen == ["hello"]
    finally:
        b.shutdown()


def test_address_parsing():
    assert br.parse_address("tcp://127.0.0.1:5000") == ("127.0.0.1", 5000)
    assert br.parse_address("tcp://rabbit") == ("rabbit", 5672)
    assert br.parse_address("localhost:5673") == ("localhost", 5673)
    assert br.parse_address("inproc-name") is None


def test_cli_bare_broker_host_is_the_socket_broker():
    """The reference's CLI form ``--broker localhost`` (a RabbitMQ host name,
    distributed.py:16, :158): in master / slave mode it means the socket broker on
    that host at pika's port 5672 - an in-process broker per process would never
    connect the two."""
    import socket

    from distributed_eigenspaces_amd import distributed as dd
    assert dd.cli_broker("localhost", "slave") == "tcp://localhost:5672"
    assert dd.cli_broker("10.0.0.7", "master") == "tcp://10.0.0.7:5672"
    assert dd.cli_broker("tcp://h:1234", "master") == "tcp://h:1234"
    assert dd.cli_broker("h:1234", "slave") == "h:1234"
    assert dd.cli_broker("inproc-x", "local") == "inproc-x"
    try:
        b = br.SocketBroker("127.0.0.1", 5672).start()
    except OSError:
        pytest.skip("port 5672 busy")
    try:
        pub = br.connect(dd.cli_broker("127.0.0.1", "master")).channel()
        sub = br.connect(dd.cli_broker("127.0.0.1", "slave")).channel()
        sub.queue_declare("slaves")
        seen = []

        def cb(ch, m, p, body):
            seen.append(body.decode())
            ch.basic_ack(m.delivery_tag)
            ch.stop_consuming()
        sub.basic_consume("slaves", cb)
        pub.basic_publish("", "slaves", '{"rank": 2, "batch": [0, 10]}')
        sub.start_consuming()
        assert seen == ['{"rank": 2, "batch": [0, 10]}']
    finally:
        b.shutdown()
    del socket


def test_slow_consumer_does_not_block_the_broker():
    """A consumer that never reads its deliveries (large bodies fill its socket
    buffers) must not stall other connections: deliveries are written by per-client
    sender threads, outside the broker lock."""
    b = br.SocketBroker("127.0.0.1", 0).start()
    try:
        stuck = br.connect(b.address).channel()
        stuck.basic_consume("big", lambda *a: None)  # never reads
        pub = br.connect(b.address).channel()
        body = "x" * (4 << 20)
        for _ in range(8):  # 32 MB queued towards the stuck consumer
            pub.basic_publish("", "big", body)
        other = br.connect(b.address).channel()
        seen = []

        def cb(ch, m, p, bd):
            seen.append(bd.decode())
            ch.basic_ack(m.delivery_tag)
            ch.stop_consuming()
        other.basic_consume("small", cb)
        pub.basic_publish("", "small", "ping")
        import threading
        t = threading.Thread(target=other.start_consuming, daemon=True)
        t.start()
        t.join(timeout=20)
        assert seen == ["ping"]
    finally:
        b.shutdown()
