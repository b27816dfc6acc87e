"""Master/slave protocol of the drop-in distributed.py over the in-process broker.

CPU-only: the worker / server arithmetic is replaced by a deterministic fake so the
test covers only the message flow (shard split, LIFO dispatch, window of 5, JSON
schema, completion).  The same protocol with the real GPU path is in
tests/test_gpu_pipeline.py."""
import json

import numpy as np
import pytest
import torch

from distributed_eigenspaces_amd import broker as br
from distributed_eigenspaces_amd import distributed as dd
from distributed_eigenspaces_amd.my_threading import Slave
from tests.conftest import load_golden


class FakeSlave(dd.SlaveNode):
    def _device_rows(self, lo, hi):
        return torch.as_tensor(self.data[lo:hi])

    def compute_sigma_hat_(self, x):
        return x  # pass the rows through; the fake basis encodes the shard

    def top_k_eigenvectors(self, matrix, k):
        d = matrix.shape[1]
        V = torch.zeros((d, k), dtype=torch.float64)
        V[0, 0] = float(matrix.shape[0])  # rows in the shard
        V[1, 0] = float(matrix[0, 0])     # first value of the shard
        return V


class FakeMaster(dd.MasterNode):
    def server_solve_(self):
        class R:  # minimal EigResult stand-in
            pass
        r = R()
        k = int(self.rank)
        r.evals = torch.arange(k, dtype=torch.float32)
        r.V = torch.zeros((self.computed_eigens[0].shape[0], k))
        return r


def _data(n=1003, d=8):
    return np.arange(n * d, dtype=np.float64).reshape(n, d)


@pytest.mark.parametrize("m", [5, 8, 13])
def test_single_thread_protocol(m):
    data = _data()
    b = br.InProcBroker("t-single")
    FakeSlave(b, data)
    master = FakeMaster(b, 3, m, data)
    master.start()
    assert len(master.batches_in_process) == 0 and master.batches == []
    step = data.shape[0] // m
    reqs = [json.loads(body) for q, body in b.delivered if q == "slaves"]
    resps = [json.loads(body) for q, body in b.delivered if q == "master"]
    # LIFO dispatch of contiguous N // M shards, remainder dropped
    assert [tuple(r["batch"]) for r in reqs] == [(i * step, (i + 1) * step)
                                                 for i in reversed(range(m))]
    assert all(r["rank"] == 3 for r in reqs)
    assert [r["batch"] for r in resps] == [r["batch"] for r in reqs]
    for r in resps:
        V = np.array(r["eigenspace"])
        assert V.shape == (8, 3)
        lo, hi = r["batch"]
        assert V[0, 0] == hi - lo and V[1, 0] == data[lo, 0]
    assert len(master.computed_eigens) == m
    assert master.eigenspace.shape == (8, 3) and master.eigenspace.flags["F_CONTIGUOUS"]
    assert b.acks == 2 * m


def test_window_smaller_than_five_is_accepted():
    """The reference raises IndexError for M < 5 (distributed.py:108-111); the drop-in
    sends min(5, M) requests instead."""
    data = _data(40, 4)
    b = br.InProcBroker("t-small")
    FakeSlave(b, data)
    master = FakeMaster(b, 2, 3, data)
    master.start()
    assert len(master.computed_eigens) == 3


def test_golden_dispatch_order_reproduced():
    g = load_golden("spiked_d128_k2_m5_ragged")
    b = br.InProcBroker("t-golden")
    FakeSlave(b, g["X"])
    master = FakeMaster(b, int(g["k"]), int(g["m"]), g["X"])
    master.start()
    resps = [json.loads(body)["batch"] for q, body in b.delivered if q == "master"]
    np.testing.assert_array_equal(np.array(resps), g["ranges"])


def test_duplicate_result_raises_keyerror_like_reference():
    data = _data(50, 4)
    b = br.InProcBroker("t-dup")
    master = FakeMaster(b, 2, 5, data)
    master.batches_in_process = {(0, 10)}
    body = json.dumps({"batch": [0, 10], "eigenspace": [[1.0, 0.0]] * 4}).encode()
    ch = master.channel
    master.batches_in_process = {(0, 10), (10, 20)}
    master.callback_(ch, type("M", (), {"delivery_tag": 1})(), None, body)
    with pytest.raises(KeyError):
        master.callback_(ch, type("M", (), {"delivery_tag": 2})(), None, body)


def test_threaded_slaves_with_my_threading():
    """Slave threads each serve their own channel; the master thread drives the flow."""
    data = _data(600, 6)
    b = br.InProcBroker("t-threads")
    slaves = [FakeSlave(b, data) for _ in range(3)]  # 3 consumers share one queue name
    # only the last registered consumer of 'slaves' receives (one consumer per queue)
    threads = [Slave(s.start) for s in slaves[-1:]]
    for t in threads:
        t.start()
    master = FakeMaster(b, 2, 6, data)
    mt = Slave(master.start)
    mt.start()
    mt.join(timeout=30, raise_error=True)
    assert not mt.is_alive()
    b.shutdown()
    for t in threads:
        t.join(timeout=30, raise_error=True)
        assert not t.is_alive()
    assert len(master.computed_eigens) == 6


def test_connect_by_name_shares_broker():
    br.reset("shared-x")
    a = br.connect("shared-x").broker
    c = br.connect("shared-x").broker
    assert a is c


def test_competing_slave_threads():
    """Several SlaveNodes, each in its own my_threading.Slave thread on the same
    "slaves" queue (RabbitMQ work-queue semantics: competing consumers): every shard
    is computed exactly once and the master completes (config 1's 8 threaded
    workers, distributed.py:33-57 + my_threading.py:6-15)."""
    data = _data(n=4000, d=8)
    m, nslaves = 13, 4
    b = br.InProcBroker("t-compete")
    slaves = [FakeSlave(b, data) for _ in range(nslaves)]
    threads = [Slave(s.start) for s in slaves]
    for t in threads:
        t.start()
    master = FakeMaster(b, 3, m, data)
    master.start()
    b.shutdown()
    for t in threads:
        t.join(raise_error=True)
    assert len(master.batches_in_process) == 0
    resps = [json.loads(body) for q, body in b.delivered if q == "master"]
    step = data.shape[0] // m
    assert sorted(tuple(r["batch"]) for r in resps) == [(i * step, (i + 1) * step) for i in range(m)]
    for r in resps:
        lo, hi = r["batch"]
        V = np.array(r["eigenspace"])
        assert V[0, 0] == hi - lo and V[1, 0] == data[lo, 0]
