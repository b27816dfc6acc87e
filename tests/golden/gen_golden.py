#!/usr/bin/env python
"""Generate golden input/output vectors by RUNNING the reference in this container.

Test infrastructure only.  Writes small ``.npz`` fixtures into ``tests/golden/``.
Nothing from the reference is copied: the reference modules are imported from
``/root/reference`` at generation time and only their *outputs* are stored.
Skips itself (exit 0) when ``/root/reference`` is absent (e.g. on the GPU box).

Two in-process shims are needed to import/run the reference here:

* ``pika`` is not installed (``distributed.py:3``).  A minimal in-memory broker
  with the subset of the pika API the reference calls
  (``BlockingConnection``/``ConnectionParameters``/``channel``/``queue_declare``/
  ``basic_consume``/``basic_publish``/``basic_ack``/``start_consuming``) is put in
  ``sys.modules['pika']`` before import.  Delivery is FIFO per queue; one event
  loop dispatches to every registered consumer until all queues drain.
* scipy 1.15 removed ``eigh(eigvals=...)`` (used at ``distributed.py:29``).  The
  module-level name ``distributed.largest_eigh`` is rebound to a wrapper that maps
  ``eigvals=(lo,hi)`` to ``subset_by_index=(lo,hi)`` - same LAPACK ``?syevr``
  driver, same inclusive 0-based range.  The wrapper also records ``eigh(...)[0]``
  (the eigenvalues the reference discards) as a side output.

The notebook's online loop (``Online Distributed PCA.ipynb`` raw lines 149-153,
219-226, 277-316) is executed from the notebook JSON itself, with its buggy
``compute_segma_hat`` (raw 235-246: an n x n Gram) replaced by the
``distributed.py:59-70`` definition, as SURVEY.md §0.1 prescribes.

Usage:  python tests/golden/gen_golden.py
"""
import json
import os
import sys
import types
from collections import deque

import numpy as np
import scipy.linalg

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
NB_NAME = "Online Distributed PCA.ipynb"


# ----------------------------------------------------------------------------- pika stub
class _Broker:
    def __init__(self):
        self.queues = {}
        self.consumers = {}
        self.delivered = []  # (queue, body) in delivery order
        self.tag = 0

    def declare(self, q):
        self.queues.setdefault(q, deque())

    def publish(self, q, body):
        self.declare(q)
        self.queues[q].append(body)

    def run(self):
        progressed = True
        while progressed:
            progressed = False
            for q, dq in self.queues.items():
                if dq and q in self.consumers:
                    body = dq.popleft()
                    self.delivered.append((q, body))
                    self.tag += 1
                    ch, cb = self.consumers[q]
                    cb(ch, types.SimpleNamespace(delivery_tag=self.tag), None,
                       body.encode() if isinstance(body, str) else body)
                    progressed = True
                    break


BROKER = _Broker()


class _Channel:
    def queue_declare(self, queue):
        BROKER.declare(queue)

    def basic_consume(self, queue, on_message_callback):
        BROKER.consumers[queue] = (self, on_message_callback)

    def basic_publish(self, exchange, routing_key, body):
        BROKER.publish(routing_key, body)

    def basic_ack(self, delivery_tag):
        pass

    def start_consuming(self):
        BROKER.run()


class _Connection:
    def __init__(self, params):
        self.params = params

    def channel(self):
        return _Channel()


def install_pika_stub():
    mod = types.ModuleType("pika")
    mod.BlockingConnection = _Connection
    mod.ConnectionParameters = lambda host=None: {"host": host}
    sys.modules["pika"] = mod


# ----------------------------------------------------------------------------- eigh shim
EIGVALS_LOG = []


def eigh_shim(a, eigvals=None, **kw):
    w, v = scipy.linalg.eigh(a, subset_by_index=eigvals, **kw)
    EIGVALS_LOG.append(np.array(w, dtype=np.float64))
    return w, v


# ----------------------------------------------------------------------------- data
sys.path.insert(0, os.path.dirname(OUT))  # tests/: golden_data (the input generator)
from golden_data import spiked_int_data, xq_digest  # noqa: E402


def import_reference():
    install_pika_stub()
    sys.path.insert(0, REF)
    import distributed  # noqa: E402  (reference module)
    import my_threading  # noqa: F401,E402
    distributed.largest_eigh = eigh_shim
    return distributed


# ----------------------------------------------------------------------------- cases
def run_protocol(distributed, data, rank, batches_number):
    """Full master/slave protocol of distributed.py:96-139 through the stub broker."""
    BROKER.__init__()
    slave = distributed.SlaveNode("stub", data)
    master = distributed.MasterNode("stub", rank, batches_number, data)
    EIGVALS_LOG.clear()
    master.start()
    assert len(master.batches_in_process) == 0, "protocol did not complete"
    # every slave message: the response JSON, in arrival order at the master
    responses = [json.loads(b) for q, b in BROKER.delivered if q == "master"]
    requests = [json.loads(b) for q, b in BROKER.delivered if q == "slaves"]
    ranges = np.array([r["batch"] for r in responses], dtype=np.int64)
    Vs = np.stack([np.asarray(e) for e in master.computed_eigens])
    evals = np.stack(EIGVALS_LOG[: len(Vs)])
    # master's sigma_tilde (distributed.py:126-130) is a local it discards; rebuild it
    # from the master's own list with the same loop order, then the notebook's server
    # solve (raw line 306) via the reference's own top_k_eigenvectors.
    d = Vs.shape[1]
    sigma_tilde = np.zeros((d, d))
    for e in master.computed_eigens:
        sigma_tilde += e @ e.T
    sigma_tilde /= batches_number
    EIGVALS_LOG.clear()
    Vbar = distributed.Node.top_k_eigenvectors(None, sigma_tilde, rank)
    server_evals = EIGVALS_LOG[-1]
    return dict(ranges=ranges, request_ranges=np.array([r["batch"] for r in requests]),
                request_ranks=np.array([r["rank"] for r in requests]), worker_V=Vs,
                worker_evals=evals, server_V=Vbar, server_evals=server_evals,
                sigma_tilde=sigma_tilde)


def direct_workers(distributed, data, rank, batches_number, server=True):
    """Worker math of distributed.py:46-48 for each shard of :99-104 (m < 5 cannot
    run the protocol: the window of 5 at :108 pops an empty list)."""
    step = data.shape[0] // batches_number
    ranges, Vs, evs = [], [], []
    for i in range(batches_number):
        lo, hi = i * step, (i + 1) * step
        S = distributed.SlaveNode.compute_sigma_hat_(None, data[lo:hi])
        EIGVALS_LOG.clear()
        V = distributed.Node.top_k_eigenvectors(None, S, rank)
        ranges.append((lo, hi)); Vs.append(V); evs.append(EIGVALS_LOG[-1])
    Vs = np.stack(Vs)
    if not server:
        return dict(ranges=np.array(ranges), worker_V=Vs, worker_evals=np.stack(evs))
    d = Vs.shape[1]
    sigma_tilde = np.zeros((d, d))
    for e in Vs:
        sigma_tilde += e @ e.T
    sigma_tilde /= batches_number
    EIGVALS_LOG.clear()
    Vbar = distributed.Node.top_k_eigenvectors(None, sigma_tilde, rank)
    return dict(ranges=np.array(ranges), worker_V=Vs, worker_evals=np.stack(evs),
                server_V=Vbar, server_evals=EIGVALS_LOG[-1], sigma_tilde=sigma_tilde)


def notebook_online(distributed, data, batch_size):
    """Execute the notebook's own cells (make_batches, top_k_eigenvectors, online loop)."""
    nb = json.load(open(os.path.join(REF, NB_NAME)))
    cells = ["".join(c["source"]) for c in nb["cells"] if c["cell_type"] == "code"]
    src_make = next(c for c in cells if c.startswith("def make_batches"))
    src_topk = next(c for c in cells if c.startswith("def top_k_eigenvectors"))
    src_loop = next(c for c in cells if "segma_e = segma_e" in c)
    src_final = next(c for c in cells if c.startswith("matrix_w = top_k_eigenvectors"))
    ns = {"np": np, "largest_eigh": eigh_shim, "tqdm": lambda it: it}
    exec(src_make, ns)
    exec(src_topk, ns)
    # the notebook's compute_segma_hat is an n x n Gram (ValueError for
    # n != d); use the distributed.py:59-70 definition in its place.
    ns["compute_segma_hat"] = lambda x: distributed.SlaveNode.compute_sigma_hat_(None, x)
    ns["batches"] = ns["make_batches"](data, batch_size)
    exec(src_loop, ns)
    EIGVALS_LOG.clear()
    exec(src_final, ns)
    return dict(batch_size=np.int64(batch_size), n_batches=np.int64(len(ns["batches"])),
                m=np.int64(ns["m"]), T=np.int64(ns["T"]), k=np.int64(ns["k"]),
                matrix_w=ns["matrix_w"], final_evals=EIGVALS_LOG[-1],
                segma_e=ns["segma_e"], last_v_dash=ns["v_dash"])


def main():
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return 0
    distributed = import_reference()
    grid = 8.0
    cases = [
        # name, n, d, k, m, seed, protocol?, store sigma_hat of shard 0?
        ("spiked_d64_k4_m8", 8 * 128, 64, 4, 8, 11, True, True),
        ("spiked_d128_k2_m5_ragged", 5 * 100 + 3, 128, 2, 5, 12, True, True),
        ("spiked_d256_k10_m8", 8 * 320, 256, 10, 8, 13, True, True),
        ("spiked_d256_k16_m4", 4 * 300, 256, 16, 4, 14, False, False),
        ("spiked_d1024_k16_m1", 1200, 1024, 16, 1, 15, False, False),
        # config-2 width (d = 3072); inputs regenerated from the seed by the tests
        # (tests/golden_data.py, pinned by xq_sha256): 37 MB of samples not stored
        ("spiked_d3072_k16_m2_seeded", 2 * 3200, 3072, 16, 2, 16, False, False),
        # config-3 width and k (d = 8192, k = 64): one 16384-row shard (the top-64
        # subspace is well separated there: lambda_64 ~ 5 vs the noise edge ~ 2.9)
        ("spiked_d8192_k64_m1_seeded", 16384, 8192, 64, 1, 17, False, False),
        # config-5 width and k (d = 16384, k = 128: the subspace the solver runs with
        # p = k, no guard columns): one 32768-row shard; the worker outputs only,
        # stored as float32 (16 MB of float64 otherwise; the tests' bars are 1e-4 / 1e-5)
        ("spiked_d16384_k128_m1_seeded", 32768, 16384, 128, 1, 18, False, False),
        # config-3's server leg: m = 8 shards of 8192 rows at d = 8192, k = 64 (the
        # 8-basis projector average of distributed.py:126-130 + NB:306); stores the
        # server outputs, every worker's eigenvalues and shard 0's basis (float32)
        ("spiked_d8192_k64_m8_seeded", 8 * 8192, 8192, 64, 8, 19, False, False),
    ]
    only = set(sys.argv[1:])  # optional: regenerate just the named cases
    for name, n, d, k, m, seed, proto, store_s in cases:
        if only and name not in only:
            continue
        Xq, U = spiked_int_data(n, d, k, seed, grid=grid)
        data = Xq.astype(np.float64) / grid  # float64 like distributed.py:171
        if proto:
            res = run_protocol(distributed, data, k, m)
        else:
            res = direct_workers(distributed, data, k, m, server=d <= 8192)
        out = dict(Xq=Xq, grid=np.float64(grid), k=np.int64(k), m=np.int64(m),
                   U_planted=U.astype(np.float32), **res)
        if name.endswith("_seeded"):
            out.pop("Xq")
            if d > 4096:
                out.pop("U_planted")  # regenerable from the seed; keeps the fixture small
            if d > 8192:
                out["worker_V"] = out["worker_V"].astype(np.float32)
            if m > 1 and d >= 8192:  # keep the fixture small: shard 0's basis only
                out["worker_V"] = out["worker_V"][:1].astype(np.float32)
                out["server_V"] = out["server_V"].astype(np.float32)
            out.update(seed=np.int64(seed), n=np.int64(n), d=np.int64(d),
                       xq_sha256=np.array(xq_digest(Xq)))
        if (not store_s or d > 256) and "sigma_tilde" in out:
            out.pop("sigma_tilde")
        if store_s:
            lo, hi = res["ranges"][0] if not proto else (0, n // m)
            out["sigma_hat0"] = distributed.SlaveNode.compute_sigma_hat_(None, data[lo:hi])
            out["sigma_hat0_range"] = np.array([lo, hi])
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
        print("wrote", name, {k_: getattr(v, "shape", v) for k_, v in out.items()})

    if only:
        return 0
    # notebook online loop (m=10, T=10, k=2 are hard-coded in the cell; raw 277-279)
    Xq, _ = spiked_int_data(10 * 96 + 37, 64, 2, 21, grid=grid)
    data = Xq.astype(np.float64) / grid
    res = notebook_online(distributed, data, 96)
    np.savez_compressed(os.path.join(OUT, "notebook_online_d64.npz"), Xq=Xq,
                        grid=np.float64(grid), **res)
    print("wrote notebook_online_d64", {k_: getattr(v, "shape", v) for k_, v in res.items()})

    # my_threading.Slave semantics (my_threading.py:6-15): run() calls target(*args)
    import my_threading
    got = []
    t = my_threading.Slave(lambda a, b: got.append((a, b)), 3, "x")
    t.start(); t.join()
    with open(os.path.join(OUT, "my_threading.json"), "w") as f:
        json.dump({"calls": got, "is_thread": isinstance(t, __import__("threading").Thread)}, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
