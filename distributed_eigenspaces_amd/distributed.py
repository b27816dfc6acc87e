"""Drop-in for the reference's ``distributed.py`` (TimeEscaper/distributed_eigenspaces).

Same classes, methods, arguments, message schema and CLI flags; the arithmetic
runs on the GPU through the HIP hot path:

* ``SlaveNode.compute_sigma_hat_``  (distributed.py:59-70)  -> MFMA SYRK (float64 data:
  mean-shifted, float64 result; uint8: exact integer)
* ``Node.top_k_eigenvectors``       (distributed.py:22-29)  -> subspace iteration + RR
* ``MasterNode.callback_`` average  (distributed.py:126-130) -> implicit projector-average
  top-k (the reference builds the d x d sigma_tilde and discards it; the notebook's
  server solve, raw line 306, is what is computed here - without forming d x d).

Transport: the reference uses pika/RabbitMQ (out of scope).  ``broker_host`` is
either ``tcp://HOST:PORT`` - the socket broker of ``broker.py``, so ``--mode slave``
and ``--mode master`` run as separate processes like the reference's CLI - or a
name of an in-process broker with the same channel API; requests and responses
are the same JSON documents
(request ``{"rank": k, "batch": [lo, hi]}``, response
``{"batch": [lo, hi], "eigenspace": d x k nested list}``, distributed.py:49-52,
:109-112).

Deliberate differences (all additive; none changes a result for inputs the
reference accepts):
* the master's initial window is ``min(5, batches_number)`` instead of 5 (the
  reference raises IndexError for batches_number < 5, distributed.py:108-111);
* when the last shard arrives the master stores its result (``self.result``,
  ``self.eigenspace``) and calls ``channel.stop_consuming()`` so ``start()`` returns;
* ``top_k_eigenvectors`` / ``compute_sigma_hat_`` accept torch tensors on the GPU
  and then return GPU tensors (numpy in -> numpy float64 out, like the reference).
"""
from __future__ import annotations

import argparse
import json
import time
from contextlib import nullcontext

import numpy as np
import torch

from . import broker as _broker
from . import linalg

__all__ = ["Node", "SlaveNode", "MasterNode", "run_master", "run_slave", "main",
           "top_k_eigenvectors", "top_k_eigh", "compute_sigma_hat"]

WINDOW = 5  # requests in flight at start (distributed.py:108)


def _is_numpy(x) -> bool:
    return isinstance(x, np.ndarray) or not isinstance(x, torch.Tensor)


def _rows_to_device(data, lo: int, hi: int) -> torch.Tensor:
    """Rows [lo, hi) of the node's data on the GPU, read from ``data`` on every call
    like the reference's ``self.data[lo:hi]`` (distributed.py:46).  A GPU tensor is
    sliced in place (no copy); host data (numpy, CPU tensors, array-likes) has only
    the requested rows uploaded, so a write to the host array between requests is
    always seen - there is no device-side cache to go stale.  uint8 samples stay
    uint8 (the exact integer covariance path), float64 stays float64 (the
    reference's dtype: the mean-shifted covariance path), everything else becomes
    float32.  To keep one resident copy for many requests, hand the node a GPU
    tensor."""
    if isinstance(data, torch.Tensor) and data.is_cuda:
        rows = data[lo:hi]
        if rows.dtype in (torch.uint8, torch.float32, torch.float64):
            return rows
        return linalg.require_device_tensor(rows, "SlaveNode.data")
    if not torch.cuda.is_available():
        raise RuntimeError("SlaveNode: needs a ROCm GPU; there is no CPU fallback")
    if isinstance(data, torch.Tensor):
        rows = data[lo:hi]
    else:
        a = np.asarray(data[lo:hi])
        # torch cannot wrap a read-only array without a warning: copy those rows
        rows = torch.from_numpy(a if a.flags.writeable else a.copy())
    if rows.dtype == torch.uint8:
        return rows.to(torch.device("cuda", torch.cuda.current_device()))
    return linalg.require_device_tensor(rows, "SlaveNode.data", keep_f64=True)


def top_k_eigh(matrix, k: int):
    """(eigenvalues ascending, eigenvectors d x k ascending) of a symmetric matrix
    (any symmetric input, any 1 <= k <= d, like distributed.py:29's eigh)."""
    res = linalg.topk_eigh(linalg.require_device_tensor(matrix, "matrix", keep_f64=True), int(k))
    if _is_numpy(matrix):
        w = res.evals.double().cpu().numpy()
        v = np.asfortranarray(res.V.double().cpu().numpy())
        return w, v
    return res.evals, res.V


def top_k_eigenvectors(matrix, k: int):
    """``Node.top_k_eigenvectors`` (distributed.py:22-29): top-k eigenvectors, ascending."""
    return top_k_eigh(matrix, k)[1]


def compute_sigma_hat(x):
    """``SlaveNode.compute_sigma_hat_`` (distributed.py:59-70): X^T X / n, uncentered.

    numpy in -> float64 numpy out, like the reference: float samples take the
    mean-shifted path (float64 result), uint8 samples the exact integer path
    (float64 result).  GPU tensors: float32 -> the float32 SYRK, float64 -> the
    shifted path (float64), uint8 -> exact (float64)."""
    if _is_numpy(x):
        a = np.asarray(x)
        t = torch.as_tensor(a if a.dtype in (np.uint8, np.float64) else a.astype(np.float64))
        S = linalg.sigma_hat(t, dtype=torch.float64)
        return S.cpu().numpy()
    if x.dtype == torch.uint8:
        return linalg.sigma_hat(x, dtype=torch.float64)
    return linalg.sigma_hat(x)


class Node:
    """distributed.py:13-29: broker connection + top-k helper."""

    def __init__(self, broker_host):
        self.connection = _broker.connect(broker_host)
        self.channel = self.connection.channel()
        self.channel.queue_declare(queue="master")
        self.channel.queue_declare(queue="slaves")

    def top_k_eigenvectors(self, matrix, k):
        return top_k_eigenvectors(matrix, k)


class SlaveNode(Node):
    """distributed.py:32-70: worker.  Each request reads rows [lo, hi) of ``data``
    (distributed.py:46): a GPU tensor is sliced in place, host data has those rows
    uploaded (``_rows_to_device``)."""

    def __init__(self, broker_host, data):
        super().__init__(broker_host)
        print("Slave Start listening")
        self.data = data
        self._stream = None
        self.channel.basic_consume(queue="slaves", on_message_callback=self.callback_)

    def start(self):
        self.channel.start_consuming()

    def _device_rows(self, lo, hi):
        return _rows_to_device(self.data, lo, hi)

    def callback_(self, channel, method, properties, body):
        request = json.loads(body)
        print("Slave: Received, batchid: " + str(request["batch"]))
        lo, hi = request["batch"][0], request["batch"][1]
        batch = self._device_rows(lo, hi)
        if batch.is_cuda:
            if self._stream is None:  # one HIP stream per node: threaded nodes overlap
                self._stream = torch.cuda.Stream(batch.device)
            # the rows were uploaded (or written) on the current stream
            self._stream.wait_stream(torch.cuda.current_stream(batch.device))
            batch.record_stream(self._stream)  # an uploaded copy is freed only after its use
        with (torch.cuda.stream(self._stream) if self._stream is not None else nullcontext()):
            eigenspace = self.compute_sigma_hat_(batch)
            eigenspace = self.top_k_eigenvectors(eigenspace, request["rank"])
            response = dict()
            response["batch"] = request["batch"]
            response["eigenspace"] = eigenspace.double().cpu().numpy().tolist()
        self.send_to_master_(str(json.dumps(response)))
        channel.basic_ack(delivery_tag=method.delivery_tag)

    def send_to_master_(self, message):
        print("Sending to Master")
        self.channel.basic_publish(exchange="", routing_key="master", body=message)

    def compute_sigma_hat_(self, x):
        return compute_sigma_hat(x)


class MasterNode(Node):
    """distributed.py:82-143: shard split, dispatch window, projector average."""

    def __init__(self, broker_host, rank, batches_number, data):
        super().__init__(broker_host)
        self.rank = rank
        self.batches_number = batches_number
        self.data = data
        self.batches_in_process = set()
        self.batches = list()
        self.computed_eigens = list()
        self.current_batch = 0
        self.result = None      # linalg.EigResult of the server solve
        self.eigenspace = None  # numpy float64 d x k, ascending (NB:306 semantics)
        self.eigenvalues = None
        print("Master Start listening")
        self.start_time = time.time()
        self.channel.basic_consume(queue="master", on_message_callback=self.callback_)

    def start(self):
        print("Splitting dataset...")
        step = self.data.shape[0] // self.batches_number
        for i in range(self.batches_number):
            batch = (i * step, (i + 1) * step)
            self.batches.append(batch)
            self.batches_in_process.add(batch)
        print("Sending to slaves...")
        for _ in range(min(WINDOW, len(self.batches))):
            request = dict()
            request["rank"] = self.rank
            request["batch"] = self.batches.pop()
            self.send_to_slaves_(str(json.dumps(request)))
        print("Start waiting for messages")
        self.channel.start_consuming()

    def callback_(self, channel, method, properties, body):
        request = json.loads(body)
        batch = (request["batch"][0], request["batch"][1])
        print("Master: Received, batch: " + str(batch))
        eigenspace = np.array(request["eigenspace"])
        self.computed_eigens.append(eigenspace)
        self.batches_in_process.remove(batch)
        if len(self.batches_in_process) == 0:
            self.result = self.server_solve_()
            self.eigenvalues = self.result.evals.double().cpu().numpy()
            self.eigenspace = np.asfortranarray(self.result.V.double().cpu().numpy())
            print("Computed! Time (seconds): " + str(time.time() - self.start_time))
            channel.basic_ack(delivery_tag=method.delivery_tag)
            self.channel.stop_consuming()
            return
        elif len(self.batches) != 0:
            request = dict()
            request["batch"] = self.batches.pop()
            request["rank"] = self.rank
            self.send_to_slaves_(str(json.dumps(request)))
            print("Sended batch: " + str(request["batch"]))
        channel.basic_ack(delivery_tag=method.delivery_tag)

    def server_solve_(self):
        """Top-k of (1/batches_number) sum_i V_i V_i^T in arrival order, implicit."""
        bases = [linalg.require_device_tensor(e, "eigenspace") for e in self.computed_eigens]
        Wt = linalg.stack_bases(bases)
        return linalg.projavg_topk(Wt, int(self.rank), 1.0 / self.batches_number, q0=bases[0])

    def send_to_slaves_(self, message):
        print("Sending to slaves: ")
        self.channel.basic_publish(exchange="", routing_key="slaves", body=message)


def run_master(broker, rank, batches_number, data):
    master = MasterNode(broker, rank, batches_number, data)
    master.start()
    return master


def run_slave(broker, data):
    slave = SlaveNode(broker, data)
    slave.start()
    return slave


def run_local(rank, batches_number, data, broker_name="inproc-local"):
    """Both roles in one process over the in-process broker (addition)."""
    b = _broker.InProcBroker(broker_name)
    SlaveNode(b, data)
    master = MasterNode(b, rank, batches_number, data)
    master.start()
    return master


def preprocess(data):
    """distributed.py:170-173: grayscale (mean over RGB) and flatten to R^1024."""
    data = data.mean(axis=3)
    return data.reshape(data.shape[:-2] + (-1,))


def load_dataset(path):
    """The reference's data (distributed.py:169-173) for the nodes.

    A CIFAR batch directory (load_data.py:18-33) stays uint8 (N, 32, 32, 3): the
    grayscale + flatten of :170-173 is fused into the exact integer covariance on
    the GPU (linalg.sigma_hat_u8), which gives the reference's float64 result within
    one fp32 ulp (float64 output: to double rounding).  A ``.npy`` file (addition, for non-CIFAR data and
    tests) is used as stored (loaded without pickle); a 4-D float array there gets
    the reference's host preprocessing."""
    import os
    if os.path.isfile(path) and path.endswith(".npy"):
        data = np.load(path, allow_pickle=False)
    else:
        from .load_data import load_CIFAR_10_data
        data, filenames, labels = load_CIFAR_10_data(path)
    if data.ndim == 4 and data.dtype != np.uint8:
        data = preprocess(data)
    return data


def cli_broker(broker: str, mode):
    """The broker a CLI node connects to.  ``--mode slave`` / ``--mode master`` are
    separate processes, as in the reference, whose ``--broker`` is a RabbitMQ host
    name (``pika.ConnectionParameters(host)``, distributed.py:16): a bare host or IP
    there means the socket broker on that host at pika's default port 5672 (start
    it with ``python -m distributed_eigenspaces_amd.broker --serve HOST:5672``).  An
    in-process broker name cannot connect two processes, so it is never chosen for
    those modes; ``--mode local`` keeps in-process names."""
    if mode in ("slave", "master") and _broker.parse_address(broker) is None:
        return f"tcp://{broker}:5672"
    return broker


def main(argv=None):
    parser = argparse.ArgumentParser(description="Multinode PCA")
    parser.add_argument("--mode", help="Mode to run script - slave, master or local")
    parser.add_argument("--broker", help="Message broker: tcp://HOST:PORT (socket broker, separate "
                        "processes; start it with python -m distributed_eigenspaces_amd.broker "
                        "--serve HOST:PORT) or a name (in-process broker)")
    parser.add_argument("--rank", help="Approximation rank (only for master node")
    parser.add_argument("--batches", help="Total batches number")
    parser.add_argument("--data", default="cifar-10-batches-py", help="Path to dataset")
    args = parser.parse_args(argv)
    if args.broker is None:
        raise RuntimeError("Broker not specified")
    broker = cli_broker(args.broker, args.mode)
    data = load_dataset(args.data)
    if args.mode == "slave":
        return run_slave(broker, data)
    elif args.mode == "master":
        return run_master(broker, int(args.rank), int(args.batches), data)
    elif args.mode == "local":
        return run_local(int(args.rank), int(args.batches), data, args.broker)
    raise RuntimeError("Mode not specified or specified wrong")


if __name__ == "__main__":
    main()
