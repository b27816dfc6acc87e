"""In-process message broker with the subset of pika's BlockingConnection API the
reference uses (distributed.py:14-20, :37, :40, :53, :57, :143).

The reference talks AMQP to RabbitMQ (transport T1, out of scope for the GPU
build).  This broker keeps the exact call pattern - ``queue_declare``,
``basic_consume(queue, on_message_callback)``, ``basic_publish(exchange,
routing_key, body)``, ``basic_ack``, ``start_consuming`` - so SlaveNode /
MasterNode run unchanged inside one process, single-threaded (one event loop
drives every consumer) or with ``my_threading.Slave`` threads (each thread
serves its own channel; several SlaveNodes on the "slaves" queue compete for its
messages like RabbitMQ workers).  Queues are FIFO, bodies are the same JSON strings.

Brokers are addressed by the ``broker_host`` string the nodes are given;
``connect(host)`` returns a connection to the broker registered under that name
(created on first use).
"""
from __future__ import annotations

import threading
import types
from collections import deque

__all__ = ["InProcBroker", "BlockingConnection", "ConnectionParameters", "connect", "get_broker",
           "reset"]


class InProcBroker:
    def __init__(self, name: str = "inproc"):
        self.name = name
        self.queues: dict[str, deque] = {}
        self.consumers: dict[str, list] = {}        # queue -> consuming channels (competing)
        self.callbacks: dict[str, callable] = {}
        self.active: set[int] = set()               # id(channel) with a thread in start_consuming
        self.cv = threading.Condition()
        self.closed = False
        self.delivered: list[tuple[str, str]] = []  # (queue, body) in delivery order
        self.acks = 0
        self._tag = 0

    # -- broker side
    def declare(self, q: str):
        with self.cv:
            self.queues.setdefault(q, deque())

    def publish(self, q: str, body):
        with self.cv:
            self.queues.setdefault(q, deque()).append(body)
            self.cv.notify_all()

    def shutdown(self):
        with self.cv:
            self.closed = True
            self.cv.notify_all()

    def pending(self) -> int:
        with self.cv:
            return sum(len(v) for v in self.queues.values())

    def _pick(self, ch: "Channel"):
        """Next (queue, channel) this loop may serve: queues ``ch`` consumes (several
        channels may consume one queue: competing consumers, like RabbitMQ workers
        sharing a work queue), plus queues none of whose consumers has a thread of
        its own in start_consuming (one loop then drives them all)."""
        for q, dq in self.queues.items():
            owners = self.consumers.get(q)
            if not dq or not owners:
                continue
            if ch in owners:
                return q, ch
            if not any(id(o) in self.active for o in owners):
                return q, owners[0]
        return None

    def _others_active(self, ch) -> bool:
        return any(a != id(ch) for a in self.active)

    def run(self, ch: "Channel"):
        with self.cv:
            self.active.add(id(ch))
        try:
            while True:
                with self.cv:
                    while True:
                        if ch._stop or self.closed:
                            return
                        pick = self._pick(ch)
                        if pick is not None:
                            break
                        if not self._others_active(ch):
                            return  # nothing can arrive any more: drained
                        self.cv.wait(timeout=0.05)
                    q, owner = pick
                    body = self.queues[q].popleft()
                    self.delivered.append((q, body))
                    self._tag += 1
                    tag = self._tag
                    cb = owner._callbacks[q]
                data = body.encode() if isinstance(body, str) else body
                cb(owner, types.SimpleNamespace(delivery_tag=tag, routing_key=q), None, data)
                with self.cv:
                    self.cv.notify_all()
        finally:
            with self.cv:
                self.active.discard(id(ch))
                self.cv.notify_all()


class Channel:
    def __init__(self, broker: InProcBroker):
        self.broker = broker
        self._stop = False
        self._callbacks: dict[str, callable] = {}

    def queue_declare(self, queue: str):
        self.broker.declare(queue)

    def basic_consume(self, queue: str, on_message_callback):
        with self.broker.cv:
            self.broker.queues.setdefault(queue, deque())
            owners = self.broker.consumers.setdefault(queue, [])
            if self not in owners:
                owners.append(self)
            self._callbacks[queue] = on_message_callback
            self.broker.callbacks[queue] = on_message_callback

    def basic_publish(self, exchange: str = "", routing_key: str = "", body=""):
        self.broker.publish(routing_key, body)

    def basic_ack(self, delivery_tag=None):
        with self.broker.cv:
            self.broker.acks += 1

    def start_consuming(self):
        self._stop = False
        self.broker.run(self)

    def stop_consuming(self):
        self._stop = True
        with self.broker.cv:
            self.broker.cv.notify_all()


class BlockingConnection:
    def __init__(self, parameters=None):
        host = getattr(parameters, "host", None) if parameters is not None else None
        if isinstance(parameters, dict):
            host = parameters.get("host")
        self.broker = get_broker(host or "inproc")

    def channel(self) -> Channel:
        return Channel(self.broker)

    def close(self):
        pass


class ConnectionParameters:
    def __init__(self, host: str = "inproc", **kw):
        self.host = host


_registry: dict[str, InProcBroker] = {}
_reg_lock = threading.Lock()


def get_broker(host) -> InProcBroker:
    if isinstance(host, InProcBroker):
        return host
    with _reg_lock:
        b = _registry.get(host)
        if b is None or b.closed:
            b = _registry[host] = InProcBroker(host)
        return b


def reset(host=None):
    with _reg_lock:
        if host is None:
            _registry.clear()
        else:
            _registry.pop(host, None)


def connect(host) -> BlockingConnection:
    if isinstance(host, InProcBroker):
        c = BlockingConnection.__new__(BlockingConnection)
        c.broker = host
        return c
    return BlockingConnection(ConnectionParameters(host=host))
