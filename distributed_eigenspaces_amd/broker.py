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

Separate processes (the reference's CLI: ``--mode slave`` / ``--mode master`` in
different shells, distributed.py:14-20, :156-184) talk through ``SocketBroker``, a
small TCP broker with the same channel API on the client side: start it with
``python -m distributed_eigenspaces_amd.broker --serve [HOST:]PORT`` (RabbitMQ's
role) and give the nodes ``--broker tcp://HOST:PORT`` (or ``HOST:PORT``).  Frames
are 4-byte big-endian lengths + UTF-8 JSON; dispatch follows RabbitMQ's defaults
as the reference uses them (no basic_qos): messages are pushed round-robin to a
queue's consumers as they arrive, acknowledged manually (basic_ack), and the
unacknowledged ones of a connection that closes are requeued at the front.
"""
from __future__ import annotations

import json
import queue
import socket
import struct
import threading
import types
from collections import deque

__all__ = ["InProcBroker", "BlockingConnection", "ConnectionParameters", "connect", "get_broker",
           "reset", "SocketBroker", "SocketConnection", "parse_address", "serve"]


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


def parse_address(host):
    """(host, port) for a socket-broker address ("tcp://H:P", "tcp://H", "H:P"), else None."""
    if not isinstance(host, str):
        return None
    h = host
    if h.startswith("tcp://"):
        h = h[len("tcp://"):]
        if ":" not in h:
            return h, 5672  # RabbitMQ's port, like the reference's ConnectionParameters(host)
    if h.count(":") == 1:
        name, port = h.split(":")
        if port.isdigit() and name:
            return name, int(port)
    return None


def connect(host):
    if isinstance(host, InProcBroker):
        c = BlockingConnection.__new__(BlockingConnection)
        c.broker = host
        return c
    addr = parse_address(host)
    if addr is not None:
        return SocketConnection(*addr)
    return BlockingConnection(ConnectionParameters(host=host))


# ---------------------------------------------------------------- socket transport
def _send(sock, obj, lock):
    data = json.dumps(obj).encode()
    with lock:
        sock.sendall(struct.pack(">I", len(data)) + data)


def _recv(sock):
    hdr = b""
    while len(hdr) < 4:
        chunk = sock.recv(4 - len(hdr))
        if not chunk:
            return None
        hdr += chunk
    (n,) = struct.unpack(">I", hdr)
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(1 << 20, n - len(buf)))
        if not chunk:
            return None
        buf += chunk
    return json.loads(buf.decode())


class _Client:
    """Server-side state of one client connection.  Deliveries go through an outbox
    drained by the client's own sender thread, so a consumer that stops reading (a
    master busy in its callback, a stalled process) blocks only its own socket
    writes - never the broker lock that every other connection needs."""

    def __init__(self, sock):
        self.sock = sock
        self.lock = threading.Lock()
        self.queues = set()   # queues this connection consumes
        self.unacked = {}     # tag -> (queue, body)
        self.alive = True
        self.outbox = queue.SimpleQueue()
        self.sender = threading.Thread(target=self._send_loop, daemon=True)
        self.sender.start()

    def _send_loop(self):
        while True:
            obj = self.outbox.get()
            if obj is None:
                return
            try:
                _send(self.sock, obj, self.lock)
            except OSError:
                # dead peer: closing the socket ends the reader, which requeues the
                # unacked deliveries (SocketBroker._serve_client)
                self.alive = False
                try:
                    self.sock.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass
                return


class SocketBroker:
    """TCP message broker with the pika channel-API subset of the reference.

    ``SocketBroker(host, port).start()`` serves in background threads (port 0 picks
    a free one; ``address`` gives "tcp://host:port"); ``serve_forever()`` blocks."""

    def __init__(self, host: str = "127.0.0.1", port: int = 5672):
        self.srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.srv.bind((host, port))
        self.srv.listen(64)
        self.host, self.port = self.srv.getsockname()[:2]
        self.lock = threading.Lock()
        self.queues: dict[str, deque] = {}
        self.consumers: dict[str, list] = {}
        self.rr: dict[str, int] = {}
        self.clients: list[_Client] = []
        self.delivered: list[tuple[str, str]] = []  # (queue, body) in delivery order
        self._tag = 0
        self._closed = False
        self._thread = None

    @property
    def address(self) -> str:
        return f"tcp://{self.host}:{self.port}"

    def start(self):
        self._thread = threading.Thread(target=self.serve_forever, daemon=True)
        self._thread.start()
        return self

    def serve_forever(self):
        while not self._closed:
            try:
                sock, _ = self.srv.accept()
            except OSError:
                break
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            c = _Client(sock)
            with self.lock:
                self.clients.append(c)
            threading.Thread(target=self._serve_client, args=(c,), daemon=True).start()

    def shutdown(self):
        """Stop accepting and close every connection (consumers' loops then return)."""
        self._closed = True
        try:
            self.srv.close()
        except OSError:
            pass
        with self.lock:
            clients = list(self.clients)
        for c in clients:
            try:
                c.sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            c.sock.close()

    # -- dispatch (call with self.lock held)
    def _dispatch(self, q):
        dq = self.queues.setdefault(q, deque())
        while dq:
            live = [c for c in self.consumers.get(q, []) if c.alive]
            if not live:
                return
            i = self.rr.get(q, 0) % len(live)
            self.rr[q] = i + 1
            c = live[i]
            body = dq.popleft()
            self._tag += 1
            c.unacked[self._tag] = (q, body)
            self.delivered.append((q, body))
            c.outbox.put({"op": "deliver", "queue": q, "tag": self._tag, "body": body})

    def _serve_client(self, c: _Client):
        try:
            while True:
                msg = _recv(c.sock)
                if msg is None:
                    break
                op = msg.get("op")
                with self.lock:
                    if op == "declare":
                        self.queues.setdefault(msg["queue"], deque())
                    elif op == "consume":
                        q = msg["queue"]
                        c.queues.add(q)
                        self.consumers.setdefault(q, []).append(c)
                        self._dispatch(q)
                    elif op == "publish":
                        q = msg["queue"]
                        self.queues.setdefault(q, deque()).append(msg["body"])
                        self._dispatch(q)
                    elif op == "ack":
                        c.unacked.pop(msg["tag"], None)
                    elif op == "cancel":
                        for q in c.queues:
                            if c in self.consumers.get(q, []):
                                self.consumers[q].remove(c)
                        c.queues.clear()
        except OSError:
            pass
        finally:
            c.outbox.put(None)  # stop the sender
            with self.lock:
                c.alive = False
                for q in list(c.queues):
                    if c in self.consumers.get(q, []):
                        self.consumers[q].remove(c)
                # unacked messages go back to the front of their queues, in order
                for tag in sorted(c.unacked, reverse=True):
                    q, body = c.unacked[tag]
                    self.queues.setdefault(q, deque()).appendleft(body)
                c.unacked.clear()
                if c in self.clients:
                    self.clients.remove(c)
                for q in list(self.queues):
                    self._dispatch(q)
            try:
                c.sock.close()
            except OSError:
                pass


class SocketChannel:
    """Client channel of a SocketConnection: the pika BlockingChannel subset the
    reference uses (distributed.py:19-20, :37, :40, :53, :57, :115, :139, :143)."""

    def __init__(self, conn: "SocketConnection"):
        self.conn = conn
        self._callbacks: dict[str, callable] = {}
        self._stop = False

    def queue_declare(self, queue: str):
        _send(self.conn.sock, {"op": "declare", "queue": queue}, self.conn.lock)

    def basic_consume(self, queue: str, on_message_callback):
        self._callbacks[queue] = on_message_callback
        _send(self.conn.sock, {"op": "consume", "queue": queue}, self.conn.lock)

    def basic_publish(self, exchange: str = "", routing_key: str = "", body=""):
        if isinstance(body, bytes):
            body = body.decode()
        _send(self.conn.sock, {"op": "publish", "queue": routing_key, "body": body}, self.conn.lock)

    def basic_ack(self, delivery_tag=None):
        _send(self.conn.sock, {"op": "ack", "tag": delivery_tag}, self.conn.lock)

    def start_consuming(self):
        """Deliver messages to the callbacks until stop_consuming() or the broker
        closes the connection."""
        self._stop = False
        while not self._stop:
            msg = _recv(self.conn.sock)
            if msg is None:
                return
            if msg.get("op") != "deliver":
                continue
            q = msg["queue"]
            method = types.SimpleNamespace(delivery_tag=msg["tag"], routing_key=q)
            self._callbacks[q](self, method, None, msg["body"].encode())

    def stop_consuming(self):
        self._stop = True
        try:
            _send(self.conn.sock, {"op": "cancel"}, self.conn.lock)
        except OSError:
            pass


class SocketConnection:
    """``pika.BlockingConnection`` stand-in for a SocketBroker at (host, port)."""

    def __init__(self, host: str, port: int, timeout: float = 30.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.settimeout(None)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.lock = threading.Lock()

    def channel(self) -> SocketChannel:
        return SocketChannel(self)

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass


def serve(argv=None):
    """``python -m distributed_eigenspaces_amd.broker --serve [HOST:]PORT``."""
    import argparse
    ap = argparse.ArgumentParser(description="socket broker for the distributed eigenspace nodes")
    ap.add_argument("--serve", default="127.0.0.1:5672", help="[HOST:]PORT to listen on")
    a = ap.parse_args(argv)
    host, _, port = a.serve.rpartition(":")
    b = SocketBroker(host or "127.0.0.1", int(port))
    print(f"broker listening on {b.address}", flush=True)
    try:
        b.serve_forever()
    except KeyboardInterrupt:
        b.shutdown()


if __name__ == "__main__":
    serve()
