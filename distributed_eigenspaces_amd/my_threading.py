"""Drop-in for the reference's ``my_threading.py``: the worker-thread API.

``Slave(target, *args)`` is a ``threading.Thread`` whose ``run()`` calls
``target(*args)`` (my_threading.py:6-15).  As in the reference, keyword
arguments are not forwarded and ``start()`` / ``join()`` are the plain Thread
methods.  Additions (no behaviour change for reference callers): the target's
return value is kept in ``.result`` and an exception raised by the target in
``.exception`` (the reference loses both), and ``join(raise_error=True)``
re-raises it in the joining thread.

With the GPU hot path the threads overlap for real: the ctypes calls into
libdeig.so release the GIL, and each thread launches on its own current stream.
"""
from __future__ import annotations

import threading

__all__ = ["Slave"]


class Slave(threading.Thread):
    """Thread running ``target(*args)``; results flow through ``.result``."""

    def __init__(self, target, *args):
        super().__init__(target=target, args=args)
        self.fn = target
        self.fn_args = args
        self.result = None
        self.exception = None

    def run(self):
        try:
            self.result = self.fn(*self.fn_args)
        except BaseException as e:  # kept for join(raise_error=True)
            self.exception = e
            raise

    def join(self, timeout=None, raise_error: bool = False):
        super().join(timeout)
        if raise_error and self.exception is not None:
            raise self.exception
