"""Streaming (online) estimator: mini-batch Oja per rank + periodic basis aggregation.

BASELINE.json configs[3] / north_star ("a streaming Oja / mini-batch update for
the online variant"): each rank consumes its own stream of row batches (4096 x
3072 at config 4) and updates its d x k basis with one Oja step per batch
(``linalg.oja_step``: V <- orth(V + eta/b Xb^T (Xb V))).  Every ``agg_every``
batches the ranks exchange bases exactly like the one-shot estimator: one RCCL
all-gather of the fp32 bases (estimator.gather_bases), the server rank takes the
top-k of the projector average (1/m) sum V_i V_i^T with the implicit operator
(distributed.py:126-130 + NB:306, never forming d x d), and broadcasts the result,
which every rank adopts as its next iterate (warm start).

The reference has no Oja code (parity unpinned w.r.t. the reference): the step
and the aggregation schedule are checked against the float64 restatement
``oracle.ref_cpu.oja_stream`` and the estimate by sin(theta) against the planted
subspace.

The collective layer only uses ``torch.distributed``; the per-batch update and
the server solve are injectable so the control flow runs on ``gloo`` with CPU
tensors in the multi-process tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import linalg
from .estimator import comm_tensor, gather_bases

__all__ = ["StreamingOja", "broadcast_basis"]


def _rank_world(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def broadcast_basis(Vt: torch.Tensor, src: int, group=None) -> torch.Tensor:
    """Broadcast a contiguous k x d basis image from ``src`` (in place)."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return Vt
    buf = comm_tensor(Vt, group)  # Vt itself under RCCL, a host copy under gloo
    dist.broadcast(buf, src=src, group=group)
    if buf is not Vt:
        Vt.copy_(buf)
    return Vt


def _gpu_server(Wt: torch.Tensor, k: int, scale: float, q0: torch.Tensor) -> torch.Tensor:
    return linalg.projavg_topk(Wt, k, scale, q0=q0).V


class StreamingOja:
    """Per-rank Oja iterate with periodic projector-average aggregation.

    V0: (d, k) float32 initial basis on the rank's device (any strides; it is
    copied into a column-major buffer).  After ``aggregate()`` every rank holds
    the server's basis, columns in ascending-eigenvalue order.
    """

    def __init__(self, V0: torch.Tensor, eta: float, agg_every: int = 64, server_rank: int = 0,
                 group=None, step_fn=None, server_fn=None, block_fn=None):
        d, k = V0.shape
        self.k = int(k)
        self.V = torch.empty((k, d), dtype=torch.float32, device=V0.device).t()
        self.V.copy_(V0)
        self.eta = float(eta)
        self.agg_every = int(agg_every)
        self.server_rank = int(server_rank)
        self.group = group
        self.step_fn = step_fn or linalg.oja_step
        self.server_fn = server_fn or _gpu_server
        self.block_fn = block_fn or linalg.oja_steps
        self.batches_seen = 0
        self.aggregations = 0

    def partial_fit(self, Xb: torch.Tensor) -> torch.Tensor:
        """One Oja step on a row batch; aggregates every ``agg_every`` batches."""
        self.step_fn(Xb, self.V, self.eta)
        self.batches_seen += 1
        if self.agg_every > 0 and self.batches_seen % self.agg_every == 0:
            self.aggregate()
        return self.V

    def partial_fit_block(self, X: torch.Tensor, batch: int, orth_every: int = 8) -> torch.Tensor:
        """Oja steps over the consecutive row batches of X (rows beyond the last full
        batch are ignored), one ``linalg.oja_steps`` call per run of batches between
        two aggregation points; aggregates exactly where ``partial_fit`` would."""
        nb = X.shape[0] // int(batch)
        i = 0
        while i < nb:
            seg = nb - i
            if self.agg_every > 0:
                seg = min(seg, self.agg_every - self.batches_seen % self.agg_every)
            self.block_fn(X[i * batch:(i + seg) * batch], self.V, self.eta, batch, orth_every)
            self.batches_seen += seg
            i += seg
            if self.agg_every > 0 and self.batches_seen % self.agg_every == 0:
                self.aggregate()
        return self.V

    def aggregate(self) -> torch.Tensor:
        """All-gather the rank bases, server top-k of their projector average,
        broadcast; every rank continues from the aggregated basis."""
        rank, world = _rank_world(self.group)
        Vt = self.V.t()  # contiguous k x d image of the column-major basis
        Wt = gather_bases(Vt.contiguous(), self.group)
        if rank == self.server_rank:
            vbar = self.server_fn(Wt, self.k, 1.0 / world, self.V)
            Vt.copy_(vbar.t())
        broadcast_basis(Vt, self.server_rank, self.group)
        self.aggregations += 1
        return self.V
