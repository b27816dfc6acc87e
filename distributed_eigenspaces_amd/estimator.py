"""One-shot distributed eigenspace estimator across GPUs (one process per GPU).

The reference distributes shards through a RabbitMQ work queue
(distributed.py:96-143): M contiguous shards of N // M rows (remainder dropped,
:99-104), each worker returns its d x k basis as JSON, the master averages the
projectors (:126-130).  Here:

* shards: the same contiguous split; rank r owns global shards
  [r * W, (r + 1) * W) for W = workers_per_rank logical workers (they run back to
  back on the rank's GPU - each SYRK fills the chip);
* exchange: ONE collective - an all-gather of the fp32 bases (k x d rows each,
  i.e. the column-major d x k bytes) over RCCL/xGMI into Wt = [V_1^T; ...; V_M^T];
* server: the implicit projector-average top-k on ``server_rank`` (GPU 0),
  warm-started from V_1; the d x d average is never formed.

The collective layer only uses ``torch.distributed`` with tensors on the rank's
device, so it runs on ``gloo`` with CPU tensors too (multi-process tests); the
per-worker compute is injectable for those tests and defaults to the GPU ops.
"""
from __future__ import annotations

import inspect
from dataclasses import dataclass

import torch
import torch.distributed as dist

from . import linalg

__all__ = ["shard_ranges", "rank_shards", "EstimatorResult", "DistributedEigenspaceEstimator",
           "gather_bases"]


def shard_ranges(n_rows: int, batches_number: int):
    """distributed.py:99-104: M contiguous (lo, hi) ranges of N // M rows."""
    step = n_rows // batches_number
    return [(i * step, (i + 1) * step) for i in range(batches_number)]


def rank_shards(n_rows: int, world: int, rank: int, workers_per_rank: int = 1):
    """The global shard ranges owned by ``rank`` (contiguous block of shards)."""
    allr = shard_ranges(n_rows, world * workers_per_rank)
    return allr[rank * workers_per_rank:(rank + 1) * workers_per_rank]


def comm_tensor(t: torch.Tensor, group=None) -> torch.Tensor:
    """The tensor the process group's backend moves for ``t``: ``t`` itself (RCCL
    moves device tensors over xGMI; gloo moves host tensors), or a host copy of a
    device tensor under gloo (the multi-rank rehearsal, several ranks sharing one
    GPU).  The collective calls are the same on both backends; only this staging
    differs."""
    if t.is_cuda and dist.get_backend(group) != "nccl":
        return t.cpu()
    return t


def gather_bases(Wt_local: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather the per-rank stacks of bases ((W k) x d each) in rank order: ONE
    ``all_gather_into_tensor`` (ncclAllGather under RCCL) into Wt = [V_1^T; ...; V_M^T]."""
    if not dist.is_available() or not dist.is_initialized():
        return Wt_local
    world = dist.get_world_size(group)
    if world == 1:
        return Wt_local
    src = comm_tensor(Wt_local.contiguous(), group)
    out = torch.empty((world * src.shape[0], src.shape[1]), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src, group=group)
    return out.to(Wt_local.device)


@dataclass
class EstimatorResult:
    evals: torch.Tensor | None     # (k,) ascending, server rank only
    V: torch.Tensor | None         # (d, k) column-major, server rank only
    Wt: torch.Tensor               # gathered bases ((M k) x d)
    worker_evals: list             # this rank's workers' eigenvalues
    sweeps_worker: list
    sweeps_server: int


def _batch_accepts(solver_kw: dict) -> bool:
    """The batched worker solve takes these solver options (topk_eigh_batch has no
    per-problem warm start q0, for one): others fall back to the serial worker loop,
    which passes them to topk_eigh as before."""
    params = inspect.signature(linalg.topk_eigh_batch).parameters
    return all(key in params and key not in ("Ss", "k") for key in solver_kw)


def _gpu_worker(x: torch.Tensor, k: int, **kw):
    S = linalg.sigma_hat(x)
    r = linalg.topk_eigh(S, k, check_finite=False, **kw)
    return r.V, r.evals, r.sweeps


class DistributedEigenspaceEstimator:
    def __init__(self, k: int, workers_per_rank: int = 1, server_rank: int = 0, group=None,
                 worker_fn=None, solver_kw=None, concurrent_workers: bool = False,
                 batched_workers: bool = True):
        self.k = int(k)
        self.wpr = int(workers_per_rank)
        # concurrent_workers (default GPU worker, W > 1): covariances back to back on
        # the caller's stream, each worker's eigensolve in a my_threading.Slave
        # thread on its own HIP stream, chained by an event (bench.py's c5 mode).
        self.concurrent = bool(concurrent_workers) and worker_fn is None
        # batched_workers (default GPU worker, W > 1, unless concurrent_workers): the W
        # covariances back to back, then ONE batched solve (linalg.topk_eigh_batch:
        # same results as W topk_eigh calls, the small Rayleigh-Ritz solves of all
        # workers in one launch per step).
        self.batched = bool(batched_workers) and worker_fn is None and not self.concurrent
        self.server_rank = server_rank
        self.group = group
        self.worker_fn = worker_fn or _gpu_worker
        self.solver_kw = dict(solver_kw or {})

    def _rank_world(self):
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(self.group), dist.get_world_size(self.group)
        return 0, 1

    def local_bases(self, X_local: torch.Tensor):
        """Run this rank's logical workers on contiguous pieces of X_local."""
        parts = shard_ranges(X_local.shape[0], self.wpr)
        if self.concurrent and len(parts) > 1 and X_local.is_cuda:
            return self._local_bases_concurrent(X_local, parts)
        if self.batched and len(parts) > 1 and X_local.is_cuda and _batch_accepts(self.solver_kw):
            Ss = [linalg.sigma_hat(X_local[lo:hi]) for lo, hi in parts]
            rs = linalg.topk_eigh_batch(Ss, self.k, check_finite=False, **self.solver_kw)
            return (torch.cat([r.V.t() for r in rs], dim=0).contiguous(), [r.evals for r in rs],
                    [r.sweeps for r in rs])
        rows, evs, sw = [], [], []
        for lo, hi in parts:
            V, ev, s = self.worker_fn(X_local[lo:hi], self.k, **self.solver_kw)
            rows.append(V.t())  # k x d view of the column-major basis
            evs.append(ev)
            sw.append(s)
        return torch.cat(rows, dim=0).contiguous(), evs, sw

    def _local_bases_concurrent(self, X_local: torch.Tensor, parts):
        from .my_threading import Slave
        dev = X_local.device
        main = torch.cuda.current_stream(dev)
        slaves = []
        try:
            for lo, hi in parts:
                S = linalg.sigma_hat(X_local[lo:hi])
                ev = torch.cuda.Event()
                ev.record(main)
                st = torch.cuda.Stream(dev)
                S.record_stream(st)

                def solve(S=S, ev=ev, st=st):
                    with torch.cuda.stream(st):
                        st.wait_event(ev)
                        r = linalg.topk_eigh(S, self.k, check_finite=False, **self.solver_kw)
                        st.synchronize()
                    return r

                sl = Slave(solve)
                sl.start()
                slaves.append((sl, st))
        finally:
            # every started solve is joined before anything propagates (no orphaned
            # threads still launching on their streams)
            for sl, _ in slaves:
                sl.join()
        errors = [sl.exception for sl, _ in slaves if sl.exception is not None]
        if errors:
            raise errors[0]
        rows, evs, sw = [], [], []
        for sl, st in slaves:
            main.wait_stream(st)
            r = sl.result
            # both outputs were allocated on the side stream; the main stream reads them
            r.V.record_stream(main)
            r.evals.record_stream(main)
            rows.append(r.V.t())
            evs.append(r.evals)
            sw.append(r.sweeps)
        return torch.cat(rows, dim=0).contiguous(), evs, sw

    def server(self, Wt: torch.Tensor, batches_number: int):
        q0 = Wt[: self.k].t()
        return linalg.projavg_topk(Wt, self.k, 1.0 / batches_number, q0=q0, **self.solver_kw)

    def fit(self, X_local: torch.Tensor) -> EstimatorResult:
        rank, world = self._rank_world()
        Wt_local, evs, sw = self.local_bases(X_local)
        Wt = gather_bases(Wt_local, self.group)
        m = world * self.wpr
        if rank == self.server_rank:
            r = self.server(Wt, m)
            return EstimatorResult(r.evals, r.V, Wt, evs, sw, r.sweeps)
        return EstimatorResult(None, None, Wt, evs, sw, 0)
