"""World-size-2 gloo test of the multi-GPU path's host logic on CPU: shard ownership
(distributed.py:99-104 split across ranks) and the all-gather of bases in rank order.
The per-worker GPU compute is replaced by a deterministic fake."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_eigenspaces_amd.estimator import (DistributedEigenspaceEstimator, gather_bases,
                                                   rank_shards, shard_ranges)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_worker(x, k, **kw):
    d = x.shape[1]
    V = torch.zeros((d, k))
    V[:, 0] = x[0]          # first row of the shard identifies it
    V[0, 1 % k] = x.shape[0]
    return V, torch.arange(k, dtype=torch.float32), 1


def _run(rank, world, port, n, d, k, wpr, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = torch.arange(n * d, dtype=torch.float32).reshape(n, d)
    mine = rank_shards(n, world, rank, wpr)
    lo, hi = mine[0][0], mine[-1][1]
    est = DistributedEigenspaceEstimator(k, workers_per_rank=wpr, worker_fn=_fake_worker)
    Wt_local, evs, sw = est.local_bases(data[lo:hi])
    Wt = gather_bases(Wt_local)
    torch.save(Wt, os.path.join(out, f"wt{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_gather_order(tmp_path):
    world, n, d, k, wpr = 2, 103, 8, 2, 2
    port = _free_port()
    mp.spawn(_run, args=(world, port, n, d, k, wpr, str(tmp_path)), nprocs=world, join=True)
    W0 = torch.load(os.path.join(tmp_path, "wt0.pt"), weights_only=True)
    W1 = torch.load(os.path.join(tmp_path, "wt1.pt"), weights_only=True)
    assert torch.equal(W0, W1)
    data = torch.arange(n * d, dtype=torch.float32).reshape(n, d)
    shards = shard_ranges(n, world * wpr)
    assert W0.shape == (world * wpr * k, d)
    # rank-major, worker-minor order == global shard order of distributed.py:99-104
    for s, (lo, hi) in enumerate(shards):
        np.testing.assert_array_equal(W0[s * k].numpy(), data[lo].numpy())
    # each rank's local split of its block reproduces the global split when
    # the global row count is a multiple of world * wpr; otherwise the rank block
    # is what rank_shards assigned
    assert rank_shards(n, world, 1, wpr) == shards[2:4]


def _oja_batches(rank, nb, b, d):
    rng = np.random.default_rng(100 + rank)
    scale = np.linspace(3.0, 1.0, d)
    return [(rng.standard_normal((b, d)) * scale).astype(np.float32) for _ in range(nb)]


def _cpu_oja_step(Xb, V, eta):
    """CPU stand-in for linalg.oja_step (float32): V <- qr(V + eta/b Xb^T Xb V)."""
    v = V.double() + eta * (Xb.double().t() @ (Xb.double() @ V.double())) / Xb.shape[0]
    V.copy_(torch.linalg.qr(v)[0])


def _cpu_server(Wt, k, scale, q0):
    from oracle import ref_cpu
    W = Wt.double().numpy()
    Vs = [W[i * k:(i + 1) * k].T for i in range(W.shape[0] // k)]
    _, v = ref_cpu.top_k_eigh(ref_cpu.projector_average(Vs, 1) * scale, k)
    return torch.from_numpy(v).float()


def _run_oja(rank, world, port, nb, b, d, k, agg, out):
    from distributed_eigenspaces_amd.streaming import StreamingOja
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    V0 = torch.linalg.qr(torch.from_numpy(np.random.default_rng(7).standard_normal((d, k))))[0]
    est = StreamingOja(V0.float(), eta=0.3, agg_every=agg, step_fn=_cpu_oja_step,
                       server_fn=_cpu_server)
    for xb in _oja_batches(rank, nb, b, d):
        est.partial_fit(torch.from_numpy(xb))
    torch.save(est.V.contiguous(), os.path.join(out, f"v{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_streaming_oja_aggregation(tmp_path):
    """Streaming Oja control flow (gather -> server solve -> broadcast every
    agg_every batches) on 2 gloo ranks == the float64 restatement oja_stream."""
    from oracle import ref_cpu
    world, nb, b, d, k, agg = 2, 4, 64, 12, 3, 2
    port = _free_port()
    mp.spawn(_run_oja, args=(world, port, nb, b, d, k, agg, str(tmp_path)), nprocs=world,
             join=True)
    V0r = torch.load(os.path.join(tmp_path, "v0.pt"), weights_only=True).numpy()
    V1r = torch.load(os.path.join(tmp_path, "v1.pt"), weights_only=True).numpy()
    np.testing.assert_array_equal(V0r, V1r)  # every rank adopted the broadcast basis
    V0 = np.linalg.qr(np.random.default_rng(7).standard_normal((d, k)))[0]
    ref = ref_cpu.oja_stream([_oja_batches(r, nb, b, d) for r in range(world)], V0, 0.3, agg)
    assert ref_cpu.projector_distance(V0r, ref) <= 1e-5


def test_shard_ranges_match_reference_split():
    from oracle import ref_cpu
    for n, m in [(60000, 8), (503, 5), (7, 8), (16777216, 8)]:
        assert shard_ranges(n, m) == ref_cpu.split_batches(n, m)
