"""World-size-2 runs of the multi-GPU path with the REAL GPU compute (VERDICT r1:
the CPU gloo tests fake the worker).  Two rank processes share cuda:0 and talk
gloo (the rehearsal backend: ``gather_bases`` / ``broadcast_basis`` bounce the
device tensors through host memory), so every step of the N > 1 path runs: the
rank's block of the distributed.py:99-104 shards, its logical workers' SYRK +
eigensolve on the GPU, the all-gather of the bases in rank order, the server
solve on rank 0 (distributed.py:126-130 + NB:306), and for the streaming variant
the broadcast back to every rank.

The ranks are fresh interpreters (multiprocessing spawn), started by the test
process; results come back as files and are compared with the float64 oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import ref_cpu
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu
P_TOL, EV_TOL = 1e-4, 1e-5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _run_estimator(rank, world, port, wpr, out):
    dist = _init(rank, world, port)
    from distributed_eigenspaces_amd.estimator import DistributedEigenspaceEstimator, rank_shards
    g = load_golden("spiked_d256_k10_m8")
    X = torch.from_numpy(g["X"].astype(np.float32)).cuda()
    mine = rank_shards(X.shape[0], world, rank, wpr)
    lo, hi = mine[0][0], mine[-1][1]
    est = DistributedEigenspaceEstimator(int(g["k"]), workers_per_rank=wpr)
    r = est.fit(X[lo:hi])
    torch.save({"Wt": r.Wt.cpu(), "V": None if r.V is None else r.V.cpu(),
                "evals": None if r.evals is None else r.evals.cpu()},
               os.path.join(out, f"est{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_world2_estimator_real_gpu_workers(tmp_path):
    """2 ranks x 4 logical workers on the golden 8-shard problem == the golden
    (reference-run) server result and the float64 one-shot."""
    if torch.cuda.device_count() < 1:
        pytest.skip("no ROCm GPU visible")
    world, wpr = 2, 4
    mp.spawn(_run_estimator, args=(world, _free_port(), wpr, str(tmp_path)), nprocs=world,
             join=True)
    r0 = torch.load(os.path.join(tmp_path, "est0.pt"), weights_only=True)
    r1 = torch.load(os.path.join(tmp_path, "est1.pt"), weights_only=True)
    assert r1["V"] is None and torch.equal(r0["Wt"], r1["Wt"])  # same gathered stack
    g = load_golden("spiked_d256_k10_m8")
    k = int(g["k"])
    # the golden worker bases are stored in the reference run's arrival (LIFO) order
    by_range = {tuple(int(v) for v in r): i for i, r in enumerate(g["ranges"])}
    shards = ref_cpu.split_batches(g["X"].shape[0], world * wpr)
    for s, (lo, hi) in enumerate(shards):  # rank-major, worker-minor == global shard order
        Vs = r0["Wt"][s * k:(s + 1) * k].t().double().numpy()
        assert ref_cpu.projector_distance(Vs, g["worker_V"][by_range[(lo, hi)]]) <= P_TOL, s
    _, _, sw, sv = ref_cpu.one_shot(g["X"], k, int(g["m"]))
    assert ref_cpu.projector_distance(r0["V"].numpy(), sv) <= P_TOL
    np.testing.assert_allclose(r0["evals"].numpy(), sw, rtol=EV_TOL)


def _oja_data(world, nb, b, d, k):
    rng = np.random.default_rng(11)
    U = np.linalg.qr(rng.standard_normal((d, k)))[0]
    theta = np.linspace(6.0, 3.0, k)
    out = []
    for r in range(world):
        rr = np.random.default_rng(200 + r)
        out.append([(rr.standard_normal((b, d)) + (rr.standard_normal((b, k)) * np.sqrt(theta)) @ U.T)
                    .astype(np.float32) for _ in range(nb)])
    V0 = np.linalg.qr(np.random.default_rng(7).standard_normal((d, k)))[0]
    return out, V0


def _run_oja(rank, world, port, nb, b, d, k, agg, out):
    dist = _init(rank, world, port)
    from distributed_eigenspaces_amd.streaming import StreamingOja
    batches, V0 = _oja_data(world, nb, b, d, k)
    est = StreamingOja(torch.from_numpy(V0).float().cuda(), eta=0.3, agg_every=agg)
    X = torch.from_numpy(np.concatenate(batches[rank])).cuda()
    est.partial_fit_block(X, b)
    torch.save(est.V.contiguous().cpu(), os.path.join(out, f"v{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_world2_streaming_oja_real_gpu(tmp_path):
    """2 ranks: GPU Oja steps, all-gather, GPU server solve on rank 0, broadcast,
    every agg batches == ref_cpu.oja_stream (parity unpinned w.r.t. the reference:
    no Oja there)."""
    if torch.cuda.device_count() < 1:
        pytest.skip("no ROCm GPU visible")
    world, nb, b, d, k, agg = 2, 6, 1024, 256, 6, 3
    mp.spawn(_run_oja, args=(world, _free_port(), nb, b, d, k, agg, str(tmp_path)),
             nprocs=world, join=True)
    v0 = torch.load(os.path.join(tmp_path, "v0.pt"), weights_only=True).numpy()
    v1 = torch.load(os.path.join(tmp_path, "v1.pt"), weights_only=True).numpy()
    np.testing.assert_array_equal(v0, v1)  # every rank adopted the broadcast basis
    batches, V0 = _oja_data(world, nb, b, d, k)
    ref = ref_cpu.oja_stream(batches, V0, 0.3, agg)
    assert ref_cpu.projector_distance(v0, ref) <= P_TOL
