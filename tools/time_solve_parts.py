"""Isolated single-stream runs of the c1 worker pieces (for a kernel trace): the u8
covariance of a 6250 x 3072 byte shard and one top-10 solve of it, and one top-128
solve at d = 16384 (config 5's worker), so the Rayleigh-quotient / sweep kernels
are timed without the other workers' streams sharing the GPU."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import distributed_eigenspaces_amd as de
from distributed_eigenspaces_amd import synthetic

dev = torch.device("cuda", 0)
U = synthetic.planted_basis(3072, 10, 0, dev)
X = synthetic.spiked_bytes(6250, U, seed=1)
for _ in range(5):
    S = de.linalg.sigma_hat_u8(X)
torch.cuda.synchronize()
for _ in range(3):
    t0 = time.perf_counter()
    r = de.topk_eigh(S, 10, check_finite=False)
    torch.cuda.synchronize()
    print(f"c1 worker solve: {(time.perf_counter() - t0) * 1e3:.2f} ms, {r.sweeps} sweeps", flush=True)
d, k = 16384, 128
U = synthetic.planted_basis(d, k, 0, dev)
Xs = synthetic.spiked_samples(65536, U, seed=1)
S = de.sigma_hat(Xs)
del Xs
for _ in range(2):
    t0 = time.perf_counter()
    r = de.topk_eigh(S, k, check_finite=False)
    torch.cuda.synchronize()
    print(f"c5 worker solve: {(time.perf_counter() - t0) * 1e3:.2f} ms, {r.sweeps} sweeps", flush=True)
