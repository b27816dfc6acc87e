"""Run the config-3 shard SYRK (2^21 x 8192) twice (for PMC / trace passes)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import distributed_eigenspaces_amd as de
from distributed_eigenspaces_amd import synthetic
dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 21)
d = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
U = synthetic.planted_basis(d, 64, 0, dev)
X = synthetic.spiked_samples(n, U, seed=1)
S = de.sigma_hat(X)
de.sigma_hat(X, out=S)
torch.cuda.synchronize()
print("ok", n, d, flush=True)
