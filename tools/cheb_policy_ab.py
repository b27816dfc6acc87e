"""Time-to-solution of topk_eigh under Chebyshev start thresholds (deig_solver_opts
cheb_above; < 0 = the library's per-solve default) on planted spectra shaped like the
solver tests' (tests/test_gpu_solver_robust.py) - median of reps, one process, with
sweep counts and the float64 parity check.  Measurement tooling.
usage: python tools/cheb_policy_ab.py [reps]"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import distributed_eigenspaces_amd as de  # noqa: E402
from distributed_eigenspaces_amd import _lib  # noqa: E402
from oracle import ref_cpu  # noqa: E402


def matrix(lams, seed):
    d = len(lams)
    U = np.linalg.qr(np.random.default_rng(seed).standard_normal((d, d)))[0]
    S = ((U * lams) @ U.T).astype(np.float32)
    return (S + S.T) / 2


reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
rng = np.random.default_rng(2)
cases = {
    # tests/test_gpu_solver_robust.py::test_chebyshev_keeps_spiked_sweep_counts
    "spiked_d3072_k16": (np.concatenate([np.linspace(9, 5, 16), np.sort(rng.uniform(0.7, 1.4, 3072 - 16))[::-1]]), 16, 7),
    # ::test_no_guard_columns_p_equals_k (config 5's spike / bulk shape)
    "p_eq_k_d2048_k128": (np.concatenate([np.linspace(9.3, 5.3, 128),
                                          np.sort(np.random.default_rng(3).uniform(0.25, 2.25, 2048 - 128))[::-1]]), 128, 8),
}
for name, (lams, k, seed) in cases.items():
    S = matrix(lams, seed)
    w, V = ref_cpu.top_k_eigh(S.astype(np.float64), k)
    St = torch.from_numpy(S).cuda()
    for vname, above in (("auto", -1.0), ("r04_1e-2", 1e-2)):
        o = _lib.solver_opts(cheb_above=above)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = de.topk_eigh(St, k, opts=o)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        pd = ref_cpu.projector_distance(r.V.cpu().numpy(), V)
        ev = float(np.max(np.abs(r.evals.cpu().numpy() - w) / np.abs(w)))
        print(json.dumps({"case": name, "policy": vname, "ms": round(statistics.median(ts), 3),
                          "sweeps": r.sweeps, "converged": r.converged, "P_dist": pd, "eval_rel": ev}),
              flush=True)
