"""Rank-deficient top-k diagnostic (tests/test_gpu_kernels.py::test_topk_rank_deficient)
under the solver's env knobs; one subprocess per setting (knobs are read once)."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, ROOT)
    import numpy as np, torch
    import distributed_eigenspaces_amd as de
    from oracle import ref_cpu
    for n, d, k in [(8, 256, 2), (8, 256, 4), (5, 64, 3)]:
        rng = np.random.default_rng(5)
        X = rng.standard_normal((n, d)).astype(np.float32)
        S = de.sigma_hat(torch.from_numpy(X).cuda())
        r = de.topk_eigh(S, k)
        w, v = ref_cpu.top_k_eigh(ref_cpu.sigma_hat(X.astype(np.float64)), k)
        V = r.V.cpu().numpy()
        print(f"  n={n} d={d} k={k}: dist={ref_cpu.projector_distance(V, v):.2e} "
              f"sweeps={r.sweeps} resid={r.resid:.2e} colnorms={np.linalg.norm(V, axis=0)} "
              f"ev={r.evals.cpu().numpy()} ref={w}", flush=True)
    sys.exit(0)
for env in [{}, {"DEIG_RR_EVERY": "1"}, {"DEIG_SWEEP_ALGO": "fp32"},
            {"DEIG_RR_EVERY": "1", "DEIG_SWEEP_ALGO": "fp32"}]:
    print(env, flush=True)
    e = dict(os.environ, **env, DEIG_DEBUG="1")
    subprocess.run([sys.executable, __file__, "child"], env=e, check=False, timeout=120)
