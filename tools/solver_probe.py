"""Time the worker eigensolver on a spiked shard under solver env knobs (one
subprocess per setting).  usage: python tools/solver_probe.py d n k [KEY=V,KEY=V ...]"""
import os, subprocess, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, ROOT)
    import torch
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import synthetic
    d, n, k = map(int, sys.argv[2:5])
    U = synthetic.planted_basis(d, k, 0, torch.device("cuda", 0))
    X = synthetic.spiked_samples(n, U, seed=1)
    S = de.sigma_hat(X)
    del X
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        r = de.topk_eigh(S, k, check_finite=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        s = torch.linalg.svdvals(U.double().t() @ r.V.double()).min().item()
        print(f"  rep {rep}: {dt*1e3:8.2f} ms sweeps={r.sweeps} resid={r.resid:.2e} "
              f"cos_min={s:.6f} conv={r.converged}", flush=True)
    sys.exit(0)
d, n, k = sys.argv[1:4]
for setting in sys.argv[4:] or [""]:
    env = dict(os.environ)
    for kv in filter(None, setting.split(",")):
        key, _, val = kv.partition("=")
        env[key] = val
    print(f"setting {setting or '(default)'}", flush=True)
    subprocess.run([sys.executable, __file__, "child", d, n, k], env=env, check=False, timeout=300)
