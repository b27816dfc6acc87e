"""Projector-average solve on a golden set under the solver's env knobs (one
subprocess per setting; knobs are read once per process)."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, ROOT)
    import numpy as np, torch
    import distributed_eigenspaces_amd as de
    from oracle import ref_cpu
    from tests.conftest import golden_names, load_golden
    for name in golden_names():
        g = load_golden(name)
        k, m = int(g["k"]), int(g["m"])
        bases = [torch.from_numpy(v.astype(np.float32)).cuda() for v in g["worker_V"]]
        Wt = de.stack_bases(bases)
        try:
            r = de.projavg_topk(Wt, k, 1.0 / m, q0=bases[0])
            V = r.V.cpu().numpy().astype(np.float64)
            print(f"  {name}: dist={ref_cpu.projector_distance(V, g['server_V']):.2e} "
                  f"sweeps={r.sweeps} resid={r.resid:.2e}", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"  {name}: ERROR {e}", flush=True)
    sys.exit(0)
for env in [{}, {"DEIG_RR_EVERY": "1"}]:
    print(env, flush=True)
    e = dict(os.environ, **env, DEIG_DEBUG="1")
    subprocess.run([sys.executable, __file__, "child"], env=e, check=False, timeout=120)
