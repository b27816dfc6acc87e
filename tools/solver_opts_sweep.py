"""Solver schedule A/B through deig_solver_opts (no rebuild): for the worker shapes of
c1 / c3 / c5, time topk_eigh under several option sets (median of reps, one process)
and check each result against the float64 eigendecomposition of the same S (‖P - P_ref‖_F,
eigenvalues) - the bars are the parity bars (1e-4 / 1e-5).  Measurement tooling.

  python tools/solver_opts_sweep.py [--reps R] [--cases c5,c3] [--variants name:key=val;key=val,...]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = {
    "default": {},
    "fast3e-4": {"fast_until": 3e-4},
    "fast1e-4": {"fast_until": 1e-4},
    "fast1e-4_round1e-5": {"fast_until": 1e-4, "round_until": 1e-5},
    "fast3e-5_round3e-6": {"fast_until": 3e-5, "round_until": 3e-6},
    "round1e-5": {"round_until": 1e-5},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cases", default="c5,c3,c1")
    ap.add_argument("--variants", default="", help="name:key=val;key=val,... (default: the built-in set)")
    a = ap.parse_args()
    variants = VARIANTS
    if a.variants:
        variants = {}
        for item in a.variants.split(","):
            name, _, kv = item.partition(":")
            variants[name] = {k: (int(v) if v.lstrip("-").isdigit() else float(v))
                              for k, v in (x.split("=") for x in kv.split(";") if x)}
    import torch
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import _lib, synthetic
    dev = torch.device("cuda", 0)
    shapes = {"c1": (6250, 3072, 10), "c3": (16384, 8192, 64), "c5": (32768, 16384, 128),
              "c5n": (65536, 16384, 128), "c2": (1 << 20, 3072, 16), "c3n": (1 << 21, 8192, 64),
              "c1b": (6250, 3072, 10)}
    for name in a.cases.split(","):
        n, d, k = shapes[name]
        U = synthetic.planted_basis(d, k, seed=0, device=dev)
        if name == "c1b":  # config 1's uncentered byte covariance (dominant mean direction)
            X = synthetic.spiked_bytes(n, U, seed=1)
            from distributed_eigenspaces_amd import linalg
            S = linalg.sigma_hat_u8(X)
        else:
            X = synthetic.spiked_samples(n, U, seed=1)
            S = de.sigma_hat(X)
        del X
        # float64 reference top-k of the same S (fp64 eigh on the device)
        w, V = torch.linalg.eigh(S.double())
        wr, Vr_ = w[-k:].flip(0), V[:, -k:].flip(1)
        Pr = Vr_ @ Vr_.t() if d <= 8192 else None
        del w, V
        torch.cuda.synchronize()
        for vname, fields in variants.items():
            o = _lib.solver_opts(**fields)
            ts, r = [], None
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r = de.topk_eigh(S, k, check_finite=False, opts=o)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
            Vg = r.V.double()
            if Pr is not None:
                pd = float(torch.linalg.matrix_norm(Vg @ Vg.t() - Pr))
            else:
                sv = torch.linalg.svdvals(Vg.t() @ Vr_).clamp(max=1)
                pd = float(((1 - sv.pow(2)).clamp(min=0).sum() * 2).sqrt())
            ev = float(((r.evals.double().flip(0) - wr).abs() / wr.abs()).max())
            print(json.dumps({"case": name, "variant": vname, "ms": round(statistics.median(ts), 3),
                              "sweeps": r.sweeps, "resid": r.resid, "converged": r.converged,
                              "P_dist": pd, "eval_rel": ev}), flush=True)
        del S, Vr_, Pr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
