"""Interleaved A/B of the split3 covariance op (deig_syrk_f32_ex) across library
builds in ONE process on the same X (box-to-box spread is 3-4 %, so only
interleaved runs compare).  Measurement tooling.

  python tools/syrk_ab.py [--n ROWS] [--d D] [--reps R] LIB [LIB ...]
  (LIB "shipped" = distributed_eigenspaces_amd/libdeig.so)
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _bind(path):
    from distributed_eigenspaces_amd import _lib
    L = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--n", type=int, default=1 << 21)
    ap.add_argument("--d", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from distributed_eigenspaces_amd import _lib, synthetic
    dev = torch.device("cuda", 0)
    paths = [_lib.LIB_PATH if x == "shipped" else x for x in a.libs]
    libs = [_bind(p) for p in paths]
    U = synthetic.planted_basis(a.d, 64, seed=0, device=dev)
    X = synthetic.spiked_samples(a.n, U, seed=1)
    st = torch.cuda.current_stream(dev)
    code = _lib.DEIG_SYRK_SPLIT3
    # one workspace of the largest size for every library (each gets its own size)
    sizes = [L.deig_syrk_workspace_ex(a.n, a.d, code) for L in libs]
    big = torch.empty(max(sizes), dtype=torch.uint8, device=dev)
    wss = [(big, nb) for nb in sizes]
    outs = [torch.empty(a.d, a.d, device=dev) for _ in libs]
    times = [[] for _ in libs]
    for rep in range(a.reps + 1):
        for i, L in enumerate(libs):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            rc = L.deig_syrk_f32_ex(X.data_ptr(), a.n, a.d, a.d, ctypes.c_float(1.0 / a.n), outs[i].data_ptr(),
                                    a.d, code, wss[i][0].data_ptr(), wss[i][1], st.cuda_stream)
            e1.record(st)
            assert rc == 0, rc
            torch.cuda.synchronize()
            if rep:
                times[i].append(e0.elapsed_time(e1))
    ref = outs[0].double()
    for i, p in enumerate(paths):
        diff = float((outs[i].double() - ref).abs().max() / ref.abs().max())
        print(json.dumps({"lib": os.path.relpath(p, ROOT), "ws_GB": round(wss[i][1] / 1e9, 2),
                          "ms_median": statistics.median(times[i]), "ms": [round(t, 2) for t in times[i]],
                          "max_rel_diff_vs_first": diff,
                          "bit_identical_to_first": bool(torch.equal(outs[i], outs[0]))}), flush=True)


if __name__ == "__main__":
    main()
