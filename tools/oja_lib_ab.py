"""Interleaved A/B of libdeig variants on the config-4 Oja op (64 batches of 4096 x 3072,
k = 32, DEIG_OJA_AUTO): us per batch by HIP events, and whether each build reproduces the
first one's basis bit for bit.
usage: python tools/oja_lib_ab.py reps orth_every lib [lib ...]   ("shipped" = the in-tree build)"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_eigenspaces_amd import _lib  # noqa: E402

reps, orth = int(sys.argv[1]), int(sys.argv[2])
libs = []
for path in sys.argv[3:]:
    L = ctypes.CDLL(_lib.LIB_PATH if path == "shipped" else path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    libs.append((path, L))
b, d, k, nb = 4096, 3072, 32, 64
dev = torch.device("cuda", 0)
X = torch.randn(nb * b, d, device=dev)
V0 = torch.linalg.qr(torch.randn(d, k, device=dev, dtype=torch.float64))[0].float()
nbytes = max(L.deig_oja_workspace(b, d, k) for _, L in libs)
ws = torch.zeros(nbytes // 4 + 64, dtype=torch.float32, device=dev)
times = {p: [] for p, _ in libs}
outs = {}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(reps + 1):
    order = libs if r % 2 == 0 else libs[::-1]
    for path, L in order:
        V = V0.t().contiguous().t()
        torch.cuda.synchronize()
        e0.record()
        rc = L.deig_oja_steps_f32(X.data_ptr(), nb, b, d, X.stride(0), ctypes.c_float(0.02), V.data_ptr(),
                                  k, V.stride(1), orth, ws.data_ptr(), nbytes, None)
        e1.record()
        e1.synchronize()
        assert rc == 0
        if r:
            times[path].append(e0.elapsed_time(e1) / nb * 1e3)
        outs[path] = V
ref = outs[libs[0][0]]
for path, ts in times.items():
    st = sorted(ts)
    print(f"{path}: median {st[len(st) // 2]:.2f} us/batch (min {st[0]:.2f}) bit-identical to first: "
          f"{torch.equal(outs[path], ref)} finite: {bool(torch.isfinite(outs[path]).all())} "
          f"{[round(t, 2) for t in ts]}")
