"""Interleaved A/B of libdeig builds on the split3 covariance (deig_syrk_f32_ex,
DEIG_SYRK_SPLIT3) at one shape: ms per op by HIP events on the launch stream, and
whether each build reproduces the first one's S bit for bit (measurement tooling).
usage: python tools/syrk_lib_ab.py reps n d lib [lib ...]   ("shipped" = in-tree build)"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_eigenspaces_amd import _lib, synthetic  # noqa: E402

reps, n, d = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
libs = []
for path in sys.argv[4:]:
    L = ctypes.CDLL(_lib.LIB_PATH if path == "shipped" else path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    libs.append((path, L))
dev = torch.device("cuda", 0)
U = synthetic.planted_basis(d, 64, 0, dev)
X = synthetic.spiked_samples(n, U, seed=1)
nbytes = max(L.deig_syrk_workspace_ex(n, d, 1) for _, L in libs)
ws = torch.empty(nbytes // 4 + 64, dtype=torch.float32, device=dev)
S = {p: torch.empty(d, d, device=dev) for p, _ in libs}
stream = torch.cuda.current_stream(dev)
times = {p: [] for p, _ in libs}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(reps + 1):
    order = libs if r % 2 == 0 else libs[::-1]
    for path, L in order:
        torch.cuda.synchronize()
        e0.record(stream)
        rc = L.deig_syrk_f32_ex(X.data_ptr(), n, d, X.stride(0), ctypes.c_float(1.0 / n),
                                S[path].data_ptr(), d, 1, ws.data_ptr(), nbytes, stream.cuda_stream)
        e1.record(stream)
        e1.synchronize()
        assert rc == 0, L.deig_last_error()
        if r:
            times[path].append(e0.elapsed_time(e1))
    print(f"rep {r} done", flush=True)
ref = S[libs[0][0]]
flop = 3.0 * n * d * (d + 1)
# float64 reference of 64 sampled columns of X^T X / n (chunked over the rows)
cols = torch.randperm(d, generator=torch.Generator().manual_seed(3))[:64].to(dev)
S64 = torch.zeros(d, 64, dtype=torch.float64, device=dev)
for r0 in range(0, n, 1 << 17):
    Xc = X[r0:r0 + (1 << 17)].double()
    S64 += Xc.t() @ Xc[:, cols]
    del Xc
S64 /= n
scale = S64.abs().max().item()
for path, ts in times.items():
    st = sorted(ts)
    med = st[len(st) // 2]
    same = torch.equal(S[path], ref)
    dev_max = (S[path] - ref).abs().max().item()
    err = ((S[path][:, cols].double() - S64).abs().max().item()) / scale
    print(f"{path}: median {med:.2f} ms (min {st[0]:.2f}) = {flop / med / 1e9 / 2.5e3:.4f} of bf16 peak; "
          f"bit-identical to first: {same} (max dev {dev_max:.2e}); max|S - S_f64| / max|S| on 64 columns "
          f"{err:.2e} {[round(t, 2) for t in ts]}")
