"""Phase timeline of the resident Oja kernel (A/B build with -DDEIG_AB_OJA_TRACE:
tools/ab_libs/libdeig_ojatrace.so): per block and batch, wall_clock64 stamps (10 ns)
at the phase boundaries; prints the median over blocks / batches of each phase.
usage: python tools/oja_trace.py [lib] [d] [k]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributed_eigenspaces_amd import _lib  # noqa: E402

path = sys.argv[1] if len(sys.argv) > 1 else "tools/ab_libs/libdeig_ojatrace.so"
d = int(sys.argv[2]) if len(sys.argv) > 2 else 3072
k = int(sys.argv[3]) if len(sys.argv) > 3 else 32
L = ctypes.CDLL(path)
for name, (res, args) in _lib.SIGNATURES.items():
    f = getattr(L, name)
    f.restype, f.argtypes = res, args
b, nb = 4096, 8
dev = torch.device("cuda", 0)
X = torch.randn(nb * b, d, device=dev)
nbytes = L.deig_oja_workspace(b, d, k)
ws = torch.zeros(nbytes // 4 + 64, dtype=torch.float32, device=dev)
TB = 256 * 64 * 16 * 8
for rep in range(3):
    V = torch.linalg.qr(torch.randn(d, k, device=dev))[0].t().contiguous().t()
    rc = L.deig_oja_steps_ex(X.data_ptr(), nb, b, d, X.stride(0), ctypes.c_float(0.02), V.data_ptr(),
                             k, V.stride(1), nb, _lib.DEIG_OJA_RESIDENT, ws.data_ptr(), nbytes, None)
    assert rc == 0
    torch.cuda.synchronize()
raw = ws.view(torch.uint8)[nbytes - TB:nbytes].cpu().numpy().view(np.uint64).reshape(256, 64, 16)
tr = raw[:, :nb, :].astype(np.int64)
names = ["step1 (X wait + MFMA + P stores)", "signal+wait A", "step2 (P loads, T image)", "signal+wait B",
         "step3 (T load, transposes, Q)", "wait C (wave 7)", "step4 (wave 7)", "-", "wait D",
         "  step3: T fragments land", "  step3: chunk 0 products", "  step3: chunk 0 barrier 1",
         "  step3: chunk 0 sums, barrier 2, chunk 1 products", "  step3: chunk 1 barrier 1",
         "  step3: chunk 1 sums + barrier 2"]
pairs = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (6, 7), None, (8, 9),
         (4, 10), (10, 11), (11, 12), (12, 13), (13, 14), (14, 5)]
for nm, pr in zip(names, pairs):
    if pr is None:
        continue
    dt = (tr[:, 1:, pr[1]] - tr[:, 1:, pr[0]]) * 10 / 1000.0  # us, batches 1..
    print(f"{nm:36s} median {np.median(dt):6.2f} us  p10 {np.percentile(dt, 10):6.2f}  p90 {np.percentile(dt, 90):6.2f}")
per = (tr[:, 2:, 0] - tr[:, 1:-1, 0]) * 10 / 1000.0
print(f"{'batch period (s0 -> s0)':36s} median {np.median(per):6.2f} us")
vl = (tr[:, 2:, 0] - tr[:, 1:-1, 9]) * 10 / 1000.0
print(f"{'V image load (s9 -> next s0)':36s} median {np.median(vl):6.2f} us")
span = (tr[:, nb - 1, 9].max() - tr[:, 0, 0].min()) * 10 / 1000.0
print(f"launch span batches 0..{nb - 1}: {span:.1f} us = {span / nb:.2f} us/batch")
