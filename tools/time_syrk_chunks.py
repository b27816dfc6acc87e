"""Time split3 SYRK at several row-chunk sizes (workspace-limited chunking) to
measure how much of the kernel is lost to CU drift (each launch restarts every
CU of an XCD at the same K).  usage: python tools/time_syrk_chunks.py [n] [d]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_eigenspaces_amd import _lib, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 19)
d = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
dev = torch.device("cuda", 0)
L = _lib.lib()
U = synthetic.planted_basis(d, 64, 0, dev)
X = synthetic.spiked_samples(n, U, seed=1)
S = torch.empty((d, d), dtype=torch.float32, device=dev)
base = L.deig_syrk_workspace_ex(32, d, _lib.DEIG_SYRK_SPLIT3) - 32 * d * 4
ws = torch.empty(base + n * d * 4, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream().cuda_stream
ref = None
for chunk in [n, n // 4, n // 16, n // 64, 1 << 13]:
    nb = base + chunk * d * 4

    def run():
        rc = L.deig_syrk_f32_ex(X.data_ptr(), n, d, d, ctypes.c_float(1.0 / n), S.data_ptr(), d,
                                _lib.DEIG_SYRK_SPLIT3, ws.data_ptr(), nb, st)
        _lib.check(rc, "syrk")
    run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    if ref is None:
        ref = S.clone()
    rel = float((S - ref).abs().max() / ref.abs().max())
    print(f"chunk {chunk:8d} rows ({n // chunk:3d} launches): {min(ts):8.2f} ms  "
          f"{3 * n * d * (d + 1) / (min(ts) * 1e-3) / 1e12:7.1f} TF/s  max|dS|/max|S| vs 1 chunk {rel:.1e}",
          flush=True)
