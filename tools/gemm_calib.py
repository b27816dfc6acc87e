"""Calibration: what a vendor bf16 GEMM (torch.matmul -> hipBLASLt) reaches on
this box for SYRK-like shapes, to put the covariance kernel's MFMA fraction in
context.  usage: python tools/gemm_calib.py"""
import torch

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream()
for (m, n, k) in [(8192, 8192, 65536), (8192, 8192, 16384), (3072, 3072, 65536)]:
    A = torch.randn((k, m), device=dev, dtype=torch.bfloat16)
    B = torch.randn((k, n), device=dev, dtype=torch.bfloat16)
    C = A.t() @ B
    reps = 10
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        torch.matmul(A.t(), B, out=C)
    e1.record(st)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tf = 2.0 * m * n * k / ms / 1e9
    print(f"bf16 A^T B m={m} n={n} k={k}: {ms:.3f} ms  {tf:.0f} TFLOP/s  ({tf/2500*100:.1f}% of 2.5 PF)", flush=True)
    del A, B, C
