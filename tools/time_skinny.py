"""Time the skinny TN kernel (S*Q sweep shape) for several occupancy targets."""
import sys, os, subprocess
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    import torch
    import distributed_eigenspaces_amd as de
    dev = torch.device("cuda", 0)
    d, p = int(sys.argv[2]), int(sys.argv[3])
    S = torch.randn(d, d, device=dev); S = (S + S.t()) / 2
    Q = torch.randn(d, p, device=dev)
    C = de.linalg.gemm_skinny(S, Q, True)
    ref = (S.double().t() @ Q.double())
    err = float((C.double() - ref).abs().max() / ref.abs().max())
    st = torch.cuda.current_stream()
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st); de.linalg.gemm_skinny(S, Q, True, C=C); e1.record(st); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = sorted(ts)[len(ts) // 2]
    fl = 2.0 * d * d * p
    print(f"BPC={os.environ.get('DEIG_SKINNY_BPC')} d={d} p={p}: {ms*1e3:.1f} us  {fl/ms/1e9:.1f} TF/s  {4*d*d/ms/1e6:.0f} GB/s  err={err:.1e}", flush=True)
else:
    for d, p in [(8192, 80), (8192, 64), (3072, 32), (16384, 128)]:
        for bpc in [2, 4, 6, 8]:
            env = dict(os.environ, DEIG_SKINNY_BPC=str(bpc))
            subprocess.run([sys.executable, __file__, "child", str(d), str(p)], env=env, check=True)
