"""MI355X-native distributed eigenspace estimation (drop-in for TimeEscaper/distributed_eigenspaces).

Hot path (HIP, gfx950, behind the C ABI in include/deig.h):
  * sigma_hat      - covariance SYRK, split-bf16 or f32 MFMA  (distributed.py:59-70)
  * topk_eigh      - block subspace iteration + RR            (distributed.py:22-29)
  * sym_apply      - one solver sweep S Q (split-bf16 MFMA)
  * sym_power      - the solver's chain of sweeps with fused power steps
  * projavg_topk   - implicit projector-average solve         (distributed.py:126-130, NB:306)
  * oja_step(s)    - mini-batch Oja (online variant, config 4); streaming.StreamingOja
                     adds the periodic all-gather / server solve / broadcast

Drop-in modules: ``distributed`` (Node / SlaveNode / MasterNode / run_* / main),
``my_threading`` (Slave) and ``notebook`` (make_batches, top_k_eigenvectors,
compute_segma_hat, online loop).
"""
from .linalg import (EigResult, default_subspace, oja_step, oja_steps, projavg_topk,  # noqa: F401
                     sigma_hat, stack_bases, sym_apply, sym_power, topk_eigh, topk_eigh_batch)

__version__ = "0.1.0"
