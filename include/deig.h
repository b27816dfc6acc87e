/*
 * deig.h - C ABI of libdeig.so, the MI355X (gfx950) hot path of the distributed
 * eigenspace estimator (TimeEscaper/distributed_eigenspaces).
 *
 * Every entry point takes raw device pointers, sizes and leading dimensions (in
 * elements), caller-provided device workspace and a hipStream_t (passed as
 * void*).  The library never allocates or frees device memory.  Its only
 * process-global state is thread-safe: a thread-local error string, a per-device
 * CU-count cache (atomics) and a mutex-protected free list of small pinned host
 * blocks (a few hundred bytes each, allocated on first use and kept) that the
 * eigensolvers read their per-cycle status from.  Work is enqueued on
 * the given stream; entry points that iterate (the eigensolvers) synchronise that
 * stream between sweeps to test convergence, and return when done.
 *
 * Layouts: sample matrices X are row-major n x d (row stride ldx); symmetric
 * matrices S are row-major d x d (full storage, both triangles written); bases V
 * are COLUMN-major d x k (Fortran order, column stride ldv), columns in ASCENDING
 * eigenvalue order, exactly like LAPACK ?syevr / scipy.linalg.eigh.  A stack of m
 * bases is passed as Wt = [V_1^T; ...; V_m^T], i.e. (m*k) x d row-major, which is
 * the byte layout of m column-major d x k bases laid end to end.
 *
 * Return codes: 0 ok; DEIG_NOT_CONVERGED (1) = results written but the residual
 * test did not pass within max_sweeps; negative = error (see deig_last_error()).
 */
#ifndef DEIG_H
#define DEIG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DEIG_OK 0
#define DEIG_NOT_CONVERGED 1
#define DEIG_EINVAL (-1)
#define DEIG_EHIP (-2)
#define DEIG_EWORKSPACE (-3)
#define DEIG_ETIMEOUT (-4) /* a resident Oja hand-off timed out (deig_oja_error) */

/* Element types of float inputs (deig_syrk_shift, deig_topk_sym_ex). */
#define DEIG_F32 0
#define DEIG_F64 1

/* Library version, e.g. 0x000400 for 0.4.0.  A caller built against an older header
 * should compare it with the version it was built for before binding entry points
 * whose signature changed (deig_topk_sym_batch: see below). */
int deig_version(void);

/* Release the library's process-lifetime host resources (the pinned per-cycle status
 * blocks of the eigensolvers) after synchronising the current device.  Optional; call
 * it at process exit BEFORE the HIP runtime is torn down (the Python binding registers
 * it with atexit, which runs before the C runtime's exit handlers).  No solver may be
 * running; later solver calls allocate new blocks. */
void deig_shutdown(void);

/* Thread-local message for the last nonzero return on this thread ("" if none). */
const char* deig_last_error(void);

/* Covariance algorithms (deig_syrk_f32_ex):
 *  DEIG_SYRK_SPLIT3: each fp32 sample split once into bf16 hi + lo; products
 *    from 3 bf16 MFMAs (hi*hi + hi*lo + lo*hi), fp32 accumulation, the dropped
 *    lo*lo term restored exactly on the diagonal.  Per-product error <= ~3*2^-16
 *    relative, zero-mean, so it averages out over rows: max |S - S_f64| / max|S|
 *    ~1e-6 at n = 512, ~2e-7 at n >= 32k (fp32 kernel: ~1e-7..2e-6), at 16/3 x
 *    the f32 MFMA rate.
 *  DEIG_SYRK_FP32: v_mfma_f32_32x32x2_f32 (exact fp32 fma chain).
 *  DEIG_SYRK_AUTO (default): SPLIT3 for n >= DEIG_SYRK_SPLIT_MIN_ROWS, else FP32. */
#define DEIG_SYRK_AUTO 0
#define DEIG_SYRK_SPLIT3 1
#define DEIG_SYRK_FP32 2
#define DEIG_SYRK_DEFAULT DEIG_SYRK_AUTO
#define DEIG_SYRK_SPLIT_MIN_ROWS 1024
/* OR-ed into the algorithm of deig_syrk_f32_ex (SPLIT3 only): S += alpha X^T X -
 * one covariance streamed through in row blocks (e.g. a shard larger than HBM). */
#define DEIG_SYRK_ACCUMULATE 0x100

/* Sigma_hat = alpha * X^T X  (alpha = 1/n reproduces the reference).
 * Replaces SlaveNode.compute_sigma_hat_  distributed.py:59-70
 * (np.zeros((d,d)) += np.dot(x.T, x); /= n  ->  OpenBLAS dsyrk).
 * fp32 in, fp32 accumulate (DEIG_SYRK_DEFAULT); output is bit-exactly symmetric.
 * Requires n >= 1, d % 4 == 0, ldx % 4 == 0, lds % 4 == 0, 16-byte aligned X, S.
 * The workspace query returns the recommended size; SPLIT3 works on row chunks
 * that fit the workspace given (more workspace -> fewer, larger chunks). */
int deig_syrk_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float alpha,
                  float* S, int64_t lds, void* ws, size_t ws_bytes, void* stream);
size_t deig_syrk_workspace(int64_t n, int64_t d);
/* Same with an explicit algorithm (DEIG_SYRK_*). */
int deig_syrk_f32_ex(const float* X, int64_t n, int64_t d, int64_t ldx, float alpha,
                     float* S, int64_t lds, int algo, void* ws, size_t ws_bytes, void* stream);
size_t deig_syrk_workspace_ex(int64_t n, int64_t d, int algo);

/* Mean-shifted covariance of float samples, float64 result (the reference's own
 * float64 data flow: distributed.py:169-173 grey values -> compute_sigma_hat_
 * :59-70):  S64 = alpha * X^T X  computed as
 *   alpha [ C^T C + s mu^T + mu s^T + n mu mu^T ],  mu = column means (double),
 *   C = fl32(X - mu), s = sum_r (x_r - mu) (double)
 * with C^T C on the split3 / fp32 SYRK (n >= / < DEIG_SYRK_SPLIT_MIN_ROWS): the
 * SYRK's rounding is then relative to the CENTRED data, not to the mean direction
 * that dominates an uncentered covariance of byte images (see shift.hip for the
 * measured effect on the top-k basis).  X: n x d row-major, element type xtype
 * (DEIG_F32 / DEIG_F64), row stride ldx elements, aligned to its element size.
 * S64 (float64, lds64) and/or S (its fp32 rounding, lds) may be NULL (not both);
 * both triangles are written (bit-exact symmetry).
 * Workspace: deig_syrk_shift_workspace(n, d, xtype) (holds an fp32 copy of C). */
int deig_syrk_shift(const void* X, int xtype, int64_t n, int64_t d, int64_t ldx, double alpha,
                    double* S64, int64_t lds64, float* S, int64_t lds, void* ws, size_t ws_bytes,
                    void* stream);
size_t deig_syrk_shift_workspace(int64_t n, int64_t d, int xtype);

/* Exact covariance of uint8 samples (fused ingest):
 *   S = alpha * V^T V,  V the n x d feature matrix of
 *   DEIG_U8_RAW:   v = x, the first d bytes of each row (e.g. raw CIFAR rows, d = 3072);
 *   DEIG_U8_GRAY3: v = (r + g + b) / 3 of d interleaved 3-byte pixels (row needs 3d
 *                  bytes) - the reference's grayscale + flatten, distributed.py:170-173
 *                  (data.mean(axis=3), reshape), fused into the covariance.
 * Replaces compute_sigma_hat_ (distributed.py:59-70) on the uint8 CIFAR bytes of
 * load_data.py:18-33 (alpha = 1/n reproduces the reference).  Every product and
 * sum is exact (int8 MFMA with int32 accumulation, int64 combination), so S64 is the
 * reference's float64 result rounded once (alpha = 1/n: one division of the exact
 * integer sum) and S its fp32 rounding (within 1 ulp of the correctly rounded
 * value); either may be NULL (not both); both triangles are
 * written (bit-exact symmetry).  Requires d % 4 == 0, d <= 32768, ldx % 4 == 0 bytes,
 * X 4-byte aligned.  Workspace: deig_syrk_u8_workspace(n, d, mode). */
#define DEIG_U8_RAW 0
#define DEIG_U8_GRAY3 1
int deig_syrk_u8(const uint8_t* X, int64_t n, int64_t d, int64_t ldx, int mode, double alpha,
                 float* S, int64_t lds, double* S64, int64_t lds64, void* ws, size_t ws_bytes,
                 void* stream);
size_t deig_syrk_u8_workspace(int64_t n, int64_t d, int mode);

/* Subspace size the solvers use for a given k when the caller passes p <= 0. */
int deig_default_subspace(int64_t d, int k);

/* Sweep algorithms for the symmetric S*Q product of the eigensolver:
 *  DEIG_SWEEP_BF16X6: S rows and Q split into three bf16 pieces in registers
 *    (x = h + m + l), 6 bf16 MFMA products per fp32 product (every term down to
 *    2^-16 |ab|), fp32 accumulation - fp32-grade products, HBM-bound on the 4 d^2
 *    bytes of S for every p <= 128;
 *  DEIG_SWEEP_FP32: f32 MFMA skinny kernel (exact fp32 fma chain, f32-MFMA-bound
 *    above p ~ 40);
 *  DEIG_SWEEP_AUTO: BF16X6 (the solvers' default; deig_solver_opts.sweep_algo). */
#define DEIG_SWEEP_AUTO 0
#define DEIG_SWEEP_BF16X6 1
#define DEIG_SWEEP_FP32 2
/* OR-ed into the algorithm of deig_sym_apply_f32 (BF16X6 only): the workspace
 * already holds the sweep image of this S from an earlier call with the same
 * S, d, p and workspace, so the re-layout pass is skipped (repeated products
 * with one S, as the solver does). */
#define DEIG_SWEEP_PREPARED 0x100
/* OR-ed into the algorithm of deig_sym_apply_f32 (BF16X6 only): the solver's
 * mode.  Q (then written in place) is rounded to Q' = h + m, its two leading
 * bf16 pieces (16 significant bits, |Q' - Q| <= 2^-17 |Q|), and Y = alpha S Q'
 * is formed to fp32 grade from five bf16 MFMA products instead of six. */
#define DEIG_SWEEP_ROUND_Q 0x200
/* OR-ed into the algorithm of deig_sym_apply_f32 (BF16X6 only; implies ROUND_Q):
 * the solver's early-sweep mode.  S is also taken as its two leading bf16 pieces
 * (from a two-piece image written by the same prepare pass), so Y = alpha S' Q' is
 * three bf16 MFMA products (hh + hm + mh) with no split in the sweep: ~2^-16
 * relative (S' rounding 2^-17, dropped m m 2^-18).  deig_topk_sym_f32 uses it while
 * its residual is above 1e-3 (after the one-product HALF sweeps above 1e-2), ROUND_Q
 * down to 1e-4, the exact product below. */
#define DEIG_SWEEP_FAST 0x400
/* OR-ed into the algorithm of deig_sym_apply_f32 / deig_sym_power_f32 (BF16X6 only;
 * implies FAST): the solver's first sweeps.  S and Q are both taken as their leading
 * bf16 piece alone (the h slots of the two-piece image: half its bytes), one bf16
 * MFMA product per fragment pair, ~2^-9 relative.  Needs p >= 64 (below, the FAST
 * mode runs).  deig_topk_sym_f32 uses it while its residual is above
 * deig_solver_opts.half_until (1e-2). */
#define DEIG_SWEEP_HALF 0x1000
/* OR-ed into the algorithm of deig_sym_apply_f32 (BF16X6 only; measurement):
 * launch the sweep kernel alone on the Q image that the previous call with the
 * same workspace, d, p and mode left - no split of Q, no split-K reduction, Y is
 * not written.  Timing such calls gives the sweep kernel's own duration. */
#define DEIG_SWEEP_KERNEL_ONLY 0x800

/* One subspace-iteration sweep Y = alpha * S Q  (S symmetric d x d row-major, lds;
 * Q d x p row-major, ldq; Y d x p row-major, ldy; p % 16 == 0, 16 <= p <= 128).
 * The S*Q product inside deig_topk_sym_f32, exposed for measurement and reuse. */
int deig_sym_apply_f32(const float* S, int64_t d, int64_t lds, const float* Q, int p,
                       int64_t ldq, float* Y, int64_t ldy, float alpha, int algo, void* ws,
                       size_t ws_bytes, void* stream);
size_t deig_sym_apply_workspace(int64_t d, int p, int algo);

/* `steps` sweeps of the solver's power chain (the sweeps between two Rayleigh-Ritz
 * steps of deig_topk_sym_f32): for i = 0 .. steps-1:  Y = S Q;  Q_j <- cs_j Y_j
 * for every column with cs_j > 0 (the others keep Q_j).  cs: p floats in device
 * memory.  Each basis step is fused into the sweep's split-K reduction together
 * with the next sweep's Q image, as inside the solver, so the time per step is
 * the solver's cost per sweep.  On return Y = S Q_{steps-1} and Q = Q_steps
 * (ROUND_Q / FAST: every Q rounded to two bf16 pieces as for deig_sym_apply_f32).
 * algo: DEIG_SWEEP_BF16X6 / AUTO with the PREPARED / ROUND_Q / FAST flags; the
 * workspace is deig_sym_apply_workspace's.  Extends the sweep entry point (no
 * reference counterpart: the reference solves with LAPACK, distributed.py:22-29). */
int deig_sym_power_f32(const float* S, int64_t d, int64_t lds, float* Q, int p, int64_t ldq,
                       float* Y, int64_t ldy, const float* cs, int steps, int algo, void* ws,
                       size_t ws_bytes, void* stream);

/* Options of the eigensolvers (deig_topk_sym_ex, deig_projavg_topk_ex).  Fill with
 * deig_solver_opts_init() and change fields; NULL options = the defaults.  These
 * replace the r02 environment knobs: the library reads no environment variables. */
typedef struct deig_solver_opts {
  int size;                  /* sizeof(deig_solver_opts), set by deig_solver_opts_init */
  int sweep_algo;            /* DEIG_SWEEP_AUTO (bf16x6 sweeps over an image of S) or
                                DEIG_SWEEP_FP32 (f32-MFMA skinny products; float32 S only) */
  int rr_every;              /* sweeps per Rayleigh-Ritz step before the Chebyshev filter
                                starts (0: 4 with >= 16 guard columns, else 2) */
  int chebyshev;             /* 1 (default): Chebyshev filter once resid <= cheb_above */
  float cheb_above;          /* < 0 (default): 1.0 - the filter from the first Rayleigh-Ritz
                                step on - for a single-block solve of an explicit S (k <= 128)
                                on a basis without guard columns (p - k < 4), else 1e-2 */
  int deflate;               /* 1 (default): lock dominant pairs (theta_1 >= 64 theta_k) and
                                iterate the rest on the deflated operator */
  int deflate_early;         /* 1 (default): lock them as soon as they are converged */
  int jacobi_early_sweeps;   /* Jacobi sweeps of early Rayleigh-Ritz steps (-1: 2 explicit S,
                                3 projector average; 0: uncapped) */
  float jacobi_early_above;  /* residual above which the cap applies (< 0: 1e-4 / 1e-2) */
  float fast_until;          /* three-product sweeps while resid > this (1e-3; 0: never) */
  float round_until;         /* five-product sweeps while resid > this (1e-4) */
  int debug;                 /* 1: per-Rayleigh-Ritz trace on stderr */
  float half_until;          /* one-product sweeps (DEIG_SWEEP_HALF) while resid > this,
                                for d >= 2048 and p >= 64 (1e-2; 0: never) */
} deig_solver_opts;
void deig_solver_opts_init(deig_solver_opts* opts);

/* Top-k eigenpairs of a dense symmetric S (d x d, row-major, lds), ascending.
 * Replaces Node.top_k_eigenvectors  distributed.py:22-29
 * (scipy.linalg.eigh(S, eigvals=(d-k, d-1))[1]  ->  LAPACK dsyevr), plus the
 * eigenvalues ([0] of the same call) as a side output.
 * Any d >= 1, any 1 <= k <= d and any symmetric S, like ?syevr.  S is read in place
 * when d % 4 == 0, d >= 16 and the subspace fits in d (then lds % 4 == 0 and a 16-byte
 * aligned S are required); otherwise it is staged as a zero-padded copy in the
 * workspace (any lds >= d, element alignment) whose padding never enters the
 * iteration or the result (deig_topk_workspace_ex accounts for it).
 * Block subspace iteration with Rayleigh-Ritz on a p-dimensional subspace
 * (k <= p <= 128, p % 16 == 0, p <= d; k > 128: blocks of p - 16 pairs on a p-column
 * subspace, p = 128 by default, each block's pairs LOCKED and deflated out of S for
 * the blocks below); between Rayleigh-Ritz steps a scaled Chebyshev filter on [0, c]
 * (c from the Ritz values; power steps while the residual is above 1e-2).  An
 * indefinite S is detected by the Ritz values (a negative one of significant size)
 * and solved as S + sigma I (the eigenvalues returned are S's).  When theta_1 >=
 * 64 theta_k (an uncentered covariance's mean direction), the dominant pairs are
 * locked and the others iterated on S - V_D L_D V_D^T (formed in double: fp32
 * products S q would otherwise lose their digits to cancellation).  Q0 (d x k0
 * column-major, ldq0) is an optional warm start for k <= 128 (NULL / k0 = 0 ->
 * deterministic pseudo-random start).  Stops when
 * max_j ||S v_j - lambda_j v_j|| <= tol * |lambda_max| (or the residual stalls
 * within 4 tol / 2e-6 of it, the fp32 floor); returns DEIG_NOT_CONVERGED after
 * max_sweeps sweeps (per block), or earlier when it stalls above that floor.
 * Outputs: V (d x k col-major, ldv), evals (k, ascending), *sweeps_out,
 * *resid_out = final max relative residual (host pointers, may be NULL). */
int deig_topk_sym_f32(const float* S, int64_t d, int64_t lds, int k, int p,
                      int max_sweeps, float tol, const float* Q0, int k0, int64_t ldq0,
                      float* V, int64_t ldv, float* evals, int* sweeps_out,
                      float* resid_out, void* ws, size_t ws_bytes, void* stream);
size_t deig_topk_workspace(int64_t d, int k, int p);
/* The same for S of element type stype (DEIG_F32 / DEIG_F64: a float64 S - the
 * reference's dtype - is read in double by the image pass and the deflation, so
 * the small eigenvectors of an uncentered covariance keep float64 parity), with
 * options (NULL: defaults). */
int deig_topk_sym_ex(const void* S, int stype, int64_t d, int64_t lds, int k, int p, int max_sweeps,
                     float tol, const float* Q0, int k0, int64_t ldq0, float* V, int64_t ldv,
                     float* evals, int* sweeps_out, float* resid_out, const deig_solver_opts* opts,
                     void* ws, size_t ws_bytes, void* stream);
size_t deig_topk_workspace_ex(int64_t d, int k, int p, int stype, const deig_solver_opts* opts);

/* Server solve: top-k eigenpairs of  scale * sum_i V_i V_i^T  without forming it.
 * Wt = [V_1^T; ...; V_m^T] is (mk) x d row-major (ldw); scale = 1/batches_number.
 * Replaces MasterNode.callback_  distributed.py:126-130 (sigma_tilde += V V^T;
 * /= batches_number) + the notebook's server solve (Online Distributed
 * PCA.ipynb raw line 306: top_k_eigenvectors(segma_bar, k)).  Same solver and
 * outputs as deig_topk_sym_f32; the operator is Q -> scale * Wt^T (Wt Q). */
int deig_projavg_topk_f32(const float* Wt, int64_t d, int64_t mk, int64_t ldw,
                          float scale, int k, int p, int max_sweeps, float tol,
                          const float* Q0, int k0, int64_t ldq0, float* V, int64_t ldv,
                          float* evals, int* sweeps_out, float* resid_out, void* ws,
                          size_t ws_bytes, void* stream);
/* W independent top-k problems (the logical workers of one GPU: same d, k, p and
 * element type; S[i] row-major with leading dimension lds, 16-byte aligned),
 * advanced in lockstep: equivalent to W deig_topk_sym_ex calls with the same
 * options (same kernels, same decisions; V[i] column-major with ldv, evals[i]
 * ascending, sweeps_out[i] / resid_out[i] as there), but each step of all problems
 * is enqueued as batched launches on `stream` (the sweeps of all problems at the same
 * point of their plans in one launch per kernel, one Gram, one small-solve launch of
 * one workgroup per problem, one update) and one stream sync serves every problem's
 * host decisions; for d >= 2048 the problems run as two interleaved groups, the second
 * on an internal stream created for the call that waits for `stream` on entry and
 * that `stream` waits for on return.  All work is ordered on `stream`.  Workspace:
 * deig_topk_batch_workspace(W, ...) bytes.  Returns the first error;
 * DEIG_NOT_CONVERGED if any problem stopped above tol.  status_out[i] (host array,
 * may be NULL): problem i's own return code, the one deig_topk_sym_ex would have
 * returned for it.
 * Replaces W concurrent Node.top_k_eigenvectors calls (distributed.py:22-29, one
 * per SlaveNode shard :42-53). */
size_t deig_topk_batch_workspace(int W, int64_t d, int k, int p, int stype,
                                 const deig_solver_opts* opts);
int deig_topk_sym_batch_ex(int W, const void* const* S, int stype, int64_t d, int64_t lds, int k, int p,
                           int max_sweeps, float tol, float* const* V, int64_t ldv,
                           float* const* evals, int* sweeps_out, float* resid_out, int* status_out,
                           const deig_solver_opts* opts, void* ws, size_t ws_bytes, void* stream);
/* The r03 (0x000300) signature, unchanged: deig_topk_sym_batch_ex with
 * status_out = NULL.  streams: ignored since 0x000400 (r03 ran one stream per
 * problem; may be NULL).  (0x000400 had inserted status_out into THIS signature, an
 * in-place ABI break; 0x000500 restores it and moves status_out to the _ex form.  A
 * binary built against the 0x000400 header links but passes status_out where opts is
 * read: check deig_version() >= 0x000500 before calling, or call the _ex form.) */
int deig_topk_sym_batch(int W, const void* const* S, int stype, int64_t d, int64_t lds, int k, int p,
                        int max_sweeps, float tol, float* const* V, int64_t ldv, float* const* evals,
                        int* sweeps_out, float* resid_out, const deig_solver_opts* opts, void* ws,
                        size_t ws_bytes, void* const* streams, void* stream);

size_t deig_projavg_workspace(int64_t d, int64_t mk, int k, int p);
/* With options (k > 128: block locking with the locked pairs deflated by products
 * with them - the operator stays implicit). */
int deig_projavg_topk_ex(const float* Wt, int64_t d, int64_t mk, int64_t ldw, float scale, int k,
                         int p, int max_sweeps, float tol, const float* Q0, int k0, int64_t ldq0,
                         float* V, int64_t ldv, float* evals, int* sweeps_out, float* resid_out,
                         const deig_solver_opts* opts, void* ws, size_t ws_bytes, void* stream);
size_t deig_projavg_workspace_ex(int64_t d, int64_t mk, int k, int p, const deig_solver_opts* opts);

/* One mini-batch Oja step (online variant, BASELINE.json config 4; not in the
 * reference - parity unpinned):  V <- orth(V + eta/b * Xb^T (Xb V)).
 * Xb is b x d row-major (ldx), V is d x k column-major (ldv), updated in place.
 * k <= 64.  Orthonormalisation: Cholesky-QR2. */
int deig_oja_step_f32(const float* Xb, int64_t b, int64_t d, int64_t ldx, float eta,
                      float* V, int k, int64_t ldv, void* ws, size_t ws_bytes,
                      void* stream);
size_t deig_oja_workspace(int64_t b, int64_t d, int k);

/* nb consecutive Oja steps over the batches X[i*b:(i+1)*b] (X: (nb*b) x d row-major,
 * ldx), V updated in place.  The basis is re-orthonormalised (CholQR2) every
 * orth_every batches and after the last one: the update is linear in V, so the
 * span after each batch equals that of per-batch orthonormalisation.  Same
 * workspace as deig_oja_step_f32 (deig_oja_workspace(b, d, k)). */
int deig_oja_steps_f32(const float* X, int64_t nb, int64_t b, int64_t d, int64_t ldx, float eta,
                       float* V, int k, int64_t ldv, int orth_every, void* ws, size_t ws_bytes,
                       void* stream);

/* deig_oja_steps_f32 with the algorithm chosen explicitly.  DEIG_OJA_AUTO (what
 * deig_oja_steps_f32 does): the resident path where its shape allows, else the
 * two-pass path.  DEIG_OJA_TWO_PASS: two launches per batch (Xb V, then Xb^T T: Xb
 * read twice).  DEIG_OJA_RESIDENT: one launch per run of batches between two
 * re-orthonormalisations, each workgroup holding its block of Xb in registers (Xb
 * read once per batch); needs b = 4096, d a multiple of 512 up to 3072, k <= 32 and
 * 256 CUs (DEIG_EINVAL otherwise).  Its 256 workgroups wait on each other, so the
 * grid is checked against the occupancy query (one 512-thread workgroup per CU on
 * >= 256 CUs) before its plain launch: when it does not fit, DEIG_OJA_RESIDENT
 * returns DEIG_EHIP and DEIG_OJA_AUTO runs the two-pass path.  If a hand-off still
 * waits longer than 2 s (CUs held by other persistent work), V comes back all NaN -
 * the call is asynchronous, so NaN in V is how such a timeout shows in the data, and
 * deig_oja_error reports it as an error.  Same workspace as deig_oja_steps_f32. */
#define DEIG_OJA_AUTO 0
#define DEIG_OJA_TWO_PASS 1
#define DEIG_OJA_RESIDENT 2
int deig_oja_steps_ex(const float* X, int64_t nb, int64_t b, int64_t d, int64_t ldx, float eta,
                      float* V, int k, int64_t ldv, int orth_every, int algo, void* ws,
                      size_t ws_bytes, void* stream);

/* Status of the last deig_oja_steps_ex / deig_oja_steps_f32 / deig_oja_step_f32 call
 * on workspace ws (same b, d, k): synchronises `stream`, then returns DEIG_ETIMEOUT if
 * a resident hand-off of that call waited past its 2-s bound (V was written as NaN),
 * else DEIG_OK.  Call it before the next Oja call on the same workspace (each call
 * clears the word). */
int deig_oja_error(const void* ws, size_t ws_bytes, int64_t b, int64_t d, int k, void* stream);

/* Projection onto an estimated eigenspace: Y = X W.
 * Replaces the notebook's  online_distributed_PCA = lambda X: X @ matrix_w
 * (Online Distributed PCA.ipynb raw line 345).  X: n x d row-major (ldx), W: d x k
 * column-major (ldw, the solvers' V), Y: n x k row-major (ldy).  k <= 256. */
int deig_project_f32(const float* X, int64_t n, int64_t d, int64_t ldx, const float* W, int k,
                     int64_t ldw, float* Y, int64_t ldy, void* ws, size_t ws_bytes,
                     void* stream);
size_t deig_project_workspace(int64_t n, int64_t d, int k);

/* Building block of the solvers, exposed for direct testing / reuse:
 * C[M x N] = alpha * op(A) * B + beta * C  on fp32 MFMA (16x16x4), N % 16 == 0, N <= 256.
 * trans_a != 0: A is K x M row-major (lda), op(A) = A^T  (S*Q with S symmetric, Gram)
 * trans_a == 0: A is M x K row-major (lda)              (Wt*Q, Xb*V)
 * B is K x N row-major (ldb), C is M x N row-major (ldc).  Deterministic split-K. */
int deig_gemm_skinny_f32(int trans_a, const float* A, int64_t lda, const float* B, int64_t ldb,
                         float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, float alpha,
                         float beta, void* ws, size_t ws_bytes, void* stream);
size_t deig_gemm_skinny_workspace(int64_t M, int64_t N, int64_t K);

#ifdef __cplusplus
}
#endif

#endif /* DEIG_H */
