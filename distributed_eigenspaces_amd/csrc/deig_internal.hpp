// Internal declarations shared by the libdeig translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/deig.h"

namespace deig {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void;

// ---------------------------------------------------------------- error handling
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);

#define DEIG_HIP_CHECK(expr)                                                          \
  do {                                                                                \
    hipError_t e__ = (expr);                                                          \
    if (e__ != hipSuccess)                                                            \
      return ::deig::fail(DEIG_EHIP, "%s:%d %s: %s", __FILE__, __LINE__, #expr,       \
                          hipGetErrorString(e__));                                    \
  } while (0)

#define DEIG_REQUIRE(cond, ...)                                                       \
  do {                                                                                \
    if (!(cond)) return ::deig::fail(DEIG_EINVAL, __VA_ARGS__);                       \
  } while (0)

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Bijective XCD-aware relabel of a 1-D grid of G blocks: blocks b, b+8, ... (one
// XCD under round-robin dispatch) get consecutive logical ids, so neighbouring
// logical work items share that XCD's L2.
__device__ __forceinline__ int xcd_logical(int b, int G) {
  const int x = b & 7, qq = G >> 3, rr = G & 7;
  const int base = (x < rr) ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq;
  return base + (b >> 3);
}
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Number of CUs of the current device (cached per device id).
int num_cus();

// Workspace carving helper: hands out 256-byte aligned slices.
struct Carve {
  char* base;
  size_t cap;
  size_t off = 0;
  Carve(void* b, size_t c) : base(static_cast<char*>(b)), cap(c) {}
  template <class T>
  T* take(size_t count) {
    off = align_up(off, 256);
    T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
    off += count * sizeof(T);
    return p;
  }
  bool ok() const { return off <= cap; }
};

// ---------------------------------------------------------------- launchers
// Covariance SYRK (syrk.hip).
size_t syrk_workspace_bytes(int64_t n, int64_t d);
int syrk_launch(const float* X, int64_t n, int64_t d, int64_t ldx, float alpha, float* S,
                int64_t lds, void* ws, size_t ws_bytes, hipStream_t stream);
// Split-bf16 covariance SYRK (syrk_split.hip).
size_t syrk_split_workspace_bytes(int64_t n, int64_t d);
// accumulate: S += alpha X^T X (row chunks of one long shard, or several shards).
int syrk_split_launch(const float* X, int64_t n, int64_t d, int64_t ldx, float alpha, float* S,
                      int64_t lds, void* ws, size_t ws_bytes, hipStream_t stream,
                      bool accumulate = false);

// Mean-shifted covariance of float samples (shift.hip); xtype DEIG_F32 / DEIG_F64.
size_t syrk_shift_workspace_bytes(int64_t n, int64_t d, int xtype);
int syrk_shift_launch(const void* X, int xtype, int64_t n, int64_t d, int64_t ldx, double alpha,
                      double* S64, int64_t lds64, float* S, int64_t lds, void* ws, size_t ws_bytes,
                      hipStream_t stream);

// Exact uint8 covariance on int8 MFMA (syrk_u8.hip); mode DEIG_U8_RAW / DEIG_U8_GRAY3.
size_t syrk_u8_workspace_bytes(int64_t n, int64_t d, int mode);
int syrk_u8_launch(const uint8_t* X, int64_t n, int64_t d, int64_t ldx, int mode, double alpha,
                   float* S, int64_t lds, double* S64, int64_t lds64, void* ws, size_t ws_bytes,
                   hipStream_t stream);

// Skinny GEMM (skinny.hip):  C[M x N] = alpha * op(A) * B + beta * C
//   trans_a = true : A is K x M row-major (op(A) = A^T)
//   trans_a = false: A is M x K row-major
//   B is K x N row-major; N % 16 == 0, N <= 256.
// Launches that cover several problems of one shape (solve_batch): problem i's
// workspace buffers sit off[i] bytes after problem 0's (off[0] = 0; the solver
// workspaces are equally carved slices of one allocation); outputs outside the
// workspaces are per problem.
constexpr int kMaxProbBatch = 16;
struct ProbBatch {
  int n;
  int64_t off[kMaxProbBatch];
  float* V[kMaxProbBatch];      // rr_update: the block's eigenvectors
  float* evals[kMaxProbBatch];  // rr_update: its eigenvalues
  void* hs[kMaxProbBatch];      // solver status blocks (pinned host memory)
};
inline ProbBatch one_problem() {
  ProbBatch b{};
  b.n = 1;
  return b;
}

size_t skinny_workspace_bytes(int64_t M, int64_t N, int64_t K);
// batch (optional): the same product for batch->n problems, A, B, C and slab of
// problem i at off[i] bytes from the arguments.
int skinny_launch(bool trans_a, const float* A, int64_t lda, const float* B, int64_t ldb,
                  float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, float alpha,
                  float beta, float* slab, size_t slab_bytes, hipStream_t stream,
                  const ProbBatch* batch = nullptr);

// bf16x6 symmetric sweep (sweep.hip): Y = alpha * S Q, S symmetric d x d
// row-major, Q d x p (ldq), Y d x p (ldy), p % 16 == 0, p <= 128.
size_t sweep_workspace_bytes(int64_t d, int p);
// sweep_prepare builds the image of  S + shift I - Vd diag(lamd) Vd^T  in the
// workspace (once per operator; stype DEIG_F32 / DEIG_F64; the shift and the r
// deflated pairs - Vd column-major, ldv - are formed in double), sweep_apply runs
// one product from it.
int sweep_prepare(const void* S, int stype, int64_t d, int64_t lds, int p, void* ws,
                  size_t ws_bytes, hipStream_t st, const float* Vd = nullptr, int64_t ldv = 0,
                  const float* lamd = nullptr, int r = 0, double shift = 0.0);
// mode 0: exact (six products).  mode 1 (round_q): the solver's in-place mode - Q
// (which must then be writable) is rounded to 16 significant bits (Q' = h + m, two
// bf16 pieces) and the product S Q' formed with five bf16 products instead of six
// (sweep.hip split_q_kernel).  mode 2 (early sweeps): as 1, and S is taken as its
// two leading bf16 pieces from the prepared two-piece image - three products, no
// split in the sweep, ~2^-16 relative.
constexpr int kSweepExact = 0, kSweepRoundQ = 1, kSweepFast = 2, kSweepHalf = 3;
// Optional epilogue of a sweep in the solver's chain, fused with the split-K
// reduction (sweep_finish_kernel): the basis step that turns Y = S Q into the next
// Q (the elementwise rr_power_kernel / cheb_step_kernel forms), and the next
// sweep's Q image (next_mode: the mode of the sweep that will read it, which then
// runs with q_ready and skips its own split_q_kernel).
struct SweepStep {
  int kind;  // 1 = power (Q_j <- Y_j cs_j on live columns), 2 = Chebyshev degree
  float* Q;  // the basis (row stride ldq), updated in place
  int64_t ldq;
  float* T;  // Chebyshev: X_{j-1} (row stride p)
  const float* cs;
  const float* lam;
  float tau;                // power: live if cs_j > 0 and |lam_j| >= tau |lam_0|
  float thr, a, cc, gamma;  // Chebyshev: X_{j+1} = a (Y - cc X_j) - gamma X_{j-1} if lam_j >= thr
  int next_mode;            // kSweep* of the next sweep
  int write_y;              // 1: also store Y = alpha S Q (split-K sums); 0: Y is dead (the
                            // solver's intermediate sweeps: only the basis step reads it)
};
// Several problems of the same d, p and mode in one launch per kernel (solve_batch):
// problem i's Q, Y, workspace and step buffers sit off[i] bytes after problem 0's
// (off[0] = 0); the fused step's scalars are per problem, its pointers and next_mode
// problem 0's.
constexpr int kMaxSweepBatch = kMaxProbBatch;
struct SweepBatch {
  int n;
  int64_t off[kMaxSweepBatch];
  int kind[kMaxSweepBatch];
  float tau[kMaxSweepBatch], thr[kMaxSweepBatch], a[kMaxSweepBatch], cc[kMaxSweepBatch],
      gamma[kMaxSweepBatch];
};
int sweep_apply(const float* Q, int64_t d, int p, int64_t ldq, float* Y, int64_t ldy, float alpha,
                void* ws, size_t ws_bytes, hipStream_t st, int mode = kSweepExact,
                const SweepStep* step = nullptr, bool q_ready = false,
                bool kernel_only = false,  // kernel_only: no split-K reduction (measurement)
                const SweepBatch* batch = nullptr);

// Rayleigh-Ritz pieces (rr.hip).
struct RRBuffers {
  float* Z;          // d x 2p row-major: [Q | Y]
  float* C;          // 2p x 2p Gram of Z
  float* Linv;       // p x p
  float* Wtmp;       // p x p
  float* W;          // p x p, columns sorted by descending Ritz value
  float* lam;        // p, descending
  float* cs;         // p, column scales (0 = dead column)
  float* qs;         // p, 1 / ||Q w_j|| (Ritz vector normalisation)
  float* resid_part; // nblk_update x k
  float* resid;      // k  (relative residual per top-k column; [k] = max)
  int* info;         // small int scratch
};
// Start basis (Q0's k0 columns, then pseudo-random ones); rows >= valid zero (< 0: none).
int rr_init_launch(float* Z, int64_t d, int p, const float* Q0, int k0, int64_t ldq0,
                   uint64_t seed, hipStream_t stream, int64_t valid = -1);
// max_jsweeps caps the Jacobi sweeps of the small eigenproblem (30 = converge);
// jrel: a pair is rotated while |h_ab| > jrel sqrt(|h_aa h_bb|) (2e-7: to rounding).
int rr_small_launch(const RRBuffers& b, int p, hipStream_t stream, int max_jsweeps = 30,
                    float jrel = 2e-7f);
// n independent small solves in launches of up to kRRBatch workgroups (one each).
constexpr int kRRBatch = 16;
int rr_small_batch_launch(const RRBuffers* const* bs, const int* max_jsweeps, int n, int p,
                          hipStream_t stream, float jrel = 2e-7f);
int rr_update_blocks(int64_t d);
int rr_power_launch(const RRBuffers& b, int64_t d, int p, float tau, hipStream_t stream);
// One scaled Chebyshev filter degree on Z = [X_j | A X_j] with T = X_{j-1} (d x p).
int cheb_step_launch(const RRBuffers& b, float* T, int64_t d, int p, float thr, float alpha,
                     float cc, float gamma, hipStream_t stream);
int rr_update_launch(const RRBuffers& b, int64_t d, int p, int k, float* V, int64_t ldv,
                     float* evals, hipStream_t stream);
// The same for batch.n problems (RRBuffers of problem i at off[i]; V / evals per problem).
int rr_update_batch_launch(const RRBuffers& b0, int64_t d, int p, int k, int64_t ldv,
                           const ProbBatch& batch, hipStream_t stream);
// Columns 0..kc-1 of V (col-major, ldv) made orthogonal to columns kc..kc+r-1, normalised.
int deflate_orth_launch(float* V, int64_t ldv, int64_t d, int kc, int r, hipStream_t stream);
// Columns 0..kc-1 of V orthonormalised among themselves in order (modified Gram-Schmidt,
// one launch per column; the rare path of a block in the deflation-residue band).
int block_mgs_launch(float* V, int64_t ldv, int64_t d, int kc, hipStream_t stream);
// evals[0..k) -= shift (device).
int unshift_launch(float* evals, int k, double shift, hipStream_t stream);
// evals[j] = v_j^T S v_j / v_j^T v_j in double for the k columns of V (S: stype).
size_t rq_workspace_bytes(int64_t d, int k);
int rq_launch(const void* S, int stype, int64_t d, int64_t lds, const float* V, int64_t ldv, int k,
              float* evals, void* ws, hipStream_t stream);

// Oja (oja.hip).
size_t oja_workspace_bytes(int64_t b, int64_t d, int k);
int oja_launch(const float* Xb, int64_t b, int64_t d, int64_t ldx, float eta, float* V,
               int k, int64_t ldv, void* ws, size_t ws_bytes, hipStream_t stream);
int oja_steps_launch(const float* X, int64_t nb, int64_t b, int64_t d, int64_t ldx, float eta,
                     float* V, int k, int64_t ldv, int orth_every, void* ws, size_t ws_bytes,
                     hipStream_t stream, int algo);
int oja_error(const void* ws, size_t ws_bytes, int64_t b, int64_t d, int k, hipStream_t st);

// Projection Y = X W (project.hip).
size_t project_workspace_bytes(int64_t n, int64_t d, int k);
int project_launch(const float* X, int64_t n, int64_t d, int64_t ldx, const float* W, int k,
                   int64_t ldw, float* Y, int64_t ldy, void* ws, size_t ws_bytes, hipStream_t st);

}  // namespace deig
