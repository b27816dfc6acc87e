// Mini-batch Oja steps for the online / streaming variant (BASELINE.json config 4):
//   V <- orth(V + eta/b * Xb^T (Xb V)),   orth = Cholesky-QR2.
// Not present in the reference (parity unpinned; judged by sin(theta) against
// the one-shot float64 oracle and ref_cpu.oja_epoch).  Xb is read twice (Xb V
// and Xb^T T), each pass a skinny GEMM at ~k/2 flop/B (HBM-bound for k <= 32).
#include "deig_internal.hpp"

namespace deig {
namespace {

__global__ __launch_bounds__(256) void col_to_rowpad(const float* __restrict__ V, int64_t ldv,
                                                     int64_t d, int k, int kp,
                                                     float* __restrict__ Vr) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * kp) return;
  const int64_t r = idx / kp;
  const int j = (int)(idx - r * kp);
  Vr[idx] = (j < k) ? V[r + (int64_t)j * ldv] : 0.f;
}

__global__ __launch_bounds__(256) void rowpad_to_col(const float* __restrict__ Vr, int64_t d,
                                                     int k, int kp, float* __restrict__ V,
                                                     int64_t ldv) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * k) return;
  const int j = (int)(idx / d);
  const int64_t r = idx - (int64_t)j * d;
  V[r + (int64_t)j * ldv] = Vr[r * kp + j];
}

// G (kp x kp, leading k x k used) = L L^T;  Rinv = L^-T (upper), zero-padded to kp.
// ONE wave, everything in registers, loops fully unrolled over KP so that every
// register index is static: lane c holds column c of the trailing matrix
// (right-looking Cholesky; the pivot row is broadcast with v_readlane), then
// column c of X = L^-1 (forward substitution, L's rows broadcast the same way).
// No LDS, no barriers: the former 256-thread version spent 48.6 us (config 4,
// k = 32) in barrier-separated steps and an LDS-latency-bound inverse.
__device__ __forceinline__ float lane_bcast(float v, int src) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
}

template <int KP>
__global__ __launch_bounds__(64) void chol_rinv_kernel(const float* __restrict__ G, int k, int kp,
                                                       float* __restrict__ Rinv) {
  // One wave; lane r keeps row r of the matrix in registers (static indices: the
  // loops over KP are unrolled).  G is extended to KP x KP by the identity beyond k
  // (its Cholesky factor and inverse are then block-diagonal with an identity
  // block), so nothing depends on the runtime k.  Columns / rows of L are exchanged
  // through LDS with broadcast ds_read_b128 (all lanes read the same address):
  // per Cholesky step one column, for the inverse the finished rows.  (A version
  // broadcasting with v_readlane took ~23 us for k = 32: ~1000 readlanes with their
  // hazard s_nops, plus runtime-k branches.)
  __shared__ __attribute__((aligned(16))) float col[KP];
  __shared__ __attribute__((aligned(16))) float Ls[KP][KP];
  const int r = threadIdx.x;  // row owned by this lane (lanes >= KP idle but in step)
  const bool live = r < KP;
  float a[KP];
#pragma unroll
  for (int c = 0; c < KP; ++c) {
    const bool in = r < k && c < k;
    a[c] = in ? G[r * kp + c] : (r == c ? 1.f : 0.f);
  }
  const float ref0 = fmaxf(fabsf(__shfl(a[0], 0, 64)), 1e-30f);
  float dinv[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    // pivot A[j][j] from lane j; L[r][j] = A[r][j] / L[j][j] for r > j
    const float v = fmaxf(__shfl(a[j], j, 64), 1e-12f * ref0);
    const float ljj = sqrtf(v);
    dinv[j] = 1.0f / ljj;
    const float l = (r == j) ? ljj : (r > j ? a[j] * dinv[j] : 0.f);
    a[j] = l;
    if (live) col[r] = l;
    __syncthreads();
    // trailing update of this lane's row: A[r][c] -= L[r][j] L[c][j]  (c > j)
#pragma unroll
    for (int c4 = (j + 1) / 4; c4 < KP / 4; ++c4) {
      const f32x4 lc = *reinterpret_cast<const f32x4*>(col + 4 * c4);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * c4 + e > j) a[4 * c4 + e] = fmaf(-l, lc[e], a[4 * c4 + e]);
    }
    __syncthreads();
  }
  // lane r holds row r of L in a[0 .. r] (zeros above the diagonal)
  if (live)
#pragma unroll
    for (int c4 = 0; c4 < KP / 4; ++c4)
      *reinterpret_cast<f32x4*>(&Ls[r][4 * c4]) =
          f32x4{a[4 * c4], a[4 * c4 + 1], a[4 * c4 + 2], a[4 * c4 + 3]};
  __syncthreads();
  // X = L^-1, lane c = column c: X[i] = (delta_ic - sum_{t < i} L[i][t] X[t]) / L[i][i]
  const int c = r;
  float X[KP];
#pragma unroll
  for (int i = 0; i < KP; ++i) {
    float sacc = (c == i) ? 1.0f : 0.0f;
#pragma unroll
    for (int t4 = 0; t4 < (i + 3) / 4; ++t4) {
      const f32x4 li = *reinterpret_cast<const f32x4*>(&Ls[i][4 * t4]);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * t4 + e < i) sacc = fmaf(-li[e], X[4 * t4 + e], sacc);
    }
    X[i] = sacc * dinv[i];
  }
  // Rinv = L^-T: Rinv[c][i] = X[i][c] (lane c); zero outside the k x k block
  if (c < kp) {
#pragma unroll
    for (int i = 0; i < KP; ++i)
      if (i < kp) Rinv[c * kp + i] = (c < k && i < k) ? X[i] : 0.f;
  }
}

void launch_chol_rinv(const float* G, int k, int kp, float* Rinv, hipStream_t st) {
  if (kp <= 16)
    hipLaunchKernelGGL(chol_rinv_kernel<16>, dim3(1), dim3(64), 0, st, G, k, kp, Rinv);
  else if (kp <= 32)
    hipLaunchKernelGGL(chol_rinv_kernel<32>, dim3(1), dim3(64), 0, st, G, k, kp, Rinv);
  else if (kp <= 48)
    hipLaunchKernelGGL(chol_rinv_kernel<48>, dim3(1), dim3(64), 0, st, G, k, kp, Rinv);
  else
    hipLaunchKernelGGL(chol_rinv_kernel<64>, dim3(1), dim3(64), 0, st, G, k, kp, Rinv);
}

struct OjaWs {
  float *Vr, *Vr2, *T, *G, *Rinv, *slab;
  size_t slab_bytes;
};

OjaWs carve_oja(void* ws, size_t cap, int64_t b, int64_t d, int kp, size_t* total) {
  Carve c(ws, cap);
  OjaWs o;
  o.Vr = c.take<float>((size_t)d * kp);
  o.Vr2 = c.take<float>((size_t)d * kp);
  o.T = c.take<float>((size_t)b * kp);
  o.G = c.take<float>((size_t)kp * kp);
  o.Rinv = c.take<float>((size_t)kp * kp);
  size_t sb = skinny_workspace_bytes(b, kp, d);
  size_t s2 = skinny_workspace_bytes(d, kp, b);
  size_t s3 = skinny_workspace_bytes(kp, kp, d);
  size_t s4 = skinny_workspace_bytes(d, kp, kp);
  if (s2 > sb) sb = s2;
  if (s3 > sb) sb = s3;
  if (s4 > sb) sb = s4;
  o.slab = c.take<float>(sb / sizeof(float) + 1);
  o.slab_bytes = sb;
  *total = c.off;
  return o;
}

// Cholesky-QR of the row-padded d x kp basis `in` (`scratch` has the same size) with
// `passes` passes (2 = CholQR2, orthonormal to fp32 rounding; 1 = one pass, used
// between batches where only the span and a bounded condition number matter);
// the result is in *result (in or scratch: one buffer swap per pass).
int cholqr(float* in, float* scratch, const OjaWs& o, int64_t d, int k, int kp, hipStream_t st,
           int passes, float** result) {
  int rc;
  float* cur = in;
  float* nxt = scratch;
  for (int pass = 0; pass < passes; ++pass) {
    if ((rc = skinny_launch(true, cur, kp, cur, kp, o.G, kp, kp, kp, d, 1.f, 0.f, o.slab,
                            o.slab_bytes, st)))
      return rc;
    launch_chol_rinv(o.G, k, kp, o.Rinv, st);
    DEIG_HIP_CHECK(hipGetLastError());
    if ((rc = skinny_launch(false, cur, kp, o.Rinv, kp, nxt, kp, d, kp, kp, 1.f, 0.f, o.slab,
                            o.slab_bytes, st)))
      return rc;
    float* t = cur;
    cur = nxt;
    nxt = t;
  }
  *result = cur;
  return DEIG_OK;
}

}  // namespace

size_t oja_workspace_bytes(int64_t b, int64_t d, int k) {
  const int kp = (int)cdiv(k, 16) * 16;
  size_t total = 0;
  carve_oja(nullptr, 0, b, d, kp, &total);
  return total;
}

// nb consecutive batches of b rows (batch i starts at row i * b of X).  Each
// batch applies V <- V + eta/b Xb^T (Xb V); the basis is re-orthonormalised
// (CholQR2) every orth_every batches and after the last one.  The update is
// linear in V and an orthonormalisation only right-multiplies V by an
// invertible k x k factor, so the span after every batch equals the one of
// per-batch orthonormalisation (ref_cpu.oja_epoch); deferring it only lets the
// column norms grow by ~(1 + eta lambda_max)^orth_every in between.
int oja_steps_launch(const float* X, int64_t nb, int64_t b, int64_t d, int64_t ldx, float eta,
                     float* V, int k, int64_t ldv, int orth_every, void* ws, size_t ws_bytes,
                     hipStream_t st) {
  DEIG_REQUIRE(nb >= 1 && b >= 1 && d >= 4 && d % 4 == 0,
               "oja: need nb >= 1, b >= 1 and d %% 4 == 0");
  DEIG_REQUIRE(k >= 1 && k <= 64 && k <= d, "oja: need 1 <= k <= min(64, d)");
  DEIG_REQUIRE(ldx >= d && ldx % 4 == 0 && ldv >= d, "oja: bad leading dims");
  DEIG_REQUIRE(orth_every >= 1, "oja: orth_every must be >= 1");
  const int kp = (int)cdiv(k, 16) * 16;
  size_t total = 0;
  OjaWs o = carve_oja(ws, ws_bytes, b, d, kp, &total);
  if (!ws || total > ws_bytes)
    return fail(DEIG_EWORKSPACE, "oja: workspace %zu < %zu", ws_bytes, total);
  int rc;
  // the basis lives in `cur` (o.Vr or o.Vr2: each CholQR pass swaps the two)
  float* cur = o.Vr;
  float* spare = o.Vr2;
  hipLaunchKernelGGL(col_to_rowpad, dim3((unsigned)cdiv(d * kp, 256)), dim3(256), 0, st, V, ldv, d,
                     k, kp, cur);
  DEIG_HIP_CHECK(hipGetLastError());
  for (int64_t i = 0; i < nb; ++i) {
    const float* Xb = X + i * b * ldx;
    // T = Xb V
    if ((rc = skinny_launch(false, Xb, ldx, cur, kp, o.T, kp, b, kp, d, 1.f, 0.f, o.slab,
                            o.slab_bytes, st)))
      return rc;
    // V += eta/b * Xb^T T
    if ((rc = skinny_launch(true, Xb, ldx, o.T, kp, cur, kp, d, kp, b, eta / (float)b, 1.f,
                            o.slab, o.slab_bytes, st)))
      return rc;
    // intermediate re-orthonormalisations only bound the basis' condition number
    // (the span is what the update carries): one CholQR pass; the last one is CholQR2
    const int passes = (i + 1 == nb) ? 2 : ((i + 1) % orth_every == 0 ? 1 : 0);
    if (passes) {
      float* res = cur;
      if ((rc = cholqr(cur, spare, o, d, k, kp, st, passes, &res))) return rc;
      spare = res == cur ? spare : cur;
      cur = res;
    }
  }
  hipLaunchKernelGGL(rowpad_to_col, dim3((unsigned)cdiv(d * k, 256)), dim3(256), 0, st, cur, d, k,
                     kp, V, ldv);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

int oja_launch(const float* Xb, int64_t b, int64_t d, int64_t ldx, float eta, float* V, int k,
               int64_t ldv, void* ws, size_t ws_bytes, hipStream_t st) {
  return oja_steps_launch(Xb, 1, b, d, ldx, eta, V, k, ldv, 1, ws, ws_bytes, st);
}

}  // namespace deig
