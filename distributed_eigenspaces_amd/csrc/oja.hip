// Mini-batch Oja steps for the online / streaming variant (BASELINE.json config 4):
//   V <- orth(V + eta/b * Xb^T (Xb V)),   orth = Cholesky-QR2.
// Not present in the reference (parity unpinned; judged by sin(theta) against
// the one-shot float64 oracle and ref_cpu.oja_epoch).  Xb is read twice (Xb V
// and Xb^T T), each pass a skinny GEMM at ~k/2 flop/B (HBM-bound for k <= 32).
#include <stdlib.h>

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
  const int c = threadIdx.x;  // column owned by this lane
  const bool live = c < k;
  float A[KP];
#pragma unroll
  for (int i = 0; i < KP; ++i) A[i] = (live && i < k) ? G[i * kp + c] : 0.f;
  const float ref0 = fabsf(lane_bcast(A[0], 0)) > 0.f ? fabsf(lane_bcast(A[0], 0)) : 1.f;
  float dinv[KP];  // 1 / L[j][j], uniform
  // Right-looking Cholesky: after step j, A[j] (lane c) = L[c][j] for c >= j.
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    if (j < k) {
      float v = lane_bcast(A[j], j);
      if (!(v > 1e-12f * ref0)) v = 1e-12f * ref0;
      const float ljj = sqrtf(v);
      dinv[j] = 1.0f / ljj;
      const float l = (c == j) ? ljj : (c > j ? A[j] * dinv[j] : 0.f);
      A[j] = l;
#pragma unroll
      for (int i = j + 1; i < KP; ++i)
        if (i < k) A[i] = fmaf(-lane_bcast(l, i), l, A[i]);  // A[i][c] -= L[i][j] L[c][j]
    } else {
      dinv[j] = 0.f;
    }
  }
  // Lane r now holds row r of L in A[0 .. r].  X = L^-1 column c: for i = 0..k-1,
  // X[i] = (delta_ic - sum_{t < i} L[i][t] X[t]) / L[i][i].
  float X[KP];
#pragma unroll
  for (int i = 0; i < KP; ++i) {
    if (i < k) {
      float s = (c == i) ? 1.0f : 0.0f;
#pragma unroll
      for (int t = 0; t < i; ++t) s = fmaf(-lane_bcast(A[t], i), X[t], s);
      X[i] = s * dinv[i];
    } else {
      X[i] = 0.f;
    }
  }
  // Rinv = L^-T: Rinv[c][i] = X[i][c] (lane c); rows / columns >= k are zero.
  if (c < kp) {
#pragma unroll
    for (int i = 0; i < KP; ++i)
      if (i < kp) Rinv[c * kp + i] = (live && i < k) ? X[i] : 0.f;
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

// ---------------------------------------------------------------- batch products
// Per batch (b rows of X, d features, KP = 16 NB padded columns), two passes over Xb:
//   oja_nn_kernel : T = Xb V          (b x KP row-major)
//   oja_tn_kernel : Vc += c Xb^T T    (Vc: d x KP column-major work basis)
// fp32 MFMA 16x16x4 (exact fp32 fma chains).  Both read Xb with float4 loads and
// need no separate reduce kernel: NN gives each block 16 complete rows (K split
// over its 8 waves, summed in LDS in wave order) and TN's row-slice partials are
// summed by the last block to finish each feature block (fixed slice order:
// deterministic), so a batch is exactly two launches.
constexpr int NN_ROWS = 16, NN_THR = 1024, NN_WAVES = NN_THR / 64;
// TN: a block = TN_WAVES waves on one 64-feature tile, each wave a row sub-slice;
// the waves' partial tiles are summed in LDS (wave order) before the block's slab.
constexpr int TN_FEAT = 64, TN_WAVES = 8, TN_THR = 64 * TN_WAVES;

// Lane (r = l & 15, g = l >> 4) loads Xb[r0 + r][16 c + 4 g .. + 3] and the B
// fragments V[16 c + 4 g .. + 3][16 j + r] (column-major V: contiguous in k); MFMA
// step s uses component s of both, i.e. k = 16 c + 4 g + s for lane group g - the
// same permuted k on both operands, so the product is exact.
template <int NB>
__global__ __launch_bounds__(NN_THR) void oja_nn_kernel(const float* __restrict__ X, int64_t ldx,
                                                       int64_t b, int64_t d, int64_t dpad,
                                                       const float* __restrict__ Vc,
                                                       float* __restrict__ T) {
  constexpr int KP = 16 * NB;
  __shared__ f32x4 red[NN_WAVES][NB][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * NN_ROWS;
  const int64_t row = r0 + r;
  const bool rok = row < b;
  const float* xr = X + (rok ? row : 0) * ldx + 4 * g;
  const int64_t nch = d / 16;  // d % 16 == 0 (padded by the caller)
  const int64_t c0 = nch * w / NN_WAVES, c1 = nch * (w + 1) / NN_WAVES;
  f32x4 acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  const float* vb = Vc + (int64_t)r * dpad + 4 * g;
  // U chunks per iteration: their loads are all issued before the MFMAs
  constexpr int U = 4;
  auto step = [&](const f32x4& a, const f32x4 (&bv)[NB]) {
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
      for (int j = 0; j < NB; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s2], bv[j][s2], acc[j], 0, 0, 0);
  };
  int64_t c = c0;
  for (; c + U <= c1; c += U) {
    f32x4 a[U], bv[U][NB];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = rok ? *reinterpret_cast<const f32x4*>(xr + 16 * (c + u)) : zero;
#pragma unroll
      for (int j = 0; j < NB; ++j)
        bv[u][j] = *reinterpret_cast<const f32x4*>(vb + (int64_t)16 * j * dpad + 16 * (c + u));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) step(a[u], bv[u]);
  }
  for (; c < c1; ++c) {
    f32x4 bv[NB];
    const f32x4 a = rok ? *reinterpret_cast<const f32x4*>(xr + 16 * c) : zero;
#pragma unroll
    for (int j = 0; j < NB; ++j)
      bv[j] = *reinterpret_cast<const f32x4*>(vb + (int64_t)16 * j * dpad + 16 * c);
    step(a, bv);
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) red[w][j][lane] = acc[j];
  __syncthreads();
  // C/D map: column = lane & 15, row = 4 (lane >> 4) + e
  for (int idx = tid; idx < NB * 64; idx += NN_THR) {
    const int j = idx >> 6, l = idx & 63;
    f32x4 s = red[0][j][l];
#pragma unroll
    for (int ww = 1; ww < NN_WAVES; ++ww) s += red[ww][j][l];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t rr = r0 + 4 * (l >> 4) + e;
      if (rr < b) T[rr * KP + 16 * j + (l & 15)] = s[e];
    }
  }
}

// grid (dpad / 64, ns): block (fb, sl) covers features [64 fb, +64) and rows
// [b sl / ns, b (sl + 1) / ns), split over its TN_WAVES waves.  Lane (q = l & 15,
// g = l >> 4) loads Xb[row + g][f0 + 4 q .. + 3] (4 rows x 256 contiguous bytes
// per wave instruction) and the A fragments T[row + g][16 j + q]; MFMA e uses
// component e: B[k = g][col = q] = Xb[row + g][f0 + 4 q + e], so accumulator (j, e)
// holds output column 16 j + 4 (l >> 4) + reg of feature f0 + 4 (l & 15) + e.
// The waves' tiles are summed in LDS (wave order), the block's tile goes to a slab,
// and the last block of a feature tile (arrival counter) sums the ns slabs in slice
// order with independent loads, adds Vc and stores Vc.
template <int NB>
__global__ __launch_bounds__(TN_THR) void oja_tn_kernel(const float* __restrict__ X, int64_t ldx,
                                                       int64_t b, int64_t d, int64_t dpad,
                                                       const float* __restrict__ T, float coef,
                                                       float* __restrict__ Vc,
                                                       float* __restrict__ part,
                                                       unsigned* __restrict__ count) {
  constexpr int KP = 16 * NB;
  constexpr int TILE = TN_FEAT * KP;  // floats per slab: [feature 64][column KP]
  __shared__ f32x4 red[TN_WAVES][NB * 4][64];
  __shared__ unsigned last_flag;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int q = lane & 15, g = lane >> 4;
  const int fb = blockIdx.x, sl = blockIdx.y, ns = gridDim.y;
  const int64_t f0 = (int64_t)fb * TN_FEAT + 4 * q;
  const int64_t s0 = b * sl / ns, s1 = b * (sl + 1) / ns;
  const int64_t k0 = s0 + (s1 - s0) * w / TN_WAVES, k1 = s0 + (s1 - s0) * (w + 1) / TN_WAVES;
  f32x4 acc[NB][4];
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[j][e] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  const bool fok = f0 < d;
  auto ld = [&](int64_t k, f32x4& x, float (&t)[NB]) {
    const int64_t row = k + g;
    const bool ok = row < k1;
    x = (ok && fok) ? *reinterpret_cast<const f32x4*>(X + row * ldx + f0) : zero;
#pragma unroll
    for (int j = 0; j < NB; ++j) t[j] = ok ? T[row * KP + 16 * j + q] : 0.f;
  };
  auto step = [&](const f32x4& x, const float (&t)[NB]) {
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc[j][e] = __builtin_amdgcn_mfma_f32_16x16x4f32(t[j], x[e], acc[j][e], 0, 0, 0);
  };
  constexpr int U = 8;  // 4-row steps per iteration, loads issued first
  int64_t k = k0;
  for (; k + 4 * U <= k1; k += 4 * U) {
    f32x4 x[U];
    float t[U][NB];
#pragma unroll
    for (int u = 0; u < U; ++u) ld(k + 4 * u, x[u], t[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) step(x[u], t[u]);
  }
  for (; k < k1; k += 4) {
    f32x4 x;
    float t[NB];
    ld(k, x, t);
    step(x, t);
  }
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) red[w][4 * j + e][lane] = acc[j][e];
  __syncthreads();
  // block tile -> slab; thread (j, e, l) sums the TN_WAVES waves in order
  float* slab = part + ((int64_t)fb * ns + sl) * TILE;
  for (int idx = tid; idx < NB * 4 * 64; idx += TN_THR) {
    const int je = idx >> 6, l = idx & 63;
    f32x4 sacc = red[0][je][l];
#pragma unroll
    for (int ww = 1; ww < TN_WAVES; ++ww) sacc += red[ww][je][l];
    const int j = je >> 2, e = je & 3;
    *reinterpret_cast<f32x4*>(slab + (4 * (l & 15) + e) * KP + 16 * j + 4 * (l >> 4)) = sacc;
  }
  __threadfence();
  __syncthreads();
  if (tid == 0) last_flag = (atomicAdd(count + fb, 1u) == (unsigned)(ns - 1)) ? 1u : 0u;
  __syncthreads();
  if (!last_flag) return;
  __threadfence();
  // last block of this feature tile: Vc[f][c] += coef * sum_sl slab (slice order)
  const float* base = part + (int64_t)fb * ns * TILE;
  for (int idx = tid; idx < TILE / 4; idx += TN_THR) {
    f32x4 sv[8];
    f32x4 sacc = {0.f, 0.f, 0.f, 0.f};
    for (int u0 = 0; u0 < ns; u0 += 8) {  // 8 independent loads in flight
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u0 + u < ns) sv[u] = *reinterpret_cast<const f32x4*>(base + (int64_t)(u0 + u) * TILE + 4 * idx);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u0 + u < ns) sacc += sv[u];
    }
    const int f = (4 * idx) / KP, c = (4 * idx) % KP;
    const int64_t feat = (int64_t)fb * TN_FEAT + f;
    if (feat < d)
#pragma unroll
      for (int e = 0; e < 4; ++e) Vc[(int64_t)(c + e) * dpad + feat] += coef * sacc[e];
  }
  if (tid == 0) count[fb] = 0u;  // ready for the next batch (kernel boundary orders it)
}

// Column-major V (ldv, k columns) <-> the work basis Vc (d x KP column-major, zero
// columns k .. KP-1; d padded to a multiple of 256 rows with zeros).
__global__ __launch_bounds__(256) void v_to_work(const float* __restrict__ V, int64_t ldv, int64_t d,
                                                 int64_t dpad, int k, int kp, float* __restrict__ Vc) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= dpad * kp) return;
  const int j = (int)(idx / dpad);
  const int64_t r = idx - (int64_t)j * dpad;
  Vc[idx] = (j < k && r < d) ? V[r + (int64_t)j * ldv] : 0.f;
}

__global__ __launch_bounds__(256) void work_to_rowpad(const float* __restrict__ Vc, int64_t dpad,
                                                      int64_t d, int kp, float* __restrict__ Vr) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * kp) return;
  const int64_t r = idx / kp;
  const int j = (int)(idx - r * kp);
  Vr[idx] = Vc[(int64_t)j * dpad + r];
}

__global__ __launch_bounds__(256) void rowpad_to_work(const float* __restrict__ Vr, int64_t d,
                                                      int64_t dpad, int kp, float* __restrict__ Vc) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * kp) return;
  const int64_t r = idx / kp;
  const int j = (int)(idx - r * kp);
  Vc[(int64_t)j * dpad + r] = Vr[idx];
}

struct OjaWs {
  float *Vr, *Vr2, *T, *G, *Rinv, *slab, *Vc, *part;
  unsigned* count;
  size_t slab_bytes;
};

// Row slices per feature tile: about 2 waves per SIMD over the grid, >= 8 rows per
// wave (DEIG_OJA_TN_SLICES overrides, for tuning).
int tn_slices(int64_t b, int64_t d) {
  if (const char* e = getenv("DEIG_OJA_TN_SLICES"))
    if (atoi(e) > 0) return atoi(e);
  const int64_t nfb = cdiv(d, TN_FEAT);
  int64_t ns = cdiv(2 * 4 * num_cus(), nfb * TN_WAVES);
  const int64_t cap = cdiv(b, 8 * TN_WAVES);
  if (ns > cap) ns = cap;
  return (int)(ns < 1 ? 1 : ns);
}

OjaWs carve_oja(void* ws, size_t cap, int64_t b, int64_t d, int kp, size_t* total) {
  Carve c(ws, cap);
  OjaWs o;
  const int64_t dpad = cdiv(d, TN_FEAT) * TN_FEAT;
  o.Vr = c.take<float>((size_t)d * kp);
  o.Vr2 = c.take<float>((size_t)d * kp);
  o.T = c.take<float>((size_t)b * kp);
  o.G = c.take<float>((size_t)kp * kp);
  o.Rinv = c.take<float>((size_t)kp * kp);
  o.Vc = c.take<float>((size_t)dpad * kp);
  o.part = c.take<float>((size_t)(dpad / TN_FEAT) * tn_slices(b, d) * TN_FEAT * kp);
  o.count = c.take<unsigned>((size_t)(dpad / TN_FEAT));
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

// Cholesky-QR2 of the row-padded d x kp basis in o.Vr (o.Vr2 is scratch); after
// the two passes (two buffer swaps) the result is back in o.Vr.
int cholqr2(const OjaWs& o, int64_t d, int k, int kp, hipStream_t st) {
  int rc;
  float* cur = o.Vr;
  float* nxt = o.Vr2;
  for (int pass = 0; pass < 2; ++pass) {
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
template <int NB>
void launch_batch(const OjaWs& o, const float* Xb, int64_t ldx, int64_t b, int64_t d, int64_t dpad,
                  float coef, int ns, hipStream_t st) {
  hipLaunchKernelGGL(oja_nn_kernel<NB>, dim3((unsigned)cdiv(b, NN_ROWS)), dim3(NN_THR), 0, st, Xb,
                     ldx, b, d, dpad, o.Vc, o.T);
  hipLaunchKernelGGL(oja_tn_kernel<NB>, dim3((unsigned)(dpad / TN_FEAT), (unsigned)ns),
                     dim3(TN_THR), 0, st, Xb, ldx, b, d, dpad, o.T, coef, o.Vc, o.part, o.count);
}

// The v2 path (d % 16 == 0; DEIG_OJA_KERNEL=1 selects the v1 skinny-GEMM path):
// per batch oja_nn_kernel + oja_tn_kernel on the column-major work basis Vc; the
// basis is copied to the row-padded layout of cholqr2 only at orthonormalisation.
int oja_steps_v2(const float* X, int64_t nb, int64_t b, int64_t d, int64_t ldx, float eta,
                 float* V, int k, int64_t ldv, int orth_every, const OjaWs& o, int kp,
                 hipStream_t st) {
  const int64_t dpad = cdiv(d, TN_FEAT) * TN_FEAT;
  const int ns = tn_slices(b, d);
  DEIG_HIP_CHECK(hipMemsetAsync(o.count, 0, sizeof(unsigned) * (dpad / TN_FEAT), st));
  hipLaunchKernelGGL(v_to_work, dim3((unsigned)cdiv(dpad * kp, 256)), dim3(256), 0, st, V, ldv, d,
                     dpad, k, kp, o.Vc);
  DEIG_HIP_CHECK(hipGetLastError());
  const float coef = eta / (float)b;
  int rc;
  for (int64_t i = 0; i < nb; ++i) {
    const float* Xb = X + i * b * ldx;
    switch (kp / 16) {
      case 1: launch_batch<1>(o, Xb, ldx, b, d, dpad, coef, ns, st); break;
      case 2: launch_batch<2>(o, Xb, ldx, b, d, dpad, coef, ns, st); break;
      case 3: launch_batch<3>(o, Xb, ldx, b, d, dpad, coef, ns, st); break;
      default: launch_batch<4>(o, Xb, ldx, b, d, dpad, coef, ns, st); break;
    }
    DEIG_HIP_CHECK(hipGetLastError());
    if ((i + 1) % orth_every == 0 || i + 1 == nb) {
      hipLaunchKernelGGL(work_to_rowpad, dim3((unsigned)cdiv(d * kp, 256)), dim3(256), 0, st, o.Vc,
                         dpad, d, kp, o.Vr);
      if ((rc = cholqr2(o, d, k, kp, st))) return rc;
      hipLaunchKernelGGL(rowpad_to_work, dim3((unsigned)cdiv(d * kp, 256)), dim3(256), 0, st, o.Vr,
                         d, dpad, kp, o.Vc);
      DEIG_HIP_CHECK(hipGetLastError());
    }
  }
  hipLaunchKernelGGL(rowpad_to_col, dim3((unsigned)cdiv(d * k, 256)), dim3(256), 0, st, o.Vr, d, k,
                     kp, V, ldv);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

int oja_kernel_version() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DEIG_OJA_KERNEL");
    v = (e && atoi(e) == 1) ? 1 : 2;
  }
  return v;
}

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
  if (d % 16 == 0 && ldx % 4 == 0 && aligned16(X) && oja_kernel_version() == 2)
    return oja_steps_v2(X, nb, b, d, ldx, eta, V, k, ldv, orth_every, o, kp, st);
  int rc;
  hipLaunchKernelGGL(col_to_rowpad, dim3((unsigned)cdiv(d * kp, 256)), dim3(256), 0, st, V, ldv, d,
                     k, kp, o.Vr);
  DEIG_HIP_CHECK(hipGetLastError());
  for (int64_t i = 0; i < nb; ++i) {
    const float* Xb = X + i * b * ldx;
    // T = Xb V
    if ((rc = skinny_launch(false, Xb, ldx, o.Vr, kp, o.T, kp, b, kp, d, 1.f, 0.f, o.slab,
                            o.slab_bytes, st)))
      return rc;
    // V += eta/b * Xb^T T
    if ((rc = skinny_launch(true, Xb, ldx, o.T, kp, o.Vr, kp, d, kp, b, eta / (float)b, 1.f,
                            o.slab, o.slab_bytes, st)))
      return rc;
    if ((i + 1) % orth_every == 0 || i + 1 == nb)
      if ((rc = cholqr2(o, d, k, kp, st))) return rc;
  }
  hipLaunchKernelGGL(rowpad_to_col, dim3((unsigned)cdiv(d * k, 256)), dim3(256), 0, st, o.Vr, d, k,
                     kp, V, ldv);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

int oja_launch(const float* Xb, int64_t b, int64_t d, int64_t ldx, float eta, float* V, int k,
               int64_t ldv, void* ws, size_t ws_bytes, hipStream_t st) {
  return oja_steps_launch(Xb, 1, b, d, ldx, eta, V, k, ldv, 1, ws, ws_bytes, st);
}

}  // namespace deig
