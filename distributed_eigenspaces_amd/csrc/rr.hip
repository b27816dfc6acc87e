// Rayleigh-Ritz step of the block subspace-iteration eigensolver that replaces
// LAPACK dsyevr in Node.top_k_eigenvectors (distributed.py:22-29).
//
// Per sweep the driver (capi.hip) keeps Z = [Q | Y] (d x 2p, row-major) with
// Y = A Q, forms the Gram C = Z^T Z (skinny GEMM) and then:
//
//  rr_small_kernel (ONE workgroup, p <= 128, everything in LDS):
//    M = Q^T Q, H = Q^T Y, G = Y^T Y taken from C;
//    D = diag(M)^-1/2;  D M D = L L^T (Cholesky, pivots floored);
//    H~ = L^-1 (D H D) L^-T;  H~ = U diag(lambda) U^T by parallel cyclic Jacobi
//    (round-robin pairing, p/2 rotations per step, both sides applied from one
//    read of the old matrix);  W = D L^-T U  (so the Ritz vectors Q W are
//    orthonormal even when Q is not);  g_j = || Y w_j ||^2 = (W^T G W)_jj;
//    columns sorted by descending lambda.  Generalised RR = robust to a
//    non-orthonormal or numerically rank-deficient Q.
//  rr_update_kernel (row-parallel):
//    Ritz vectors V = Q W, their images S V = Y W;
//    residual ||Y w_j - lambda_j Q w_j|| for the top k (fp32, no cancellation);
//    next basis Q <- Y W diag(g)^-1/2 (one power step on the Ritz vectors;
//    columns with g ~ 0 - null directions of A - keep Q w_j);
//    the top-k Ritz vectors are written to V (column-major, ascending order).
//  rr_finish_kernel: relative residuals, eigenvalues (ascending) and their max.
#include <algorithm>

#include "deig_internal.hpp"

namespace deig {
namespace {

constexpr int RT = 1024;
constexpr int UR = 32;  // rows per rr_update block

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Start basis: Q0's k0 columns, then pseudo-random columns.  Rows >= valid are zero
// (the zero padding of a staged S, capi.hip: its directions then never enter the
// basis - S Q, the shift, deflation and Rayleigh-Ritz all keep zero rows zero).
__global__ __launch_bounds__(256) void rr_init_kernel(float* __restrict__ Z, int64_t d, int p,
                                                      const float* __restrict__ Q0, int k0,
                                                      int64_t ldq0, uint64_t seed, int64_t valid) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * p) return;
  const int64_t r = idx / p;
  const int j = (int)(idx - r * p);
  float v;
  if (r >= valid) {
    v = 0.f;
  } else if (j < k0) {
    v = Q0[r + (int64_t)j * ldq0];
  } else {
    const uint64_t h = mix64(seed ^ mix64((uint64_t)r * 0x100000001B3ull + (uint64_t)j));
    v = (float)((double)(h >> 11) * (1.0 / 9007199254740992.0)) * 2.0f - 1.0f;
  }
  Z[r * 2 * p + j] = v;
}

// C = A B for p x p row-major matrices in LDS (p % 4 == 0, p <= 128): thread tid
// owns the 4 x 4 block at (a0, b0) and returns it in acc (false: no block).  Per
// 4-wide k step: 4 + 4 ds_read_b128 for 64 FMAs into independent accumulators
// (the former one-output-per-thread loops were LDS-latency-bound chains).
__device__ __forceinline__ bool lds_gemm4(const float* A, const float* B, int p, int tid,
                                          float (&acc)[4][4], int& a0, int& b0) {
  const int nt = p >> 2;
  const bool act = tid < nt * nt;
  const int tr = act ? tid / nt : 0;
  a0 = 4 * tr;
  b0 = 4 * (tid - tr * nt);
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = 0.f;
  if (!act) return false;
  for (int t = 0; t < p; t += 4) {
    f32x4 ar[4], br[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) ar[r] = *reinterpret_cast<const f32x4*>(A + (a0 + r) * p + t);
#pragma unroll
    for (int u = 0; u < 4; ++u) br[u] = *reinterpret_cast<const f32x4*>(B + (t + u) * p + b0);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(ar[r][u], br[u][c], acc[r][c]);
  }
  return true;
}

// Jacobi rotation (c, s) zeroing apq of [[app, apq], [apq, aqq]].  Hardware rcp /
// sqrt / rsq (~1 ulp): the rotation only has to be orthogonal to rounding
// (c = rsq(1 + t^2), s = t c), not the exact minimiser, and it sits on the
// latency chain of every Jacobi step.
__device__ __forceinline__ void rr_rot_cs(float app, float aqq, float apq, float& c, float& s) {
  const float tau = (aqq - app) * __builtin_amdgcn_rcpf(2.f * apq);
  const float t = (fabsf(tau) > 1e18f)
                      ? 0.5f * __builtin_amdgcn_rcpf(tau)
                      : copysignf(__builtin_amdgcn_rcpf(
                                      fabsf(tau) + __builtin_amdgcn_sqrtf(1.f + tau * tau)),
                                  tau);
  c = __builtin_amdgcn_rsqf(1.f + t * t);
  s = t * c;
}

template <int NT>
__device__ __forceinline__ void rr_small_body(const float* __restrict__ Cg, int p,
                                              float* __restrict__ Wout, float* __restrict__ lam_out,
                                              float* __restrict__ cs_out, float* __restrict__ qs_out,
                                              int* __restrict__ info, int max_jsweeps, float jrel) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int pp = p * p;
  const int half = p >> 1;
  float* X1 = sm;
  float* X2 = sm + pp;
  float* dsc = X2 + pp;   // p
  float* lamv = dsc + p;  // p
  float* gd = lamv + p;   // p
  // p/2 rotations {cos, sin, row a, row b} (16-byte aligned: p % 16 == 0)
  f32x4* rotp = reinterpret_cast<f32x4*>(gd + p);
  int* rank = reinterpret_cast<int*>(rotp + half);  // p
  float* nq = reinterpret_cast<float*>(rank + p);   // p: ||Q w_j||^2
  float* red = nq + p;                              // NT/64 + 2
  int* nrot = reinterpret_cast<int*>(red + NT / 64 + 2);
  const int tid = threadIdx.x;
  const int ldc = 2 * p;
  const float* Mg = Cg;
  const float* Hg = Cg + p;
  const float* Gg = Cg + (int64_t)p * ldc + p;
  // Phase clock (100 MHz realtime counter) into info[4..8] for DEIG_DEBUG.
  const uint64_t t0 = wall_clock64();
  auto stamp = [&](int slot) {
    if (tid == 0) info[slot] = (int)(wall_clock64() - t0);
  };

  // ---- 0. D = diag(M)^-1/2;  X1 = D M D
  for (int a = tid; a < p; a += NT) {
    const float m = Mg[a * ldc + a];
    dsc[a] = (m > 0.f && isfinite(m)) ? rsqrtf(m) : 1.0f;
  }
  if (tid == 0) {
    info[0] = 0;
    info[1] = 0;
    info[2] = 0;
    info[3] = 0;  // 1 once the Jacobi iteration has converged (not stopped by the cap)
  }
  __syncthreads();
  for (int idx = tid; idx < pp; idx += NT) {
    const int a = idx / p, b = idx - a * p;
    X1[idx] = Mg[a * ldc + b] * dsc[a] * dsc[b];
  }
  __syncthreads();

  // Thread groups for the triangular steps: eight consecutive lanes per row
  // (or column) split every dot product, reduced with three xor-shuffles.
  const int grp = tid >> 3, part = tid & 7;
  auto sum8 = [](float v) {
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    return v;
  };

  // ---- 1. Cholesky  D M D = L L^T  (left-looking, lower, in place in X1), pivots
  //         floored.  Step j: group g finishes row i = j + g of column j from the
  //         finished columns t < j - both dots split over its 8 lanes - and
  //         recomputes the pivot itself, so one barrier per column.  The pivots
  //         go to gd[] (X1's diagonal still holds D M D's, read by every group)
  //         and onto the diagonal after the loop.
  constexpr int NG = NT / 8;  // lane groups
  for (int j = 0; j < p; ++j) {
    for (int i = j + grp; i < p; i += NG) {
      float sd = 0.f, so = 0.f;
      for (int t = part; t < j; t += 8) {
        const float ljt = X1[j * p + t];
        sd = fmaf(ljt, ljt, sd);
        so = fmaf(X1[i * p + t], ljt, so);
      }
      sd = sum8(sd);
      so = sum8(so);
      float v = X1[j * p + j] - sd;
      // A pivot below 1e-6 (the column's part independent of the earlier ones is
      // < 1e-3 of its norm: numerically dependent) decouples the column: unit
      // pivot, zero sub-diagonal.  Its orthogonalised vector is then the tiny
      // Gram-Schmidt residual (Ritz value ~0, renormalised in rr_update by qs),
      // and L^-1 stays bounded - dividing the sub-diagonal by a floored pivot
      // grew L^-1 geometrically over consecutive dependent columns (r02: inf).
      const bool floored = !(v > 1e-6f);
      const float ljj = floored ? 1.0f : sqrtf(v);
      if (part == 0) {
        if (i == j) {
          gd[j] = ljj;
          if (floored) info[0] += 1;
        } else {
          X1[i * p + j] = floored ? 0.f : (X1[i * p + j] - so) / ljj;
        }
      }
    }
    __syncthreads();
  }
  for (int a = tid; a < p; a += NT) X1[a * p + a] = gd[a];
  for (int idx = tid; idx < pp; idx += NT) X2[idx] = 0.f;
  __syncthreads();
  stamp(4);

  // ---- 2. L^-1 (lower) into X2, row by row; group c owns column c of row i,
  //         its dot over t in [c, i) split over the group's 8 lanes.
  for (int i = 0; i < p; ++i) {
    for (int c = grp; c <= i; c += NG) {
      float sacc = 0.f;
      for (int t = c + part; t < i; t += 8) sacc = fmaf(X1[i * p + t], X2[t * p + c], sacc);
      sacc = sum8(sacc);
      if (part == 0) X2[i * p + c] = ((c == i ? 1.0f : 0.0f) - sacc) / X1[i * p + i];
    }
    __syncthreads();
  }
  stamp(5);

  // ---- 3. X1 = D H D ; 4. T = L^-1 X1, stored transposed (X1 = T^T = X1^T L^-T);
  //         5. X1 = L^-1 X1 = L^-1 H^T L^-T (symmetrised below: the same H~).
  //         Register-blocked 4 x 4 products (lds_gemm4).
  for (int idx = tid; idx < pp; idx += NT) {
    const int a = idx / p, b = idx - a * p;
    X1[idx] = Hg[a * ldc + b] * dsc[a] * dsc[b];
  }
  __syncthreads();
  {
    float acc[4][4];
    int a0, b0;
    bool act = lds_gemm4(X2, X1, p, tid, acc, a0, b0);
    __syncthreads();
    if (act)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) X1[(b0 + c) * p + a0 + r] = acc[r][c];
    __syncthreads();
    act = lds_gemm4(X2, X1, p, tid, acc, a0, b0);
    __syncthreads();
    if (act)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) X1[(a0 + r) * p + b0 + c] = acc[r][c];
    __syncthreads();
  }
  // symmetrise H~ and turn X2 = L^-1 into the eigenvector accumulator V0 = L^-T:
  // every Jacobi rotation right-multiplies it, so at the end X2 = L^-T U.
  for (int idx = tid; idx < pp; idx += NT) {
    const int a = idx / p, b = idx - a * p;
    if (a < b) {
      const float v = 0.5f * (X1[a * p + b] + X1[b * p + a]);
      X1[a * p + b] = v;
      X1[b * p + a] = v;
      const float l = X2[b * p + a];  // L^-1 is lower: (b, a) holds the value
      X2[a * p + b] = l;
      X2[b * p + a] = 0.f;
    }
  }
  __syncthreads();

  stamp(6);
  // ---- 6. parallel cyclic Jacobi on X1 (round-robin pairs; each thread owns a 2x2
  //         block of the rotated matrix, updated in place from one read).
  // nrot[0]: rotations in this sweep; nrot[1], nrot[2]: per-step counters used on
  // alternating steps, so a counter is only reset after every thread has read it.
  if (tid == 0) {
    nrot[1] = 0;
    nrot[2] = 0;
  }
  // idx = tid + u NT  ->  (idx / half, idx % half), stepped without divisions
  const int tr0 = tid / half, tc0 = tid - tr0 * half;
  const int dq = NT / half, dr = NT - dq * half;
  for (int sw = 0; sw < max_jsweeps; ++sw) {
    if (tid == 0) nrot[0] = 0;
    // scale for the absolute rotation threshold
    float dmax = 0.f;
    for (int a = tid; a < p; a += NT) dmax = fmaxf(dmax, fabsf(X1[a * p + a]));
    for (int o = 32; o > 0; o >>= 1) dmax = fmaxf(dmax, __shfl_xor(dmax, o, 64));
    if ((tid & 63) == 0) red[tid >> 6] = dmax;
    __syncthreads();
    float amax = 0.f;
    for (int i = 0; i < NT / 64; ++i) amax = fmaxf(amax, red[i]);
    const float abs_thr = 1e-9f * amax;
    // Convergence pre-check (one pass, one barrier): if no pair passes the
    // rotation test now, the first step rotates nothing, the matrix stays as it
    // is and so does every later step - the sweep would be a no-op.  Saves the
    // all-identity sweep that used to end every solve (p - 1 steps, 2 barriers each).
    {
      int need = 0;
      for (int idx = tid; idx < p * p && !need; idx += NT) {
        const int a = idx / p, b = idx - a * p;
        if (b < a) {
          const float apq = X1[a * p + b];
          need = fabsf(apq) > abs_thr &&
                 fabsf(apq) > jrel * sqrtf(fabsf(X1[a * p + a] * X1[b * p + b]));
        }
      }
      need = __syncthreads_or(need);
      if (!need) {
        if (tid == 0) info[3] = 1;
        break;
      }
    }
    for (int st = 0; st < p - 1; ++st) {
      const int ci = 1 + (st & 1);
      if (tid < half) {
        int a, b;
        if (tid == 0) {
          a = p - 1;
          b = st;
        } else {
          a = (st + tid) % (p - 1);
          b = (st - tid + (p - 1)) % (p - 1);
        }
        const float app = X1[a * p + a], aqq = X1[b * p + b], apq = X1[a * p + b];
        float c = 1.f, s = 0.f;
        if (fabsf(apq) > abs_thr &&
            fabsf(apq) > jrel * __builtin_amdgcn_sqrtf(fabsf(app * aqq))) {
          rr_rot_cs(app, aqq, apq, c, s);
          atomicAdd(nrot + ci, 1);
        }
        rotp[tid] = f32x4{c, s, __int_as_float(a), __int_as_float(b)};
      }
      __syncthreads();
      const int step_rot = nrot[ci];
      if (step_rot != 0) {  // wave-uniform: identity steps apply nothing
        int tr = tr0, tc = tc0;
        for (int idx = tid; idx < half * half; idx += NT) {
          const f32x4 qr = rotp[tr], qc = rotp[tc];
          const int ar = __float_as_int(qr[2]), br = __float_as_int(qr[3]);
          const int ac = __float_as_int(qc[2]), bc = __float_as_int(qc[3]);
          const float cr = qr[0], sr = qr[1], cc = qc[0], sc = qc[1];
          const float x = X1[ar * p + ac], y = X1[ar * p + bc];
          const float z = X1[br * p + ac], w = X1[br * p + bc];
          // columns: col_a' = c col_a - s col_b ; col_b' = s col_a + c col_b
          const float x1 = cc * x - sc * y, y1 = sc * x + cc * y;
          const float z1 = cc * z - sc * w, w1 = sc * z + cc * w;
          // rows
          X1[ar * p + ac] = cr * x1 - sr * z1;
          X1[br * p + ac] = sr * x1 + cr * z1;
          X1[ar * p + bc] = cr * y1 - sr * w1;
          X1[br * p + bc] = sr * y1 + cr * w1;
          tr += dq;
          tc += dr;
          if (tc >= half) {
            tc -= half;
            ++tr;
          }
        }
        tr = tr0;
        tc = tc0;
        for (int idx = tid; idx < p * half; idx += NT) {
          const int r = tr, t = tc;
          tr += dq;
          tc += dr;
          if (tc >= half) {
            tc -= half;
            ++tr;
          }
          const f32x4 qt = rotp[t];
          const int a = __float_as_int(qt[2]), b = __float_as_int(qt[3]);
          const float c = qt[0], s = qt[1];
          const float va = X2[r * p + a], vb = X2[r * p + b];
          X2[r * p + a] = c * va - s * vb;
          X2[r * p + b] = s * va + c * vb;
        }
      }
      __syncthreads();
      if (tid == 0) {
        nrot[0] += step_rot;
        nrot[ci] = 0;
      }
    }
    __syncthreads();
    const int swrot = nrot[0];
    if (tid == 0) {
      info[1] = sw + 1;
      info[2] += swrot;
    }
    __syncthreads();
    if (swrot == 0) {
      if (tid == 0) info[3] = 1;
      break;
    }
  }

  stamp(7);
  // ---- 7. eigenvalues; W = D (L^-T U)  (row scaling, in place in X2)
  for (int a = tid; a < p; a += NT) lamv[a] = X1[a * p + a];
  __syncthreads();
  for (int idx = tid; idx < pp; idx += NT) {
    const int a = idx / p, b = idx - a * p;
    X2[idx] *= dsc[a];
    X1[idx] = Gg[a * ldc + b];
  }
  __syncthreads();
  // ---- 8. g_j = w_j^T G w_j:  X1 = (G W) .* W, column sums below
  {
    float acc[4][4];
    int a0, b0;
    const bool act = lds_gemm4(X1, X2, p, tid, acc, a0, b0);
    __syncthreads();
    if (act)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          X1[(a0 + r) * p + b0 + c] = acc[r][c] * X2[(a0 + r) * p + b0 + c];
    __syncthreads();
  }
  for (int j = tid; j < p; j += NT) {
    float s = 0.f;
    for (int a = 0; a < p; ++a) s += X1[a * p + j];
    gd[j] = s;
  }
  __syncthreads();
  // ---- 9. n_j = w_j^T M w_j = ||Q w_j||^2: 1 up to rounding when D M D was
  //         factored exactly, but not for columns whose pivot was floored (a
  //         numerically dependent Q): their Ritz vectors are renormalised by it,
  //         or repeated floored RR steps compound their norms until they overflow.
  for (int idx = tid; idx < pp; idx += NT) {
    const int a = idx / p, b = idx - a * p;
    X1[idx] = Mg[a * ldc + b];
  }
  __syncthreads();
  {
    float acc[4][4];
    int a0, b0;
    const bool act = lds_gemm4(X1, X2, p, tid, acc, a0, b0);
    __syncthreads();
    if (act)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          X1[(a0 + r) * p + b0 + c] = acc[r][c] * X2[(a0 + r) * p + b0 + c];
    __syncthreads();
  }
  for (int j = tid; j < p; j += NT) {
    float s = 0.f;
    for (int a = 0; a < p; ++a) s += X1[a * p + j];
    nq[j] = s;
    const float lj = lamv[j];
    int rk = 0;
    for (int b = 0; b < p; ++b) {
      const float lb = lamv[b];
      rk += (lb > lj || (lb == lj && b < j)) ? 1 : 0;
    }
    rank[j] = rk;
  }
  __syncthreads();
  if (tid == 0) {
    float mx = 0.f;
    for (int j = 0; j < p; ++j) mx = fmaxf(mx, gd[j]);
    red[0] = mx;
  }
  __syncthreads();
  const float gthr = red[0] * 1e-10f;
  for (int j = tid; j < p; j += NT) {
    const int rk = rank[j];
    lam_out[rk] = lamv[j];
    cs_out[rk] = (gd[j] > gthr && gd[j] > 0.f) ? rsqrtf(gd[j]) : 0.f;
    qs_out[rk] = (nq[j] > 1e-30f && isfinite(nq[j])) ? rsqrtf(nq[j]) : 1.f;
  }
  for (int idx = tid; idx < pp; idx += NT) {
    const int a = idx / p, j = idx - a * p;
    Wout[a * p + rank[j]] = X2[idx];
  }
  stamp(8);
}

// ---------------------------------------------------------------- small solve v2
// The same generalised Rayleigh-Ritz step as rr_small_body (same outputs, same
// decisions), restructured for the barrier / LDS-instruction budget of ONE
// workgroup (r04: rr_small_body spent ~1.4 us per Jacobi step at p = 80 - 2 barriers
// and ~40 LDS instructions per thread - and 2 x p barriers in the column-by-column
// Cholesky and L^-1):
//  * Cholesky of D M D and L^-1 in 16-column blocks: each 16 x 16 diagonal block is
//    factored and inverted by one wave in registers (readlane broadcasts, no
//    barrier), panels / trailing updates / block products are LDS-tiled products -
//    ~4 barriers per block instead of 32;
//  * Jacobi on the LOWER triangle only (half the block updates; stored with row
//    stride p + 1 so column-strided accesses spread over the banks) and the
//    eigenvector accumulator V held in REGISTERS: the round-robin ordering is the
//    circle method, so the logical columns a pair slot holds move one slot per step in
//    a fixed pattern (a-players down, b-players up); a row of V is split over 4 lanes
//    (p / 8 slots each) that pass 2 values per step to their neighbours by shuffles.
// Numerically: the Cholesky is right-looking by blocks (rounding order differs from
// rr_small_body), the pivot floor and every later decision are the same.
__device__ __forceinline__ float rdl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// One wave: Cholesky of the 16 x 16 block at (o, o) of X1 (row stride p, already
// updated by the earlier blocks), written back as L_JJ (lower; pivots floored as in
// rr_small_body: v <= 1e-6 -> unit pivot, zero sub-diagonal); L_JJ^-1 written to the
// diagonal block of X2 (row-major, zero upper) and to LS (16 x 17, row-major padded).
__device__ __forceinline__ void chol16_wave(float* X1, float* X2, float* LS, int* flo, int p, int o,
                                            int lane, int* info) {
  float a[16];
  const bool act = lane < 16;
  const int row = act ? lane : 0;
#pragma unroll
  for (int j = 0; j < 16; j += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(X1 + (o + row) * p + o + j);
    a[j] = v[0];
    a[j + 1] = v[1];
    a[j + 2] = v[2];
    a[j + 3] = v[3];
  }
  int nfl = 0;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const float v = rdl(a[c], c);
    const bool floored = !(v > 1e-6f);
    const float ljj = floored ? 1.0f : sqrtf(v);
    nfl += floored ? 1 : 0;
    if (lane == c) a[c] = ljj;
    else if (lane > c) a[c] = floored ? 0.f : a[c] / ljj;
    if (lane == 0) flo[o + c] = floored ? 1 : 0;
#pragma unroll
    for (int j = c + 1; j < 16; ++j) {
      const float ljc = rdl(a[c], j);
      if (lane >= j) a[j] = fmaf(-a[c], ljc, a[j]);
    }
  }
  if (lane == 0 && nfl) info[0] += nfl;
  // L_JJ^-1: lane j computes column j, x[i] = (delta_ij - sum_{t<i} l_it x_t) / l_ii
  float x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float s = (i == lane) ? 1.f : 0.f;
#pragma unroll
    for (int t = 0; t < i; ++t) s = fmaf(-rdl(a[t], i), x[t], s);
    x[i] = (i >= lane) ? s / rdl(a[i], i) : 0.f;
  }
  if (act) {
#pragma unroll
    for (int j = 0; j < 16; ++j) X1[(o + lane) * p + o + j] = j <= lane ? a[j] : 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      X2[(o + t) * p + o + lane] = x[t];  // Linv[t][lane]
      LS[t * 17 + lane] = x[t];
    }
  }
}

// 4 x 4 tile product acc += A[r0 + r][k] * B[k][c0 + c] over k in [k0, k1), A and B
// row-major in LDS with row strides lda / ldb (16-B aligned rows).
__device__ __forceinline__ void tile44(const float* A, int lda, const float* B, int ldb, int r0, int c0,
                                       int k0, int k1, float (&acc)[4][4]) {
  for (int k = k0; k < k1; k += 4) {
    f32x4 ar[4], br[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) ar[r] = *reinterpret_cast<const f32x4*>(A + (r0 + r) * lda + k);
#pragma unroll
    for (int u = 0; u < 4; ++u) br[u] = *reinterpret_cast<const f32x4*>(B + (k + u) * ldb + c0);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(ar[r][u], br[u][c], acc[r][c]);
  }
}

// lower-triangle item idx -> (r, c), r >= c
__device__ __forceinline__ void tri_rc(int idx, int& r, int& c) {
  int t = (int)((sqrtf(8.f * (float)idx + 1.f) - 1.f) * 0.5f);
  while ((t + 1) * (t + 2) / 2 <= idx) ++t;
  while (t * (t + 1) / 2 > idx) --t;
  r = t;
  c = idx - t * (t + 1) / 2;
}

template <int NT>
__device__ __forceinline__ void rr_small2_body(const float* __restrict__ Cg, int p,
                                               float* __restrict__ Wout, float* __restrict__ lam_out,
                                               float* __restrict__ cs_out, float* __restrict__ qs_out,
                                               int* __restrict__ info, int max_jsweeps, float jrel) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int pp = p * p;
  const int half = p >> 1;
  const int nbk = p >> 4;
  const int ldp = p + 4;  // panel scratch row stride
  float* X1 = sm;
  float* X2 = sm + pp;         // p x (p + 1)
  float* dsc = X2 + pp + p;    // p
  float* lamv = dsc + p;       // p
  float* gd = lamv + p;        // p
  f32x4* rotp = reinterpret_cast<f32x4*>(gd + p);  // half records {c, s, a, b}
  int* rank = reinterpret_cast<int*>(rotp + half);  // p
  float* nq = reinterpret_cast<float*>(rank + p);   // p
  int* flo = reinterpret_cast<int*>(nq + p);        // p
  float* LS = reinterpret_cast<float*>(flo + p);    // 16 x 17 (+ 4 pad)
  float* pan = LS + 16 * 17 + 4;                    // 16 x (p + 4)
  float* red = pan + 16 * ldp;                      // NT / 64 + 2
  int* nrot = reinterpret_cast<int*>(red + NT / 64 + 2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ldc = 2 * p;
  const float* Mg = Cg;
  const float* Hg = Cg + p;
  const float* Gg = Cg + (int64_t)p * ldc + p;
  const uint64_t t0 = wall_clock64();
  auto stamp = [&](int slot) {
    if (tid == 0) info[slot] = (int)(wall_clock64() - t0);
  };

  // ---- 0. D = diag(M)^-1/2; X1 = D M D; X2 = 0
  for (int a = tid; a < p; a += NT) {
    const float m = Mg[a * ldc + a];
    dsc[a] = (m > 0.f && isfinite(m)) ? rsqrtf(m) : 1.0f;
  }
  if (tid == 0) {
    info[0] = 0;
    info[1] = 0;
    info[2] = 0;
    info[3] = 0;
  }
  __syncthreads();
  for (int idx = tid; idx < pp; idx += NT) {
    const int a = idx / p, b = idx - a * p;
    X1[idx] = Mg[a * ldc + b] * dsc[a] * dsc[b];
    X2[idx] = 0.f;
  }
  __syncthreads();

  // ---- 1. blocked Cholesky D M D = L L^T (lower, in X1), L_JJ^-1 into X2's diagonal
  for (int J = 0; J < nbk; ++J) {
    const int o = 16 * J;
    if (wave == 0) chol16_wave(X1, X2, LS, flo, p, o, lane, info);
    __syncthreads();
    const int rem = p - o - 16;
    if (rem <= 0) break;
    // panel L_IJ = A_IJ L_JJ^-T (floored columns zero) -> pan[c][i], transposed
    for (int it = tid; it < rem * 16; it += NT) {
      const int c = it & 15, i = o + 16 + (it >> 4);
      float s = 0.f;
#pragma unroll
      for (int t = 0; t < 16; ++t) s = fmaf(X1[i * p + o + t], LS[c * 17 + t], s);
      pan[c * ldp + i] = flo[o + c] ? 0.f : s;
    }
    __syncthreads();
    // L_IJ into X1; trailing lower update A_II' -= L_IJ L_I'J^T (4 x 4 tiles)
    for (int it = tid; it < rem * 16; it += NT) {
      const int c = it & 15, i = o + 16 + (it >> 4);
      X1[i * p + o + c] = pan[c * ldp + i];
    }
    const int nt = rem >> 2;
    for (int it = tid; it < nt * (nt + 1) / 2; it += NT) {
      int ti, tj;
      tri_rc(it, ti, tj);
      const int i0 = o + 16 + 4 * ti, j0 = o + 16 + 4 * tj;
      float acc[4][4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = 0.f;
#pragma unroll 4
      for (int c = 0; c < 16; ++c) {
        const f32x4 li = *reinterpret_cast<const f32x4*>(pan + c * ldp + i0);
        const f32x4 lj = *reinterpret_cast<const f32x4*>(pan + c * ldp + j0);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) acc[r][cc] = fmaf(li[r], lj[cc], acc[r][cc]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        f32x4* dst = reinterpret_cast<f32x4*>(X1 + (i0 + r) * p + j0);
        f32x4 v = *dst;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) v[cc] -= acc[r][cc];
        *dst = v;
      }
    }
    __syncthreads();
  }
  stamp(4);

  // ---- 2. L^-1 (lower) into X2 by block rows.  M_IK = L_II^-1 L_IK (K < I), stored
  //         transposed in X1's (unused) upper triangle; then X_IJ = -sum_K M_IK X_KJ.
  for (int it = tid; it < (nbk * (nbk - 1) / 2) * 16; it += NT) {
    int I, K;
    tri_rc(it >> 4, I, K);
    I += 1;  // strictly lower blocks: (I, K) with I > K
    const int tl = it & 15, i0 = 16 * I + 4 * (tl >> 2), j0 = 16 * K + 4 * (tl & 3);
    float acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[r][c] = 0.f;
    // Linv_II[i][t] (X2 diagonal block) x L_IK[t][j] (X1)
    tile44(X2 + 16 * I, p, X1 + 16 * I * p, p, i0, j0, 0, 16, acc);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      f32x4 v{acc[0][c], acc[1][c], acc[2][c], acc[3][c]};
      *reinterpret_cast<f32x4*>(X1 + (j0 + c) * p + i0) = v;  // M^T: row j, cols i (upper)
    }
  }
  __syncthreads();
  for (int I = 1; I < nbk; ++I) {
    for (int it = tid; it < I * 16; it += NT) {
      const int J = it >> 4, tl = it & 15;
      const int i0 = 16 * I + 4 * (tl >> 2), j0 = 16 * J + 4 * (tl & 3);
      float acc[4][4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = 0.f;
      for (int k = 16 * J; k < 16 * I; ++k) {
        const f32x4 m = *reinterpret_cast<const f32x4*>(X1 + k * p + i0);  // M_I.[i0..i0+3][k]
        const f32x4 xk = *reinterpret_cast<const f32x4*>(X2 + k * p + j0);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(m[r], xk[c], acc[r][c]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *reinterpret_cast<f32x4*>(X2 + (i0 + r) * p + j0) =
            f32x4{-acc[r][0], -acc[r][1], -acc[r][2], -acc[r][3]};
    }
    __syncthreads();
  }
  stamp(5);

  // ---- 3. X1 = D H D; T = L^-1 X1 stored transposed; X1 = L^-1 T^T = L^-1 H L^-T
  for (int idx = tid; idx < pp; idx += NT) {
    const int a = idx / p, b = idx - a * p;
    X1[idx] = Hg[a * ldc + b] * dsc[a] * dsc[b];
  }
  __syncthreads();
  const int nt4 = p >> 2;
  for (int pass = 0; pass < 2; ++pass) {
    constexpr int MAXT = (1024 + NT - 1) / NT;  // p <= 128: (p/4)^2 <= 1024 tiles
    float acc[MAXT][4][4];
#pragma unroll
    for (int u = 0; u < MAXT; ++u) {
      const int it = tid + u * NT;
      if (it < nt4 * nt4) {
        const int a0 = 4 * (it / nt4), b0 = 4 * (it % nt4);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[u][r][c] = 0.f;
        tile44(X2, p, X1, p, a0, b0, 0, a0 + 4, acc[u]);  // L^-1 lower: k <= a0 + 3
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < MAXT; ++u) {
      const int it = tid + u * NT;
      if (it < nt4 * nt4) {
        const int a0 = 4 * (it / nt4), b0 = 4 * (it % nt4);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if (pass == 0) X1[(b0 + c) * p + a0 + r] = acc[u][r][c];
            else X1[(a0 + r) * p + b0 + c] = acc[u][r][c];
          }
      }
    }
    __syncthreads();
  }
  stamp(6);

  // ---- 4. Jacobi (rr_small_body's: full storage, round-robin pairs, 2 barriers per
  //         step; r04 A/B: every restructured step measured slower - V in registers
  //         moved along the circle method, lower-triangle storage, rotations per wave
  //         by shuffles - their extra VALU / shuffle issue cost more than the LDS
  //         traffic they saved, profiles/r04d_rr_phases.log).
  //         symmetrise H~; X2 = L^-1 -> the eigenvector accumulator V0 = L^-T, kept
  //         transposed (X2 = V^T, as L^-1 already is): a column pair's rotation then
  //         updates two contiguous rows, 4 entries per b128 LDS access (r06: the
  //         scalar-column V update was ~28 % of a Jacobi step, profiles/r06aq_*)
  for (int idx = tid; idx < pp; idx += NT) {
    const int a = idx / p, b = idx - a * p;
    if (a < b) {
      const float v = 0.5f * (X1[a * p + b] + X1[b * p + a]);
      X1[a * p + b] = v;
      X1[b * p + a] = v;
#if defined(DEIG_AB_RR_JOLD) || defined(DEIG_AB_RR_VROW)
      const float l = X2[b * p + a];
      X2[a * p + b] = l;
      X2[b * p + a] = 0.f;
#else
      X2[a * p + b] = 0.f;
#endif
    }
  }
  if (tid == 0) {
    nrot[1] = 0;
    nrot[2] = 0;
  }
  __syncthreads();
  const int tr0 = tid / half, tc0 = tid - tr0 * half;
#ifdef DEIG_AB_RR_JOLD
  const int dq = NT / half, dr = NT - dq * half;
#else
  const int cpt = NT / half;
#ifndef DEIG_AB_RR_VROW
  // V^T items: (column pair t, quad q of its two rows), t-major so that a wave's lanes
  // walk contiguous quads of one row pair
  const int vnq = p >> 2;
  // (counted from the last thread: at small p the first waves carry the H~ update)
  const int vt0 = (NT - 1 - tid) / vnq, vq0 = (NT - 1 - tid) - vt0 * vnq;
  const int vdt = NT / vnq, vdq = NT - vdt * vnq;
#endif
#endif
  for (int sw = 0; sw < max_jsweeps; ++sw) {
    if (tid == 0) nrot[0] = 0;
    float dmax = 0.f;
    for (int a = tid; a < p; a += NT) dmax = fmaxf(dmax, fabsf(X1[a * p + a]));
    for (int o = 32; o > 0; o >>= 1) dmax = fmaxf(dmax, __shfl_xor(dmax, o, 64));
    if (lane == 0) red[wave] = dmax;
    __syncthreads();
    float amax = 0.f;
    for (int i = 0; i < NT / 64; ++i) amax = fmaxf(amax, red[i]);
    const float abs_thr = 1e-9f * amax;
    {
      int need = 0;
      for (int idx = tid; idx < pp && !need; idx += NT) {
        const int a = idx / p, b = idx - a * p;
        if (b < a) {
          const float apq = X1[a * p + b];
          need = fabsf(apq) > abs_thr && fabsf(apq) > jrel * sqrtf(fabsf(X1[a * p + a] * X1[b * p + b]));
        }
      }
      need = __syncthreads_or(need);
      if (!need) {
        if (tid == 0) info[3] = 1;
        break;
      }
    }
    // wave 0, lane t < half: the round-robin pair of step st, a = (st + t) mod (p - 1),
    // b = (st - t) mod (p - 1) (lane 0: a = p - 1, b = st), advanced by one per step
    int pa = tid == 0 ? p - 1 : tid, pb = tid == 0 ? 0 : p - 1 - tid;
    int swsum = 0;  // wave 0: this sweep's rotations
    for (int st = 0; st < p - 1; ++st) {
      const int ci = 1 + (st & 1);
#ifdef DEIG_AB_RR_JOLD
      if (tid < half) {
        int a, b;
        if (tid == 0) {
          a = p - 1;
          b = st;
        } else {
          a = (st + tid) % (p - 1);
          b = (st - tid + (p - 1)) % (p - 1);
        }
        const float app = X1[a * p + a], aqq = X1[b * p + b], apq = X1[a * p + b];
        float c = 1.f, s = 0.f;
        if (fabsf(apq) > abs_thr && fabsf(apq) > jrel * __builtin_amdgcn_sqrtf(fabsf(app * aqq))) {
          rr_rot_cs(app, aqq, apq, c, s);
          atomicAdd(nrot + ci, 1);
        }
        rotp[tid] = f32x4{c, s, __int_as_float(a), __int_as_float(b)};
      }
#else
      // the p / 2 <= 64 pairs of a step are one wave's lanes: the step's rotation count
      // is a ballot (64 LDS atomics on one address serialised ~0.2 us per step)
      if (wave == 0) {
        bool rot = false;
        if (tid < half) {
          const int a = pa, b = pb;
          if (tid != 0) pa = pa + 1 == p - 1 ? 0 : pa + 1;
          pb = pb + 1 == p - 1 ? 0 : pb + 1;
          const float app = X1[a * p + a], aqq = X1[b * p + b], apq = X1[a * p + b];
          float c = 1.f, s = 0.f;
          if (fabsf(apq) > abs_thr && fabsf(apq) > jrel * __builtin_amdgcn_sqrtf(fabsf(app * aqq))) {
            rr_rot_cs(app, aqq, apq, c, s);
            rot = true;
          }
          rotp[tid] = f32x4{c, s, __int_as_float(a), __int_as_float(b)};
        }
        const int cnt = __popcll(__ballot(rot));
        if (tid == 0) nrot[ci] = cnt;
        swsum += cnt;
      }
#endif
      __syncthreads();
      const int step_rot = nrot[ci];
      if (step_rot != 0) {
#ifdef DEIG_AB_RR_JOLD
        int tr = tr0, tc = tc0;
        for (int idx = tid; idx < half * half; idx += NT) {
          const f32x4 qr = rotp[tr], qc = rotp[tc];
          const int ar = __float_as_int(qr[2]), br = __float_as_int(qr[3]);
          const int ac = __float_as_int(qc[2]), bc = __float_as_int(qc[3]);
          const float cr = qr[0], sr = qr[1], cc = qc[0], sc = qc[1];
          const float x = X1[ar * p + ac], y = X1[ar * p + bc];
          const float z = X1[br * p + ac], w = X1[br * p + bc];
          const float x1 = cc * x - sc * y, y1 = sc * x + cc * y;
          const float z1 = cc * z - sc * w, w1 = sc * z + cc * w;
          X1[ar * p + ac] = cr * x1 - sr * z1;
          X1[br * p + ac] = sr * x1 + cr * z1;
          X1[ar * p + bc] = cr * y1 - sr * w1;
          X1[br * p + bc] = sr * y1 + cr * w1;
          tr += dq;
          tc += dr;
          if (tc >= half) {
            tc -= half;
            ++tr;
          }
        }
        tr = tr0;
        tc = tc0;
        for (int idx = tid; idx < p * half; idx += NT) {
          const int r = tr, t = tc;
          tr += dq;
          tc += dr;
          if (tc >= half) {
            tc -= half;
            ++tr;
          }
          const f32x4 qt = rotp[t];
          const int a = __float_as_int(qt[2]), b = __float_as_int(qt[3]);
          const float c = qt[0], s = qt[1];
          const float va = X2[r * p + a], vb = X2[r * p + b];
          X2[r * p + a] = c * va - s * vb;
          X2[r * p + b] = s * va + c * vb;
        }
#else
        // thread -> column pair tc0 and every cpt-th row pair (and V row): the column
        // pair's rotation record is read once per step instead of once per 2 x 2 block
        // and V item (the step is LDS-bound: at p = 128, 524 -> 360 KB per step)
        if (tid < cpt * half) {
          const f32x4 qc = rotp[tc0];
          const int ac = __float_as_int(qc[2]), bc = __float_as_int(qc[3]);
          const float cc = qc[0], sc = qc[1];
          for (int tr = tr0; tr < half; tr += cpt) {
            const f32x4 qr = rotp[tr];
            const int ar = __float_as_int(qr[2]), br = __float_as_int(qr[3]);
            const float cr = qr[0], sr = qr[1];
            const float x = X1[ar * p + ac], y = X1[ar * p + bc];
            const float z = X1[br * p + ac], w = X1[br * p + bc];
            const float x1 = cc * x - sc * y, y1 = sc * x + cc * y;
            const float z1 = cc * z - sc * w, w1 = sc * z + cc * w;
            X1[ar * p + ac] = cr * x1 - sr * z1;
            X1[br * p + ac] = sr * x1 + cr * z1;
            X1[ar * p + bc] = cr * y1 - sr * w1;
            X1[br * p + bc] = sr * y1 + cr * w1;
          }
#if defined(DEIG_AB_RR_VROW) && !defined(DEIG_AB_RR_NO_V)  // r05 layout (measurement builds)
          for (int r = tr0; r < p; r += cpt) {
            const float va = X2[r * p + ac], vb = X2[r * p + bc];
            X2[r * p + ac] = cc * va - sc * vb;
            X2[r * p + bc] = sc * va + cc * vb;
          }
#endif
        }
#if !defined(DEIG_AB_RR_VROW) && !defined(DEIG_AB_RR_NO_V)  // NO_V: knock-out, wrong vectors
        for (int t = vt0, q = vq0; t < half;) {
          const f32x4 qc = rotp[t];
          const float cc = qc[0], sc = qc[1];
          f32x4* pa = reinterpret_cast<f32x4*>(X2 + __float_as_int(qc[2]) * p) + q;
          f32x4* pb = reinterpret_cast<f32x4*>(X2 + __float_as_int(qc[3]) * p) + q;
          const f32x4 va = *pa, vb = *pb;
          f32x4 na, nb;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            na[e] = cc * va[e] - sc * vb[e];
            nb[e] = sc * va[e] + cc * vb[e];
          }
          *pa = na;
          *pb = nb;
          t += vdt;
          q += vdq;
          if (q >= vnq) {
            q -= vnq;
            ++t;
          }
        }
#endif
#endif
      }
      __syncthreads();
#ifdef DEIG_AB_RR_JOLD
      if (tid == 0) {
        nrot[0] += step_rot;
        nrot[ci] = 0;
      }
#endif
    }
#ifndef DEIG_AB_RR_JOLD
    if (tid == 0) nrot[0] = swsum;
#endif
    __syncthreads();
    const int swrot = nrot[0];
    if (tid == 0) {
      info[1] = sw + 1;
      info[2] += swrot;
    }
    __syncthreads();
    if (swrot == 0) {
      if (tid == 0) info[3] = 1;
      break;
    }
  }

  stamp(7);
  // ---- 5. eigenvalues; W = D (L^-T U) in X2 (row scaling in place); X1 = scratch
  for (int a = tid; a < p; a += NT) lamv[a] = X1[a * p + a];
#if !defined(DEIG_AB_RR_JOLD) && !defined(DEIG_AB_RR_VROW)
  for (int it = tid; it < nt4 * (nt4 + 1) / 2; it += NT) {  // V^T -> V by 4 x 4 blocks
    int ti, tj;
    tri_rc(it, ti, tj);
    f32x4 A[4], B[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      A[r] = *reinterpret_cast<const f32x4*>(X2 + (4 * ti + r) * p + 4 * tj);
      B[r] = *reinterpret_cast<const f32x4*>(X2 + (4 * tj + r) * p + 4 * ti);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      *reinterpret_cast<f32x4*>(X2 + (4 * ti + r) * p + 4 * tj) = f32x4{B[0][r], B[1][r], B[2][r], B[3][r]};
      *reinterpret_cast<f32x4*>(X2 + (4 * tj + r) * p + 4 * ti) = f32x4{A[0][r], A[1][r], A[2][r], A[3][r]};
    }
  }
#endif
  __syncthreads();
  for (int idx = tid; idx < pp; idx += NT) X2[idx] *= dsc[idx / p];
  float* Wm = X2;   // W = D L^-T U
  float* Ts = X1;   // scratch (ld p)
  for (int idx = tid; idx < pp; idx += NT) {
    const int a = idx / p, b = idx - a * p;
    Ts[idx] = Gg[a * ldc + b];
  }
  __syncthreads();
  // ---- 6. g_j = w_j^T G w_j, n_j = w_j^T M w_j: column sums of (G W) .* W, (M W) .* W
  for (int pass = 0; pass < 2; ++pass) {
    constexpr int MAXT = (1024 + NT - 1) / NT;
    float acc[MAXT][4][4];
#pragma unroll
    for (int u = 0; u < MAXT; ++u) {
      const int it = tid + u * NT;
      if (it < nt4 * nt4) {
        const int a0 = 4 * (it / nt4), b0 = 4 * (it % nt4);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[u][r][c] = 0.f;
        tile44(Ts, p, Wm, p, a0, b0, 0, p, acc[u]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < MAXT; ++u) {
      const int it = tid + u * NT;
      if (it < nt4 * nt4) {
        const int a0 = 4 * (it / nt4), b0 = 4 * (it % nt4);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) Ts[(a0 + r) * p + b0 + c] = acc[u][r][c] * Wm[(a0 + r) * p + b0 + c];
      }
    }
    __syncthreads();
    float* dst = pass == 0 ? gd : nq;
    for (int j = tid; j < p; j += NT) {
      float s = 0.f;
      for (int a = 0; a < p; ++a) s += Ts[a * p + j];
      dst[j] = s;
    }
    __syncthreads();
    if (pass == 0) {
      for (int idx = tid; idx < pp; idx += NT) {
        const int a = idx / p, b = idx - a * p;
        Ts[idx] = Mg[a * ldc + b];
      }
      __syncthreads();
    }
  }
  for (int j = tid; j < p; j += NT) {
    const float lj = lamv[j];
    int rk = 0;
    for (int b = 0; b < p; ++b) {
      const float lb = lamv[b];
      rk += (lb > lj || (lb == lj && b < j)) ? 1 : 0;
    }
    rank[j] = rk;
  }
  if (tid == 0) {
    float mx = 0.f;
    for (int j = 0; j < p; ++j) mx = fmaxf(mx, gd[j]);
    red[0] = mx;
  }
  __syncthreads();
  const float gthr = red[0] * 1e-10f;
  for (int j = tid; j < p; j += NT) {
    const int rk = rank[j];
    lam_out[rk] = lamv[j];
    cs_out[rk] = (gd[j] > gthr && gd[j] > 0.f) ? rsqrtf(gd[j]) : 0.f;
    qs_out[rk] = (nq[j] > 1e-30f && isfinite(nq[j])) ? rsqrtf(nq[j]) : 1.f;
  }
  for (int idx = tid; idx < pp; idx += NT) {
    const int a = idx / p, j = idx - a * p;
    Wout[a * p + rank[j]] = Wm[idx];
  }
  stamp(8);
}

template <int NT>
__global__ __launch_bounds__(NT) void rr_small_kernel(const float* __restrict__ Cg, int p,
                                                      float* __restrict__ Wout,
                                                      float* __restrict__ lam_out,
                                                      float* __restrict__ cs_out,
                                                      float* __restrict__ qs_out,
                                                      int* __restrict__ info, int max_jsweeps,
                                                      float jrel) {
  rr_small_body<NT>(Cg, p, Wout, lam_out, cs_out, qs_out, info, max_jsweeps, jrel);
}

template <int NT>
__global__ __launch_bounds__(NT) void rr_small2_kernel(const float* __restrict__ Cg, int p,
                                                       float* __restrict__ Wout,
                                                       float* __restrict__ lam_out,
                                                       float* __restrict__ cs_out,
                                                       float* __restrict__ qs_out,
                                                       int* __restrict__ info, int max_jsweeps,
                                                       float jrel) {
  rr_small2_body<NT>(Cg, p, Wout, lam_out, cs_out, qs_out, info, max_jsweeps, jrel);
}

// Up to kRRBatch independent small solves in one launch, one workgroup each (the
// batched worker solves: W problems' Rayleigh-Ritz steps side by side on W CUs).
struct RRBatchArgs {
  const float* C[kRRBatch];
  float* W[kRRBatch];
  float* lam[kRRBatch];
  float* cs[kRRBatch];
  float* qs[kRRBatch];
  int* info[kRRBatch];
  int max_jsweeps[kRRBatch];
};

template <int NT>
__global__ __launch_bounds__(NT) void rr_small_batch_kernel(RRBatchArgs a, int p, float jrel) {
  const int i = blockIdx.x;
  rr_small_body<NT>(a.C[i], p, a.W[i], a.lam[i], a.cs[i], a.qs[i], a.info[i], a.max_jsweeps[i], jrel);
}

template <int NT>
__global__ __launch_bounds__(NT) void rr_small2_batch_kernel(RRBatchArgs a, int p, float jrel) {
  const int i = blockIdx.x;
  rr_small2_body<NT>(a.C[i], p, a.W[i], a.lam[i], a.cs[i], a.qs[i], a.info[i], a.max_jsweeps[i], jrel);
}

// blockIdx.y: the problem of a batched launch (its buffers at pbt.off, V = pbt.V).
__global__ __launch_bounds__(256) void rr_update_kernel(float* __restrict__ Z, int64_t d, int p,
                                                        int k, const float* __restrict__ W,
                                                        const float* __restrict__ lam,
                                                        const float* __restrict__ cs,
                                                        const float* __restrict__ qs, int64_t ldv,
                                                        float* __restrict__ resid_part,
                                                        const ProbBatch pbt) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int prob = blockIdx.y;
  float* __restrict__ V = pbt.V[prob];
  if (prob) {
    const int64_t o = pbt.off[prob];
    Z = reinterpret_cast<float*>(reinterpret_cast<char*>(Z) + o);
    W = reinterpret_cast<const float*>(reinterpret_cast<const char*>(W) + o);
    lam = reinterpret_cast<const float*>(reinterpret_cast<const char*>(lam) + o);
    cs = reinterpret_cast<const float*>(reinterpret_cast<const char*>(cs) + o);
    qs = reinterpret_cast<const float*>(reinterpret_cast<const char*>(qs) + o);
    resid_part = reinterpret_cast<float*>(reinterpret_cast<char*>(resid_part) + o);
  }
  float* Ws = sm;                  // p x p
  float* Zs = sm + p * p;          // UR x 2p
  float* rp = Zs + UR * 2 * p;     // ngrp x k partial residuals
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * UR;
  const int ld = 2 * p;
  const int ngrp = 256 / p;        // row groups (p <= 128 -> >= 2)
  for (int idx = tid; idx < p * p; idx += 256) Ws[idx] = W[idx];
  for (int idx = tid; idx < UR * ld; idx += 256) {
    const int rr = idx / ld, c = idx - rr * ld;
    const int64_t row = r0 + rr;
    Zs[idx] = (row < d) ? Z[row * ld + c] : 0.f;
  }
  __syncthreads();
  const int grp = tid / p, j = tid - grp * p;
  if (grp < ngrp) {
    const float lj = lam[j], cj = cs[j], qj = qs[j];
    float racc = 0.f;
    for (int rr = grp; rr < UR; rr += ngrp) {
      const int64_t row = r0 + rr;
      if (row >= d) break;
      const float* zq = Zs + rr * ld;
      const float* zy = zq + p;
      float qw = 0.f, yw = 0.f;
      for (int a = 0; a < p; ++a) {
        const float w = Ws[a * p + j];
        qw = fmaf(zq[a], w, qw);
        yw = fmaf(zy[a], w, yw);
      }
      qw *= qj;  // unit Ritz vector (qs = 1 / ||Q w_j||)
      yw *= qj;
      if (j < k) {
        const float e = yw - lj * qw;
        racc = fmaf(e, e, racc);
        V[row + (int64_t)(k - 1 - j) * ldv] = qw;
      }
      Z[row * ld + j] = (cj > 0.f) ? yw * (cj / qj) : qw;
    }
    if (j < k) rp[grp * k + j] = racc;
  }
  __syncthreads();
  for (int jj = tid; jj < k; jj += 256) {
    float s = 0.f;
    for (int g = 0; g < ngrp; ++g) s += rp[g * k + jj];
    resid_part[(int64_t)blockIdx.x * k + jj] = s;
  }
}

// r04: the same update on fp32 MFMA (v_mfma_f32_16x16x4_f32: fp32 products and
// sums, as the VALU form).  64 rows per block, wave w owns rows 16 w .. 16 w + 15 and
// every 16-column tile of both products (Zq = Q W, Zy = Y W: 2 p / 16 accumulator
// tiles).  Z's rows and W are staged in LDS (Z rows padded to 2 p + 1: the A reads,
// lane l -> row l & 15, k = l >> 4, hit 16 distinct banks); the epilogue is the VALU
// form's per element, the residual partials summed over lanes, then waves, in order.
// (The VALU form reloads W - 64 KB at p = 128 - per 32 rows and reads LDS twice per
// FMA pair: 575 us per 8-problem launch at d = 16384, p = 128, c5's timeline.)
constexpr int URM = 64;

template <int NC>  // NC = p / 16
__global__ __launch_bounds__(256) void rr_update_mfma_kernel(float* __restrict__ Z, int64_t d, int k,
                                                             const float* __restrict__ W,
                                                             const float* __restrict__ lam,
                                                             const float* __restrict__ cs,
                                                             const float* __restrict__ qs, int64_t ldv,
                                                             float* __restrict__ resid_part,
                                                             const ProbBatch pbt) {
  constexpr int P = 16 * NC, LD = 2 * P, LZ = 2 * P + 1;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ws = sm;               // P x P
  float* Zs = sm + P * P;       // URM x LZ
  float* rp = Zs + URM * LZ;    // 4 waves x P
  const int prob = blockIdx.y;
  float* __restrict__ V = pbt.V[prob];
  if (prob) {
    const int64_t o = pbt.off[prob];
    Z = reinterpret_cast<float*>(reinterpret_cast<char*>(Z) + o);
    W = reinterpret_cast<const float*>(reinterpret_cast<const char*>(W) + o);
    lam = reinterpret_cast<const float*>(reinterpret_cast<const char*>(lam) + o);
    cs = reinterpret_cast<const float*>(reinterpret_cast<const char*>(cs) + o);
    qs = reinterpret_cast<const float*>(reinterpret_cast<const char*>(qs) + o);
    resid_part = reinterpret_cast<float*>(reinterpret_cast<char*>(resid_part) + o);
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * URM;
  for (int idx = tid; idx < P * P / 4; idx += 256)
    *reinterpret_cast<f32x4*>(Ws + 4 * idx) = *reinterpret_cast<const f32x4*>(W + 4 * idx);
  for (int idx = tid; idx < URM * LD / 4; idx += 256) {  // 16-B loads, padded rows
    const int rr = idx / (LD / 4), c = 4 * (idx - rr * (LD / 4));
    const int64_t row = r0 + rr;
    const f32x4 v = *reinterpret_cast<const f32x4*>(Z + (row < d ? row : d - 1) * LD + c);
    const float m = row < d ? 1.f : 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) Zs[rr * LZ + c + e] = v[e] * m;
  }
  __syncthreads();
  f32x4 aq[NC], ay[NC];
#pragma unroll
  for (int ct = 0; ct < NC; ++ct) aq[ct] = ay[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* zrow = Zs + (16 * w + (lane & 15)) * LZ + (lane >> 4);
#pragma unroll 4
  for (int k0 = 0; k0 < P; k0 += 4) {
    const float a_q = zrow[k0], a_y = zrow[P + k0];
    const float* wrow = Ws + (k0 + (lane >> 4)) * P + (lane & 15);
#pragma unroll
    for (int ct = 0; ct < NC; ++ct) {
      const float b = wrow[16 * ct];
      aq[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_q, b, aq[ct], 0, 0, 0);
      ay[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_y, b, ay[ct], 0, 0, 0);
    }
  }
  // C map: row 4 (lane >> 4) + i, column lane & 15
#pragma unroll
  for (int ct = 0; ct < NC; ++ct) {
    const int j = 16 * ct + (lane & 15);
    const float lj = lam[j], cj = cs[j], qj = qs[j];
    float racc = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * (lane >> 4) + i;
      if (row < d) {
        const float qw = aq[ct][i] * qj, yw = ay[ct][i] * qj;
        if (j < k) {
          const float e = yw - lj * qw;
          racc = fmaf(e, e, racc);
          V[row + (int64_t)(k - 1 - j) * ldv] = qw;
        }
        Z[row * LD + j] = (cj > 0.f) ? yw * (cj / qj) : qw;
      }
    }
    racc += __shfl_xor(racc, 16, 64);
    racc += __shfl_xor(racc, 32, 64);
    if (lane < 16) rp[w * P + j] = racc;
  }
  __syncthreads();
  for (int jj = tid; jj < k; jj += 256)
    resid_part[(int64_t)blockIdx.x * k + jj] = ((rp[jj] + rp[P + jj]) + rp[2 * P + jj]) + rp[3 * P + jj];
}

// One wave per top-k column: lanes stride over the update blocks, shuffle-reduce
// (fixed order, deterministic).
__global__ __launch_bounds__(256) void rr_finish_kernel(const float* __restrict__ resid_part,
                                                        int nblk, int k,
                                                        const float* __restrict__ lam,
                                                        float* __restrict__ resid,
                                                        const ProbBatch pbt) {
  __shared__ float mx[4];
  const int prob = blockIdx.x;
  float* __restrict__ evals = pbt.evals[prob];
  if (prob) {
    const int64_t o = pbt.off[prob];
    resid_part = reinterpret_cast<const float*>(reinterpret_cast<const char*>(resid_part) + o);
    lam = reinterpret_cast<const float*>(reinterpret_cast<const char*>(lam) + o);
    resid = reinterpret_cast<float*>(reinterpret_cast<char*>(resid) + o);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float scale = fmaxf(fabsf(lam[0]), 1e-30f);
  float m = 0.f;
  for (int j = wave; j < k; j += 4) {
    float s = 0.f;
    for (int b = lane; b < nblk; b += 64) s += resid_part[(int64_t)b * k + j];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float rel = sqrtf(s) / scale;
    if (lane == 0) {
      resid[j] = rel;
      evals[k - 1 - j] = lam[j];
    }
    m = (rel == rel) ? fmaxf(m, rel) : rel;  // NaN propagates (fmaxf would drop it)
  }
  if (lane == 0) mx[wave] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = mx[0];
    for (int w = 1; w < 4; ++w) r = (r == r && mx[w] == mx[w]) ? fmaxf(r, mx[w]) : __int_as_float(0x7fc00000);
    resid[k] = r;
  }
}

// Power step between two Rayleigh-Ritz sweeps: Q_j <- Y_j * cs_j for the live
// Ritz columns of the last RR (cs_j = 1 / ||Y w_j||, so the columns stay ~unit
// norm) whose Ritz value satisfies |lambda_j| >= tau |lambda_0|.  Dead columns
// (cs_j == 0: null directions of a rank-deficient operator) keep Q_j, as
// rr_update treats them, and so do weak columns: every extra power step
// multiplies a column's contamination by the dominant directions by up to
// |lambda_0 / lambda_j| before the next RR re-orthogonalises, so the driver
// picks tau = 0.1^(1 / steps between RRs) and the growth stays <= 10x (a wide
// spectrum - the projector average: 1 vs << 1 - would otherwise make the
// basis numerically dependent).
__global__ __launch_bounds__(256) void rr_power_kernel(float* __restrict__ Z, int64_t d, int p,
                                                       const float* __restrict__ cs,
                                                       const float* __restrict__ lam, float tau) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * p) return;
  const int64_t r = idx / p;
  const int j = (int)(idx - r * p);
  const float c = cs[j];
  if (c > 0.f && fabsf(lam[j]) >= tau * fabsf(lam[0])) Z[r * 2 * p + j] = Z[r * 2 * p + p + j] * c;
}

// One degree of the scaled Chebyshev filter between two Rayleigh-Ritz steps
// (Zhou & Saad's scaled three-term recurrence; capi.hip plans alpha / cc / gamma
// from the last RR's Ritz values).  Z = [X_j | A X_j] (ld 2p), T = X_{j-1} (ld p):
//   X_{j+1} = alpha (A X_j - cc X_j) - gamma X_{j-1};  T <- X_j;  Z_q <- X_{j+1}
// for the active columns (Ritz value >= thr); the others keep X_0 (like the weak
// columns of rr_power_kernel: their contamination by the dominant directions
// would grow past what the fp32 Gram resolves).  A column's recurrence is linear
// in that column only, so per-column activation keeps every column a polynomial
// in A of its start vector.  float4 over columns (p % 16 == 0).
__global__ __launch_bounds__(256) void cheb_step_kernel(float* __restrict__ Z,
                                                        float* __restrict__ T, int64_t d,
                                                        int p, const float* __restrict__ lam,
                                                        float thr, float alpha, float cc,
                                                        float gamma) {
  const int pq = p >> 2;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * pq) return;
  const int64_t r = idx / pq;
  const int j = (int)(idx - r * pq) * 4;
  f32x4* zq = reinterpret_cast<f32x4*>(Z + r * 2 * p + j);
  const f32x4 y = *reinterpret_cast<const f32x4*>(Z + r * 2 * p + p + j);
  f32x4* tp = reinterpret_cast<f32x4*>(T + r * p + j);
  const f32x4 q = *zq;
  // degree 1 (gamma == 0) must not read T: it is uninitialised workspace then
  // (0 * NaN garbage would poison the column)
  const f32x4 t = gamma != 0.f ? *tp : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 xn = q;
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (lam[j + u] >= thr) xn[u] = alpha * (y[u] - cc * q[u]) - gamma * t[u];
  *tp = q;
  *zq = xn;
}

// After a deflated stage or block (capi.hip): V_j <- normalize(V_j - V_D V_D^T V_j)
// for the kc columns of the stage against the r locked ones (V_D = columns kc ..
// kc + r - 1).  The deflated operator S - lam_1 v^ v^T keeps a coupling
// lam_1 (v_1 d^T + d v_1^T) from the small error d = v^ - v_1, which tilts each
// remaining eigenvector towards v_1 by lam_1 d_j / lam_j; the span of [V, V_D] is
// right, and projecting v^ out is exact to O(lam_1 |d|^2).  One block per column;
// V_D in chunks of 8 columns (modified Gram-Schmidt by chunk, twice when r > 8:
// block locking of k > 128 pairs); fixed-order block reductions.
// (block_mgs: the same kernel with Vd = the block's own earlier columns, one column
// per launch - see deflate_orth_launch.)
__global__ __launch_bounds__(256) void deflate_orth_kernel(float* __restrict__ V,
                                                           const float* __restrict__ Vd,
                                                           int64_t ldv, int64_t d, int r,
                                                           int passes) {
  __shared__ float red[4][8];
  __shared__ float coef[8];
  const int j = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float* v = V + (int64_t)j * ldv;
  const float* vd0 = Vd;
  for (int pass = 0; pass < passes; ++pass)
    for (int q0 = 0; q0 < r; q0 += 8) {
      const int nq = r - q0 < 8 ? r - q0 : 8;
      const float* vd = vd0 + (int64_t)q0 * ldv;
      float dot[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) dot[q] = 0.f;
      for (int64_t i = tid; i < d; i += 256) {
        const float x = v[i];
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (q < nq) dot[q] = fmaf(vd[(int64_t)q * ldv + i], x, dot[q]);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float t = dot[q];
        for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
        if (lane == 0) red[w][q] = t;
      }
      __syncthreads();
      if (tid < 8) coef[tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
      __syncthreads();
      for (int64_t i = tid; i < d; i += 256) {
        float x = v[i];
        for (int q = 0; q < nq; ++q) x = fmaf(-coef[q], vd[(int64_t)q * ldv + i], x);
        v[i] = x;
      }
      __syncthreads();  // red / coef are reused by the next chunk
    }
  float nrm = 0.f;
  for (int64_t i = tid; i < d; i += 256) nrm = fmaf(v[i], v[i], nrm);
  for (int o = 32; o > 0; o >>= 1) nrm += __shfl_xor(nrm, o, 64);
  if (lane == 0) red[w][0] = nrm;
  __syncthreads();
  const float sc = rsqrtf(red[0][0] + red[1][0] + red[2][0] + red[3][0]);
  for (int64_t i = tid; i < d; i += 256) v[i] *= sc;
}

// evals[j] -= shift (the solver's indefinite-input shift, undone at the end).
__global__ void unshift_kernel(float* __restrict__ evals, int k, double shift) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < k) evals[j] = (float)((double)evals[j] - shift);
}

// Final eigenvalues as Rayleigh quotients in DOUBLE: lam_j = v_j^T S v_j / v_j^T v_j
// from the explicit S (float or double, row-major lds) and the returned vectors.
// The fp32 Rayleigh-Ritz values carry ~1e-7 of the operator's scale (a few ulps of
// |H| in the small solve); a quotient of a vector with sin(angle) ~ 1e-6 is exact to
// ~1e-12 of the spread, and it is taken on S itself - unshifted, undeflated.
// Products s * v of fp32 values are exact in double; sums are in double, in a fixed
// order (deterministic).
//   rq_vd_kernel:   Vd[r][j] = v_j[r] as double (zero for k <= j < kpad = 16 ng);
//   rq_part_kernel: block (cb, rb) = 512 columns x RQ_RB rows; lane c of wave w owns
//                   columns c0 + 128 w + c + 64 u (u < 2, coalesced row reads of S, all
//                   issued before the first FMA, kept in registers for every group).
//                   Per group g of RQ_KG = 16 vectors: the block's Vd rows of the group
//                   go to LDS, acc[u][jj] = sum_r S[r][c_u] Vd[r][16 g + jj] (each row's
//                   16 values, 8 broadcast ds_read_b128, feed 32 FMAs), then t_jj =
//                   sum_u acc[u][jj] v_{16g+jj}[c_u] is summed over the block
//                   (an LDS transpose per wave, the 4 waves in order) into
//                   part[block][16 g + jj];
//   rq_finish_kernel: block j sums the parts in block order and v_j^T v_j.
// One read of the lower block triangle of S, ~d^2 / 2 x kpad fp64 FMA (symmetry: the
// blocks left of a row block's diagonal panel count twice).  (Earlier versions: 32 rows x all
// columns per block staged through LDS, 387 us at d = 3072, k = 10 - 3.1 ms of c1's
// 11.1 ms step, profiles/r03s; one column per lane with the Vd row as scalar loads,
// 166 us: every row waited on a scalar-cache miss, profiles/r03t.)
constexpr int RQ_KG = 16;   // vectors per pass
constexpr int RQ_CPT = 2;   // columns per lane
constexpr int RQ_RB = 8;    // rows per block (16: the register budget serialised the loads)
constexpr int RQ_CB = 4 * 64 * RQ_CPT;  // columns per block

__global__ __launch_bounds__(256) void rq_vd_kernel(const float* __restrict__ V, int64_t ldv,
                                                    int64_t d, int k, int kpad,
                                                    double* __restrict__ Vd) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * kpad) return;
  const int64_t r = idx / kpad;
  const int j = (int)(idx - r * kpad);
  Vd[idx] = j < k ? (double)V[(int64_t)j * ldv + r] : 0.0;
}

template <typename T>
__global__ __launch_bounds__(256) void rq_part_kernel(const T* __restrict__ S, int64_t lds, int64_t d,
                                                      const double* __restrict__ Vd,
                                                      const float* __restrict__ V, int64_t ldv,
                                                      int k, int ng, double* __restrict__ part) {
  constexpr int KG = RQ_KG;
  const int kpad = KG * ng;
  __shared__ __attribute__((aligned(16))) double vs[RQ_RB][KG];
  __shared__ double red[4][KG];
  __shared__ double tw[4][KG][65];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = (int64_t)blockIdx.y * RQ_RB;
  // S symmetric: only blocks on or below the diagonal panel run (RQ_RB | RQ_CB, so a
  // row block lies in one column panel); those left of it count twice (exact x2),
  // the diagonal panel's once.  Skipped blocks write zero parts.
  const int panel = (int)(r0 / RQ_CB);
  if ((int)blockIdx.x > panel) {
    for (int j = tid; j < KG * ng; j += 256)
      part[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * (KG * ng) + j] = 0.0;
    return;
  }
  const double wgt = (int)blockIdx.x < panel ? 2.0 : 1.0;
  const int64_t cw = (int64_t)blockIdx.x * RQ_CB + 64 * RQ_CPT * wave + lane;
  // unpredicated, unselected loads at clamped in-range addresses: rows past d meet
  // zero Vd rows in LDS and columns past d zero epilogue factors, so no condition
  // touches a loaded value (a uniform row test became a branch per load with a
  // vmcnt(0) behind each: 32 serialised load latencies per block, 106 us at c1)
  T sv[RQ_RB][RQ_CPT];
#pragma unroll
  for (int r = 0; r < RQ_RB; ++r)
#pragma unroll
    for (int u = 0; u < RQ_CPT; ++u) {
      const int64_t c = cw + 64 * u;
      const int64_t rr = r0 + r < d ? r0 + r : d - 1;
      sv[r][u] = S[rr * lds + (c < d ? c : d - 1)];
    }
  for (int g = 0; g < ng; ++g) {
  const int j0 = KG * g;
  if (g) __syncthreads();  // the last group's vs / red reads are done
  // (no condition selects a loaded value anywhere below: the compiler turns such a
  // select into a branch around the load with a vmcnt(0) behind it - masks multiply)
  if (tid < RQ_RB * KG) {
    const int rr = tid / KG;
    const int64_t row = r0 + rr < d ? r0 + rr : d - 1;
    vs[rr][tid - rr * KG] = Vd[row * kpad + j0 + (tid - rr * KG)] * (r0 + rr < d ? 1.0 : 0.0);
  }
  // this group's epilogue factors v_j[c_u], loaded before the FMAs (latency hidden)
  // (raw values: the column / vector masks are applied in the epilogue, so nothing
  // consumes a load before the FMAs)
  float vpre[RQ_CPT][KG];
#pragma unroll
  for (int u = 0; u < RQ_CPT; ++u) {
    const int64_t c = cw + 64 * u;
    const float* vc = V + (c < d ? c : d - 1);
#pragma unroll
    for (int jj = 0; jj < KG; ++jj) {
      const int j = j0 + jj;
      vpre[u][jj] = vc[(int64_t)(j < k ? j : k - 1) * ldv];
    }
  }
  __syncthreads();
  double acc[RQ_CPT][KG];
#pragma unroll
  for (int u = 0; u < RQ_CPT; ++u)
#pragma unroll
    for (int jj = 0; jj < KG; ++jj) acc[u][jj] = 0.0;
#pragma unroll
  for (int r = 0; r < RQ_RB; ++r) {
    double vv[KG];
#pragma unroll
    for (int jj = 0; jj < KG; jj += 2) {
      const f64x2 w = *reinterpret_cast<const f64x2*>(&vs[r][jj]);
      vv[jj] = w[0];
      vv[jj + 1] = w[1];
    }
#pragma unroll
    for (int u = 0; u < RQ_CPT; ++u) {
      const double sd = (double)sv[r][u];
#pragma unroll
      for (int jj = 0; jj < KG; ++jj) acc[u][jj] = fma(sd, vv[jj], acc[u][jj]);
    }
  }
  double t[KG];
#pragma unroll
  for (int jj = 0; jj < KG; ++jj) t[jj] = 0.0;
#pragma unroll
  for (int u = 0; u < RQ_CPT; ++u) {
    const double cm = cw + 64 * u < d ? 1.0 : 0.0;
#pragma unroll
    for (int jj = 0; jj < KG; ++jj)
      t[jj] = fma(acc[u][jj], (double)vpre[u][jj] * (j0 + jj < k ? cm : 0.0), t[jj]);
  }
  // wave sums of the 16 t_jj through this wave's LDS transpose: lane l (vector
  // l >> 2, quarter q = l & 3) adds lanes q, q + 4, ... of it, then 2 shuffles.
  // (Register butterflies with per-lane selects compiled to ~1600 VALU ops per
  // group - 6x the group's FMAs, profiles/r03x.)  The wave reads only what it wrote:
  // its LDS operations complete in order, the wave barrier keeps the compiler's.
#pragma unroll
  for (int jj = 0; jj < KG; ++jj) tw[wave][jj][lane] = t[jj];
  __builtin_amdgcn_wave_barrier();
  const int jr = lane >> 2, q = lane & 3;
  double sum = 0.0;
#pragma unroll
  for (int i = 0; i < 16; ++i) sum += tw[wave][jr][q + 4 * i];
  sum += __shfl_xor(sum, 1, 64);
  sum += __shfl_xor(sum, 2, 64);
  t[0] = sum;
  __builtin_amdgcn_wave_barrier();  // (the next group's writes stay behind these reads)
  if ((lane & 3) == 0) red[wave][lane >> 2] = t[0];
  __syncthreads();
  if (tid < KG)
    part[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * kpad + j0 + tid] =
        wgt * (((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid]);
  }  // groups
}

// r04: the quotients' products on f64 MFMA (v_mfma_f64_16x16x4_f64; fp32 S with
// d % 4 == 0, lds % 4 == 0 and 16-B alignment - other inputs keep rq_part_kernel).
// Persistent: 256 workgroups walk the lower 128 x 128 tiles of S (tile t -> row block
// rb, column block cb <= rb).  Per tile W = S_tile V_cb (128 x kpad, on MFMA: wave w
// owns rows 16 w .., all kpad / 16 vector tiles) and t_j += wgt sum_r V_rb[r][j] W[r][j]
// (wgt 2 below the diagonal, 1 on it).  A operands straight from HBM: lane l loads
// S[16 w + (l & 15)][16 q + 4 (l >> 4) .. + 3] and MFMA step (q, e) sums over the
// columns 16 q + 4 g + e (g = l >> 4) - the k order is free as long as B follows it:
// V_cb is staged in LDS as [vector][column] fp32 (row stride 132: conflict-free
// 16-B reads) and lane l reads [16 nt + (l & 15)][16 q + 4 g ..].  Products of fp32
// values are exact in double; sums in double, in a fixed order (deterministic).
constexpr int RQM_T = 128, RQM_LDS = 132, RQM_G = 256;
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int NT>
__global__ __launch_bounds__(512) void rq_mfma_kernel(const float* __restrict__ S, int64_t lds, int64_t d,
                                                      const float* __restrict__ V, int64_t ldv, int k,
                                                      double* __restrict__ part) {
  constexpr int KP = 16 * NT;  // kpad
  __shared__ __attribute__((aligned(16))) float vc[KP][RQM_LDS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c16 = lane & 15;
  const int64_t nbk = cdiv(d, RQM_T);
  const int64_t ntiles = nbk * (nbk + 1) / 2;
  double tsum[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) tsum[nt] = 0.0;
  for (int64_t ti = blockIdx.x; ti < ntiles; ti += gridDim.x) {
    int64_t rb = (int64_t)((sqrt(8.0 * (double)ti + 1.0) - 1.0) * 0.5);
    while (rb * (rb + 1) / 2 > ti) --rb;
    while ((rb + 1) * (rb + 2) / 2 <= ti) ++rb;
    const int64_t cb = ti - rb * (rb + 1) / 2;
    const int64_t r0 = rb * RQM_T, c0 = cb * RQM_T;
    const double wgt = rb > cb ? 2.0 : 1.0;
    // this wave's A strip: 16 rows x 128 columns, one 16-column group ahead (clamped
    // in range: rows past d meet zero V_rb values below, columns past d zero V_cb rows)
    const int64_t row = r0 + 16 * w + c16;
    const float* srow = S + (row < d ? row : d - 1) * lds;
    auto load_a = [&](int q) {
      const int64_t c = c0 + 16 * q + 4 * g;
      return *reinterpret_cast<const f32x4*>(srow + (c < d ? c : d - 4));
    };
    f32x4 xn = load_a(0);
    __syncthreads();  // the previous tile's vc reads are done
    // V_cb -> LDS as [vector j][column]: zero for j >= k or columns past d
    for (int u = tid; u < KP * (RQM_T / 4); u += 512) {
      const int j = u / (RQM_T / 4), c4 = 4 * (u % (RQM_T / 4));
      const int64_t c = c0 + c4;
      f32x4 v = *reinterpret_cast<const f32x4*>(V + (int64_t)(j < k ? j : k - 1) * ldv + (c < d ? c : d - 4));
      const float m = (j < k && c < d) ? 1.f : 0.f;
      *reinterpret_cast<f32x4*>(&vc[j][c4]) = v * m;
    }
    __syncthreads();
    f64x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f64x4{0.0, 0.0, 0.0, 0.0};
    constexpr int NG = NT < 4 ? NT : 4;  // vector tiles per B batch (independent accumulators)
#pragma unroll 1
    for (int q = 0; q < 8; ++q) {
      const f32x4 xq = xn;
      if (q < 7) xn = load_a(q + 1);  // one column group ahead
      double a[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] = (double)xq[e];
#pragma unroll
      for (int n0 = 0; n0 < NT; n0 += NG) {
        f32x4 bv[NG];
#pragma unroll
        for (int u = 0; u < NG && n0 + u < NT; ++u)
          bv[u] = *reinterpret_cast<const f32x4*>(&vc[16 * (n0 + u) + c16][16 * q + 4 * g]);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int u = 0; u < NG && n0 + u < NT; ++u)
            acc[n0 + u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[e], (double)bv[u][e], acc[n0 + u], 0, 0, 0);
      }
    }
    // epilogue: lane l holds W[16 w + g + 4 i][16 nt + c16] (f64 C/D map), i < 4
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int j = 16 * nt + c16;
      const float* vj = V + (int64_t)(j < k ? j : k - 1) * ldv;
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t r = r0 + 16 * w + g + 4 * i;
        const double vr = (double)vj[r < d ? r : d - 1] * ((r < d && j < k) ? 1.0 : 0.0);
        t = fma(vr, acc[nt][i], t);
      }
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      tsum[nt] = fma(wgt, t, tsum[nt]);
    }
  }
  // the 8 waves' sums in wave order -> part[block][j]
  __shared__ double red[8][KP];
  if (g == 0)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) red[w][16 * nt + c16] = tsum[nt];
  __syncthreads();
  if (tid < KP) {
    double s = 0.0;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) s += red[ww][tid];
    part[(int64_t)blockIdx.x * KP + tid] = s;
  }
}

// block j: q = sum over the nblk parts (thread-strided, then a fixed LDS tree),
// n = v^T v the same way; evals[j] = q / n.
__global__ __launch_bounds__(256) void rq_finish_kernel(const double* __restrict__ part, int64_t nblk,
                                                        int kpad, const float* __restrict__ V,
                                                        int64_t ldv, int64_t d,
                                                        float* __restrict__ evals) {
  __shared__ double rq[256], rn[256];
  const int tid = threadIdx.x, j = blockIdx.x;
  double q = 0.0, nn = 0.0;
  for (int64_t b = tid; b < nblk; b += 256) q += part[b * kpad + j];
  const float* v = V + (int64_t)j * ldv;
  for (int64_t r = tid; r < d; r += 256) {
    const double x = (double)v[r];
    nn = fma(x, x, nn);
  }
  rq[tid] = q;
  rn[tid] = nn;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (tid < w) {
      rq[tid] += rq[tid + w];
      rn[tid] += rn[tid + w];
    }
    __syncthreads();
  }
  if (tid == 0 && rn[0] > 0.0) evals[j] = (float)(rq[0] / rn[0]);
}

size_t rr_small_shm(int p) {
  return (size_t)(2 * p * p + 7 * p + RT / 64 + 20) * sizeof(float);
}

#ifdef DEIG_AB_RR_THREADS
constexpr int RT2 = DEIG_AB_RR_THREADS;  // measurement builds
#else
constexpr int RT2 = 1024;  // rr_small2 (the Jacobi's per-step work wants every thread)
#endif
size_t rr_small2_shm(int p) {
  return (size_t)(2 * p * p + 9 * p + 16 * 17 + 4 + 16 * (p + 4) + RT2 / 64 + 2 + 4) * sizeof(float);
}

}  // namespace

int rr_init_launch(float* Z, int64_t d, int p, const float* Q0, int k0, int64_t ldq0,
                   uint64_t seed, hipStream_t stream, int64_t valid) {
  const int64_t tot = d * p;
  hipLaunchKernelGGL(rr_init_kernel, dim3((unsigned)cdiv(tot, 256)), dim3(256), 0, stream, Z, d,
                     p, Q0, k0, ldq0, seed, valid < 0 ? d : valid);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

int rr_small_launch(const RRBuffers& b, int p, hipStream_t stream, int max_jsweeps, float jrel) {
  DEIG_REQUIRE(p >= 16 && p <= 128 && p % 16 == 0, "rr_small: p=%d out of range", p);
#ifndef DEIG_AB_RR_V1
  static const hipError_t attr2 = hipFuncSetAttribute(
      (const void*)rr_small2_kernel<RT2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)rr_small2_shm(128));
  DEIG_HIP_CHECK(attr2);
  hipLaunchKernelGGL(rr_small2_kernel<RT2>, dim3(1), dim3(RT2), rr_small2_shm(p), stream, b.C, p, b.W, b.lam,
                     b.cs, b.qs, b.info, max_jsweeps, jrel);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
#endif
  const size_t shm = rr_small_shm(p);
  // once per process (C++11 thread-safe static initialisation)
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)rr_small_kernel<RT>, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)rr_small_shm(128));
  DEIG_HIP_CHECK(attr);
  // Workgroup size: 1024 threads at every p.  Each Jacobi step is a chain of LDS
  // round trips per thread, so the most threads (shortest per-thread chain) win:
  // measured r02 at p = 32, Jacobi 75 us (1024) vs 89 (256) vs 184 (64) per RR.
  hipLaunchKernelGGL(rr_small_kernel<RT>, dim3(1), dim3(RT), shm, stream, b.C, p, b.W, b.lam, b.cs,
                     b.qs, b.info, max_jsweeps, jrel);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

int rr_small_batch_launch(const RRBuffers* const* bs, const int* max_jsweeps, int n, int p,
                          hipStream_t stream, float jrel) {
  DEIG_REQUIRE(p >= 16 && p <= 128 && p % 16 == 0, "rr_small: p=%d out of range", p);
#ifndef DEIG_AB_RR_V1
  static const hipError_t attr2 = hipFuncSetAttribute(
      (const void*)rr_small2_batch_kernel<RT2>, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)rr_small2_shm(128));
  DEIG_HIP_CHECK(attr2);
#endif
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)rr_small_batch_kernel<RT>, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)rr_small_shm(128));
  DEIG_HIP_CHECK(attr);
  for (int i0 = 0; i0 < n; i0 += kRRBatch) {
    const int m = std::min(kRRBatch, n - i0);
    RRBatchArgs a{};
    for (int i = 0; i < m; ++i) {
      const RRBuffers& b = *bs[i0 + i];
      a.C[i] = b.C;
      a.W[i] = b.W;
      a.lam[i] = b.lam;
      a.cs[i] = b.cs;
      a.qs[i] = b.qs;
      a.info[i] = b.info;
      a.max_jsweeps[i] = max_jsweeps[i0 + i];
    }
#ifndef DEIG_AB_RR_V1
    hipLaunchKernelGGL(rr_small2_batch_kernel<RT2>, dim3(m), dim3(RT2), rr_small2_shm(p), stream, a, p, jrel);
#else
    hipLaunchKernelGGL(rr_small_batch_kernel<RT>, dim3(m), dim3(RT), rr_small_shm(p), stream, a, p, jrel);
#endif
    DEIG_HIP_CHECK(hipGetLastError());
  }
  return DEIG_OK;
}

int rr_power_launch(const RRBuffers& b, int64_t d, int p, float tau, hipStream_t stream) {
  hipLaunchKernelGGL(rr_power_kernel, dim3((unsigned)cdiv(d * p, 256)), dim3(256), 0, stream, b.Z,
                     d, p, b.cs, b.lam, tau);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

int cheb_step_launch(const RRBuffers& b, float* T, int64_t d, int p, float thr, float alpha,
                     float cc, float gamma, hipStream_t stream) {
  DEIG_REQUIRE(p % 16 == 0, "cheb_step: p=%d must be a multiple of 16", p);
  hipLaunchKernelGGL(cheb_step_kernel, dim3((unsigned)cdiv(d * (p / 4), 256)), dim3(256), 0,
                     stream, b.Z, T, d, p, b.lam, thr, alpha, cc, gamma);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

int deflate_orth_launch(float* V, int64_t ldv, int64_t d, int kc, int r, hipStream_t stream) {
  DEIG_REQUIRE(r >= 1 && kc >= 1, "deflate_orth: r=%d kc=%d out of range", r, kc);
  hipLaunchKernelGGL(deflate_orth_kernel, dim3(kc), dim3(256), 0, stream, V, V + (int64_t)kc * ldv,
                     ldv, d, r, r > 8 ? 2 : 1);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

int block_mgs_launch(float* V, int64_t ldv, int64_t d, int kc, hipStream_t stream) {
  DEIG_REQUIRE(kc >= 1, "block_mgs: kc=%d out of range", kc);
  // column j against columns 0 .. j-1 (already orthonormal), in order, projected
  // twice (a column that was mostly locked directions keeps a small remainder) and
  // normalised
  for (int j = 0; j < kc; ++j) {
    if (j == 0) {
      hipLaunchKernelGGL(deflate_orth_kernel, dim3(1), dim3(256), 0, stream, V, V, ldv, d, 0, 1);
    } else {
      hipLaunchKernelGGL(deflate_orth_kernel, dim3(1), dim3(256), 0, stream, V + (int64_t)j * ldv, V,
                         ldv, d, j, 2);
    }
    DEIG_HIP_CHECK(hipGetLastError());
  }
  return DEIG_OK;
}

size_t rq_workspace_bytes(int64_t d, int k) {
  // part[] holds one kpad-row per block of whichever kernel rq_launch picks: the VALU
  // form's grid (nblk) or the MFMA form's fixed RQM_G workgroups (more than nblk for
  // d below ~1020)
  const int64_t nblk = cdiv(d, RQ_CB) * cdiv(d, RQ_RB);
  const int64_t nprt = nblk > RQM_G ? nblk : (int64_t)RQM_G;
  return (size_t)(d + nprt) * cdiv(k, RQ_KG) * RQ_KG * sizeof(double);
}

int rq_launch(const void* S, int stype, int64_t d, int64_t lds, const float* V, int64_t ldv, int k,
              float* evals, void* ws, hipStream_t stream) {
  DEIG_REQUIRE(k >= 1 && k <= d, "rq: need 1 <= k <= d (k=%d)", k);
  const int ng = (int)cdiv(k, RQ_KG), kpad = RQ_KG * ng;
  double* Vd = static_cast<double*>(ws);
  double* part = Vd + d * kpad;
  const dim3 grid((unsigned)cdiv(d, RQ_CB), (unsigned)cdiv(d, RQ_RB));
  const int64_t nblk = (int64_t)grid.x * grid.y;
  const bool mfma = stype == DEIG_F32 && d % 4 == 0 && lds % 4 == 0 && ldv % 4 == 0 && aligned16(S) &&
                    aligned16(V) && d >= RQM_T && kpad <= 128;
  if (mfma) {
    const float* Sf = static_cast<const float*>(S);
    switch (ng) {
#define DEIG_RQM(x)                                                                                 \
  case x:                                                                                           \
    hipLaunchKernelGGL(rq_mfma_kernel<x>, dim3(RQM_G), dim3(512), 0, stream, Sf, lds, d, V, ldv, k, part); \
    break;
      DEIG_RQM(1) DEIG_RQM(2) DEIG_RQM(3) DEIG_RQM(4) DEIG_RQM(5) DEIG_RQM(6) DEIG_RQM(7) DEIG_RQM(8)
#undef DEIG_RQM
    }
  } else {
    hipLaunchKernelGGL(rq_vd_kernel, dim3((unsigned)cdiv(d * kpad, 256)), dim3(256), 0, stream, V, ldv,
                       d, k, kpad, Vd);
    DEIG_HIP_CHECK(hipGetLastError());
    if (stype == DEIG_F64)
      hipLaunchKernelGGL(rq_part_kernel<double>, grid, dim3(256), 0, stream,
                         static_cast<const double*>(S), lds, d, Vd, V, ldv, k, ng, part);
    else
      hipLaunchKernelGGL(rq_part_kernel<float>, grid, dim3(256), 0, stream,
                         static_cast<const float*>(S), lds, d, Vd, V, ldv, k, ng, part);
  }
  DEIG_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(rq_finish_kernel, dim3((unsigned)k), dim3(256), 0, stream, part,
                     mfma ? (int64_t)RQM_G : nblk, kpad, V, ldv, d, evals);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

int unshift_launch(float* evals, int k, double shift, hipStream_t stream) {
  hipLaunchKernelGGL(unshift_kernel, dim3((unsigned)cdiv(k, 256)), dim3(256), 0, stream, evals, k,
                     shift);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

int rr_update_blocks(int64_t d) { return (int)cdiv(d, UR); }

int rr_update_launch(const RRBuffers& b, int64_t d, int p, int k, float* V, int64_t ldv,
                     float* evals, hipStream_t stream) {
  ProbBatch one = one_problem();
  one.V[0] = V;
  one.evals[0] = evals;
  return rr_update_batch_launch(b, d, p, k, ldv, one, stream);
}

int rr_update_batch_launch(const RRBuffers& b, int64_t d, int p, int k, int64_t ldv,
                           const ProbBatch& pbt, hipStream_t stream) {
  const int nblk = rr_update_blocks(d);
  DEIG_REQUIRE(p >= 16 && p <= 128, "rr_update: p=%d out of range", p);
  DEIG_REQUIRE(pbt.n >= 1 && pbt.n <= kMaxProbBatch && pbt.off[0] == 0, "rr_update: batch of %d", pbt.n);
  // the MFMA form where its operands are 16-B aligned (p % 16 == 0 always holds)
  const bool mfma = aligned16(b.W) && aligned16(b.Z) && (pbt.n == 1 || pbt.off[1] % 16 == 0);
  const int nb = mfma ? (int)cdiv(d, URM) : nblk;
  if (mfma) {
    const size_t shm = (size_t)(p * p + URM * (2 * p + 1) + 4 * p) * sizeof(float);
    switch (p / 16) {
#define DEIG_RRU(x)                                                                                     \
  case x: {                                                                                           \
    static const hipError_t at = hipFuncSetAttribute((const void*)rr_update_mfma_kernel<x>,             \
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,        \
                                                     (int)((16 * x * 16 * x + URM * (32 * x + 1) + 64 * x) * sizeof(float))); \
    DEIG_HIP_CHECK(at);                                                                               \
    hipLaunchKernelGGL(rr_update_mfma_kernel<x>, dim3(nb, pbt.n), dim3(256), shm, stream, b.Z, d, k, b.W, \
                       b.lam, b.cs, b.qs, ldv, b.resid_part, pbt);                                    \
  } break;
      DEIG_RRU(1) DEIG_RRU(2) DEIG_RRU(3) DEIG_RRU(4) DEIG_RRU(5) DEIG_RRU(6) DEIG_RRU(7) DEIG_RRU(8)
#undef DEIG_RRU
    }
  } else {
    const size_t shm = (size_t)(p * p + UR * 2 * p + (256 / p) * k) * sizeof(float);
    static const hipError_t attr = hipFuncSetAttribute(
        (const void*)rr_update_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)((128 * 128 + UR * 256 + 16 * 128) * sizeof(float)));
    DEIG_HIP_CHECK(attr);
    hipLaunchKernelGGL(rr_update_kernel, dim3(nblk, pbt.n), dim3(256), shm, stream, b.Z, d, p, k, b.W,
                       b.lam, b.cs, b.qs, ldv, b.resid_part, pbt);
  }
  DEIG_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(rr_finish_kernel, dim3(pbt.n), dim3(256), 0, stream, b.resid_part, nb, k,
                     b.lam, b.resid, pbt);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

}  // namespace deig
