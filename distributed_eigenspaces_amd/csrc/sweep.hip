// Subspace-iteration sweep Y = alpha * S Q on bf16 MFMA with split fp32 operands.
//
// The S*Q product of every sweep of the eigensolver that replaces LAPACK dsyevr
// in Node.top_k_eigenvectors (distributed.py:22-29).  S (d x d fp32, symmetric,
// row-major) is streamed from HBM once per sweep and split in registers into
// three bf16 pieces x = h + m + l (|x - h - m - l| <= 2^-27 |x|); Q (d x p fp32)
// is split the same way once per sweep into an image in MFMA B-operand order
// (split_q_kernel).  Each product is formed from the six bf16 MFMA products
// h h + h m + m h + h l + l h + m m (every term down to 2^-16 |ab|), accumulated
// in fp32: the dropped terms are <= ~2^-23 |ab|, i.e. fp32-grade products.  Two
// pieces (the covariance kernel's split3) are not enough here: their ~2^-17
// representation error survives in the null-space images S q ~ 0 and the
// residual test of the solver, while the covariance averages it out over n.
// Six bf16 MFMAs cost 6/16 of one f32 MFMA, so the sweep stays under the HBM
// roof (4 d^2 bytes of S at 8 TB/s) instead of the f32-MFMA roof (2 d^2 p flop
// at 157 TF/s) for p <= 128.
//
// Y[m][:] = sum_k S[m][k] Q[k][:]  (S = S^T, so ROWS of S are read, contiguous
// along k).  v_mfma_f32_16x16x32_bf16: lane l holds A[m = l%16][k = 8(l/16)..+7]
// - 32 contiguous bytes of one row of S, loaded straight into registers, no LDS
// - and B[k = 8(l/16)..+7][n = l%16] from the Q image, staged through LDS once
// per block and K-step and shared by the 8 waves.  Block = 8 waves x 32 rows (2
// MFMA row blocks per wave, all p columns); K-step = 64 (2 MFMA k-groups) with
// register double buffering of the S rows and of the Q stage.  Split-K over
// gridDim.y; partial slabs are summed in slice order (deterministic).
#include <stdlib.h>

#include "deig_internal.hpp"

namespace deig {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int SW_THR = 512;   // 8 waves
constexpr int SW_ROWS = 256;  // rows per block: 8 waves x 2 x 16
constexpr int SW_KS = 64;     // k per stage

__device__ __forceinline__ uint32_t rne_bf16(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// 8 consecutive fp32 values -> packed bf16 h, m, l MFMA operands (x = h + m + l).
__device__ __forceinline__ void split8(const f32x4& a, const f32x4& b, u32x4& hi, u32x4& mi,
                                       u32x4& lo) {
  const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t h[2], m[2], l[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float x = v[2 * q + e];
      h[e] = rne_bf16(x);
      const float r1 = x - __uint_as_float(h[e] << 16);
      m[e] = rne_bf16(r1);
      l[e] = rne_bf16(r1 - __uint_as_float(m[e] << 16));
    }
    hi[q] = h[0] | (h[1] << 16);
    mi[q] = m[0] | (m[1] << 16);
    lo[q] = l[0] | (l[1] << 16);
  }
}

__device__ __forceinline__ f32x4 mfma16(const u32x4& a, const u32x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                  __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// Q (d x p, row stride ldq) -> image [k-group g = k/32][n-block j][h|m|l][lane][16 B],
// lane l of (g, j) holding Q[32 g + 8 (l/16) + e][16 j + l%16], e = 0..7; k-groups
// beyond d are zeros.  One thread per (g, j, lane).
__global__ __launch_bounds__(256) void split_q_kernel(const float* __restrict__ Q, int64_t ldq,
                                                      int64_t d, int nb, int64_t ngrp,
                                                      u32x4* __restrict__ QS) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= ngrp * nb * 64) return;
  const int lane = (int)(idx & 63);
  const int64_t t = idx >> 6;  // g * nb + j
  const int j = (int)(t % nb);
  const int64_t g = t / nb;
  const int n = 16 * j + (lane & 15);
  const int64_t k0 = 32 * g + 8 * (lane >> 4);
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (k0 + e < d) ? Q[(k0 + e) * ldq + n] : 0.f;
  u32x4 hi, mi, lo;
  split8(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, hi, mi, lo);
  QS[(t * 3 + 0) * 64 + lane] = hi;
  QS[(t * 3 + 1) * 64 + lane] = mi;
  QS[(t * 3 + 2) * 64 + lane] = lo;
}

template <int NB>
__global__ __launch_bounds__(SW_THR) void sweep_kernel(const float* __restrict__ S, int64_t lds,
                                                       int64_t d, const u32x4* __restrict__ QS,
                                                       int64_t nsteps, float* __restrict__ Y,
                                                       int64_t ldy, float alpha,
                                                       float* __restrict__ part) {
  constexpr int BV = 2 * NB * 3 * 64;  // 16-B units of one Q stage (2 k-groups)
  constexpr int BPT = (BV + SW_THR - 1) / SW_THR;
  __shared__ u32x4 Bs[2][BV];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, gq = lane >> 4;
  const int64_t row0 = (int64_t)blockIdx.x * SW_ROWS + 32 * wave;
  const int ks = gridDim.y, sl = blockIdx.y;
  const int64_t c0 = nsteps * sl / ks, c1 = nsteps * (sl + 1) / ks;

  f32x4 acc[2][NB];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[mb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 ra[2][2][2];  // [m-block][k-group][half] raw fp32 rows of S for one stage
  u32x4 rq[BPT];

  auto load_a = [&](int64_t step) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      const int64_t row = row0 + 16 * mb + r;
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int64_t col = step * SW_KS + 32 * g + 8 * gq;
        if (row < d && col + 8 <= d) {
          const f32x4* p = reinterpret_cast<const f32x4*>(S + row * lds + col);
          ra[mb][g][0] = p[0];
          ra[mb][g][1] = p[1];
        } else {
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (row < d && col + e < d) ? S[row * lds + col + e] : 0.f;
          ra[mb][g][0] = f32x4{v[0], v[1], v[2], v[3]};
          ra[mb][g][1] = f32x4{v[4], v[5], v[6], v[7]};
        }
      }
    }
  };
  auto load_q = [&](int64_t step) {
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      const int f = tid + u * SW_THR;
      rq[u] = (f < BV) ? QS[step * BV + f] : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto store_q = [&](int buf) {
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      const int f = tid + u * SW_THR;
      if (f < BV) Bs[buf][f] = rq[u];
    }
  };

  if (c0 < c1) {
    load_a(c0);
    load_q(c0);
    store_q(0);
    __syncthreads();
    int cur = 0;
    for (int64_t step = c0; step < c1; ++step) {
      const bool more = step + 1 < c1;
      u32x4 ah[2][2], am[2][2], al[2][2];
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int g = 0; g < 2; ++g)
          split8(ra[mb][g][0], ra[mb][g][1], ah[mb][g], am[mb][g], al[mb][g]);
      if (more) {
        load_a(step + 1);
        load_q(step + 1);
      }
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const u32x4 bh = Bs[cur][((g * NB + j) * 3 + 0) * 64 + lane];
          const u32x4 bm = Bs[cur][((g * NB + j) * 3 + 1) * 64 + lane];
          const u32x4 bl = Bs[cur][((g * NB + j) * 3 + 2) * 64 + lane];
#pragma unroll
          for (int mb = 0; mb < 2; ++mb) {  // small terms first
            acc[mb][j] = mfma16(am[mb][g], bm, acc[mb][j]);
            acc[mb][j] = mfma16(ah[mb][g], bl, acc[mb][j]);
            acc[mb][j] = mfma16(al[mb][g], bh, acc[mb][j]);
            acc[mb][j] = mfma16(ah[mb][g], bm, acc[mb][j]);
            acc[mb][j] = mfma16(am[mb][g], bh, acc[mb][j]);
            acc[mb][j] = mfma16(ah[mb][g], bh, acc[mb][j]);
          }
        }
      if (more) store_q(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  }

  // C/D layout of 16x16x32: row 4 (l / 16) + e, column l % 16
  constexpr int P = 16 * NB;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = row0 + 16 * mb + 4 * gq + e;
        if (row < d) {
          if (ks == 1)
            Y[row * ldy + 16 * j + r] = alpha * acc[mb][j][e];
          else
            part[((int64_t)sl * d + row) * P + 16 * j + r] = acc[mb][j][e];
        }
      }
}

__global__ __launch_bounds__(256) void sweep_reduce_kernel(const float* __restrict__ part, int ks,
                                                           int64_t d, int p, float alpha,
                                                           float* __restrict__ Y, int64_t ldy) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * p) return;
  const int64_t m = idx / p;
  const int n = (int)(idx - m * p);
  float s = 0.f;
  for (int k = 0; k < ks; ++k) s += part[(int64_t)k * d * p + idx];
  Y[m * ldy + n] = alpha * s;
}

int sweep_bpc() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DEIG_SWEEP_BPC");
    v = (e && atoi(e) > 0) ? atoi(e) : 1;
  }
  return v;
}

// Split-K slices: about sweep_bpc() blocks per CU, >= 4 K-steps per slice.
int sweep_ks(int64_t d) {
  const int64_t bx = cdiv(d, SW_ROWS), nsteps = cdiv(d, SW_KS);
  int64_t ks = cdiv((int64_t)num_cus() * sweep_bpc(), bx);
  const int64_t cap = nsteps / 4 > 1 ? nsteps / 4 : 1;
  if (ks > cap) ks = cap;
  if (ks < 1) ks = 1;
  return (int)ks;
}

// Q image: 3 bf16 pieces per value
size_t qs_bytes(int64_t d, int p) { return (size_t)cdiv(d, SW_KS) * SW_KS * p * 6; }

template <int NB>
void launch_nb(dim3 grid, hipStream_t st, const float* S, int64_t lds, int64_t d, const u32x4* QS,
               int64_t nsteps, float* Y, int64_t ldy, float alpha, float* part) {
  hipLaunchKernelGGL(sweep_kernel<NB>, grid, dim3(SW_THR), 0, st, S, lds, d, QS, nsteps, Y, ldy,
                     alpha, part);
}

}  // namespace

size_t sweep_workspace_bytes(int64_t d, int p) {
  const int ks = sweep_ks(d);
  size_t total = align_up(qs_bytes(d, p), 256);
  if (ks > 1) total += (size_t)ks * d * p * sizeof(float);
  return total;
}

int sweep_launch(const float* S, int64_t d, int64_t lds, const float* Q, int p, int64_t ldq,
                 float* Y, int64_t ldy, float alpha, void* ws, size_t ws_bytes, hipStream_t st) {
  DEIG_REQUIRE(d >= 1 && p >= 16 && p <= 128 && p % 16 == 0,
               "sweep: need d >= 1 and p in {16, 32, ..., 128} (p=%d)", p);
  DEIG_REQUIRE(lds >= d && lds % 4 == 0 && ldq >= p && ldy >= p, "sweep: bad leading dims");
  DEIG_REQUIRE(S && Q && Y && aligned16(S), "sweep: S must be 16-byte aligned");
  const size_t need = sweep_workspace_bytes(d, p);
  if (!ws || ws_bytes < need)
    return fail(DEIG_EWORKSPACE, "sweep: workspace %zu < %zu", ws_bytes, need);
  const int nb = p / 16;
  const int64_t nsteps = cdiv(d, SW_KS);
  const int64_t ngrp = 2 * nsteps;
  u32x4* QS = static_cast<u32x4*>(ws);
  float* part = reinterpret_cast<float*>(static_cast<char*>(ws) + align_up(qs_bytes(d, p), 256));
  hipLaunchKernelGGL(split_q_kernel, dim3((unsigned)cdiv(ngrp * nb * 64, 256)), dim3(256), 0, st,
                     Q, ldq, d, nb, ngrp, QS);
  DEIG_HIP_CHECK(hipGetLastError());
  const int ks = sweep_ks(d);
  const dim3 grid((unsigned)cdiv(d, SW_ROWS), (unsigned)ks);
  switch (nb) {
    case 1: launch_nb<1>(grid, st, S, lds, d, QS, nsteps, Y, ldy, alpha, part); break;
    case 2: launch_nb<2>(grid, st, S, lds, d, QS, nsteps, Y, ldy, alpha, part); break;
    case 3: launch_nb<3>(grid, st, S, lds, d, QS, nsteps, Y, ldy, alpha, part); break;
    case 4: launch_nb<4>(grid, st, S, lds, d, QS, nsteps, Y, ldy, alpha, part); break;
    case 5: launch_nb<5>(grid, st, S, lds, d, QS, nsteps, Y, ldy, alpha, part); break;
    case 6: launch_nb<6>(grid, st, S, lds, d, QS, nsteps, Y, ldy, alpha, part); break;
    case 7: launch_nb<7>(grid, st, S, lds, d, QS, nsteps, Y, ldy, alpha, part); break;
    default: launch_nb<8>(grid, st, S, lds, d, QS, nsteps, Y, ldy, alpha, part); break;
  }
  DEIG_HIP_CHECK(hipGetLastError());
  if (ks > 1) {
    hipLaunchKernelGGL(sweep_reduce_kernel, dim3((unsigned)cdiv(d * p, 256)), dim3(256), 0, st,
                       part, ks, d, p, alpha, Y, ldy);
    DEIG_HIP_CHECK(hipGetLastError());
  }
  return DEIG_OK;
}

}  // namespace deig
