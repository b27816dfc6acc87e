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
// two register stages of the S rows and of the Q stage.  Split-K over ks
// slices (XCD-aware block order); partial slabs are summed in slice order
// (deterministic).
//
// Measured (d = 8192, p = 80, rocprofv3, one MI355X): 90 us per launch (+4 us
// split_q, +6 us reduce) = 3.0 TB/s of S.  Attribution by knock-out builds of
// the same kernel: without S loads 64 us, without MFMAs 84 us, without both 36 us
// (Q-stage loads/LDS stores 15 us of it, the split 10 us); S read as one
// contiguous 8 KiB run per wave-step instead of 32 rows x 256 B: -11 us.  The
// phases add rather than overlap (the per-step barrier keeps the 8 waves in
// lock-step), so the next lever is a staggered / warp-specialised schedule, not
// more bandwidth.
#include <stdlib.h>

#include <type_traits>

#include "deig_internal.hpp"

namespace deig {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int SW_THR = 512;   // 8 waves
constexpr int SW_ROWS = 256;  // rows per block: 8 waves x 2 x 16
constexpr int SW_KS = 64;     // k per stage

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Two fp32 -> packed bf16 (element 0 in the low half), round to nearest even;
// one v_cvt_pk_bf16_f32 (NaN stays NaN).
__device__ __forceinline__ uint32_t cvt2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
__device__ __forceinline__ float lo_f(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float hi_f(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }

// 8 consecutive fp32 values -> packed bf16 h, m, l MFMA operands (x = h + m + l).
__device__ __forceinline__ void split8(const f32x4& a, const f32x4& b, u32x4& hi, u32x4& mi,
                                       u32x4& lo) {
  const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float x0 = v[2 * q], x1 = v[2 * q + 1];
    const uint32_t h = cvt2(x0, x1);
    const float r0 = x0 - lo_f(h), r1 = x1 - hi_f(h);
    const uint32_t m = cvt2(r0, r1);
    hi[q] = h;
    mi[q] = m;
    lo[q] = cvt2(r0 - lo_f(m), r1 - hi_f(m));
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
  // 1-D grid of bx row blocks x ks split-K slices, XCD-aware: consecutive logical
  // ids (one XCD) take consecutive row blocks of ONE slice, so an XCD's L2 holds
  // only that slice's part of the Q image.
  const int bx = (int)cdiv(d, SW_ROWS);
  const int ks = (int)(gridDim.x / bx);
  const int lid = xcd_logical(blockIdx.x, gridDim.x);
  const int sl = lid / bx;
  const int64_t row0 = (int64_t)(lid - sl * bx) * SW_ROWS + 32 * wave;
  const int64_t c0 = nsteps * sl / ks, c1 = nsteps * (sl + 1) / ks;

  f32x4 acc[2][NB];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[mb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // Two register stages of raw fp32 S rows ([stage][m-block][k-group][half]) and
  // of the Q image: S(s + 2) and Q(s + 2) are issued while step s computes, S
  // before Q, so the in-order vmcnt wait for Q(s + 1) (needed by its LDS store at
  // the end of step s) leaves S(s + 2) in flight - about two steps of latency
  // cover instead of none (__syncthreads() would wait for everything).
  f32x4 ra[2][2][2][2];
  u32x4 rq[2][BPT];

  // S rows through a per-wave buffer descriptor over this wave's 32 rows: one
  // straight-line 16-B load per operand half, no branches (a divergent branch
  // makes the compiler wait for every outstanding load).  Rows >= d read as 0
  // (range check); columns >= d are zeroed when the step is consumed.
  const int64_t wrows = d - row0 < 32 ? (d - row0 > 0 ? d - row0 : 0) : 32;
  const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(S + (row0 < d ? row0 : 0) * lds), 0, (int)(wrows * lds * 4), 0x00020000);
  auto load_a = [&](f32x4 (&dst)[2][2][2], int64_t step) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int off = (int)(((16 * mb + r) * lds + step * SW_KS + 32 * g + 8 * gq + 4 * h) * 4);
          dst[mb][g][h] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(srs, off, 0, 0));
        }
  };
  auto mask_cols = [&](f32x4 (&v)[2][2][2], int64_t step) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (step * SW_KS + 32 * g + 8 * gq + 4 * h + e >= d) v[mb][g][h][e] = 0.f;
  };
  auto load_q = [&](u32x4 (&dst)[BPT], int64_t step) {
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      const int f = tid + u * SW_THR;
      dst[u] = QS[step * BV + (f < BV ? f : BV - 1)];  // lanes past BV are not stored
    }
  };
  auto store_q = [&](const u32x4 (&src)[BPT], int buf) {
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      const int f = tid + u * SW_THR;
      if (f < BV) Bs[buf][f] = src[u];
    }
  };
  auto barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // Step `step` with its S rows in ra[B] and its Q stage in Bs[B].
  auto body = [&](auto Bc, int64_t step) {
    constexpr int B = decltype(Bc)::value;
    u32x4 ah[2][2], am[2][2], al[2][2];
    if ((step + 1) * SW_KS > d) mask_cols(ra[B], step);  // wave-uniform, last step only
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int g = 0; g < 2; ++g)
        split8(ra[B][mb][g][0], ra[B][mb][g][1], ah[mb][g], am[mb][g], al[mb][g]);
    // Unconditional (the last two steps re-load the last step: straight-line
    // code, no phi copies of in-flight registers).
    const int64_t pf = step + 2 < c1 ? step + 2 : c1 - 1;
    load_a(ra[B], pf);
    load_q(rq[B], pf);
    __builtin_amdgcn_sched_barrier(0);  // issue the loads here, ahead of the MFMAs
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const u32x4 bh = Bs[B][((g * NB + j) * 3 + 0) * 64 + lane];
        const u32x4 bm = Bs[B][((g * NB + j) * 3 + 1) * 64 + lane];
        const u32x4 bl = Bs[B][((g * NB + j) * 3 + 2) * 64 + lane];
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
    // Bs[B ^ 1] was last read in step - 1, before the previous barrier.
    store_q(rq[B ^ 1], B ^ 1);  // Q(step + 1) (after the last step: unread)
    barrier();
  };

  if (c0 < c1) {
    const int64_t c01 = c0 + 1 < c1 ? c0 + 1 : c0;
    load_a(ra[0], c0);
    load_q(rq[0], c0);
    load_a(ra[1], c01);
    load_q(rq[1], c01);
    store_q(rq[0], 0);
    barrier();
    int64_t step = c0;
    for (; step + 1 < c1; step += 2) {
      body(std::integral_constant<int, 0>{}, step);
      body(std::integral_constant<int, 1>{}, step + 1);
    }
    if (step < c1) body(std::integral_constant<int, 0>{}, step);
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
  DEIG_REQUIRE(lds >= d && lds % 4 == 0 && lds <= (1 << 24) && ldq >= p && ldy >= p,
               "sweep: bad leading dims");
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
  const dim3 grid((unsigned)(cdiv(d, SW_ROWS) * ks));
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
