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
// along k).  S is re-laid once per solve into an image in MFMA A-operand order
// (sweep_prepare_kernel), which the sweep kernels stream as one contiguous run per
// wave (v2: independent waves, Q fragments in registers; v3: the Q image shared
// through an LDS-DMA ring).  Split-K over an XCD-aware grid; slabs summed in slice
// order (deterministic), fused with the solver's basis step (sweep_finish_kernel).
#include <type_traits>

#include "deig_internal.hpp"

namespace deig {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int SW_KS = 64;  // k per sweep step (two 32-deep MFMA k-groups)

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

// Q (d x p, row stride ldq) -> image [k-group g = k/32][n-block j][piece][lane][16 B],
// lane l of (g, j) holding Q[32 g + 8 (l/16) + e][16 j + l%16], e = 0..7; k-groups
// beyond d are zeros.  One thread per (g, j, lane).
// NP = 3: pieces h|m|l, Q represented to 2^-27 (the exact product, Q read-only).
// NP = 2 (the solver's in-place mode): pieces h|m, and Q itself is rounded to
// Q' = h + m (exact in fp32: 17 significant bits at most) and written back, so
// the sweep computes S Q' to fp32 grade with five products (the dropped l*m term
// is ~2^-24) and the Gram / Rayleigh-Ritz that follow see the same Q'.  The
// solver only needs Y = S Q for the basis it holds; a 2^-17 perturbation of
// that basis changes nothing it reports (the generalised RR accepts any Q).
template <int NP>
__global__ __launch_bounds__(256) void split_q_kernel(float* __restrict__ Q, int64_t ldq,
                                                      int64_t d, int nb, int64_t ngrp,
                                                      u32x4* __restrict__ QS, int per,
                                                      const SweepBatch sb) {
  const int prob = blockIdx.x / per;
  if (prob) {
    Q = reinterpret_cast<float*>(reinterpret_cast<char*>(Q) + sb.off[prob]);
    QS = reinterpret_cast<u32x4*>(reinterpret_cast<char*>(QS) + sb.off[prob]);
  }
  const int64_t idx = (int64_t)(blockIdx.x - prob * per) * 256 + threadIdx.x;
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
  QS[(t * NP + 0) * 64 + lane] = hi;
  QS[(t * NP + 1) * 64 + lane] = mi;
  if constexpr (NP == 3) {
    QS[(t * NP + 2) * 64 + lane] = lo;
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t k = k0 + 2 * q;
      if (k < d) Q[k * ldq + n] = lo_f(hi[q]) + lo_f(mi[q]);
      if (k + 1 < d) Q[(k + 1) * ldq + n] = hi_f(hi[q]) + hi_f(mi[q]);
    }
  }
}

// The products of one Q fragment (pieces bh, bm[, bl]) with MB split S
// fragments into column block j, small terms first, MB independent accumulators
// between dependent MFMAs.  NP = 3: hh + hm + mh + hl + lh + mm (six); NP = 2
// (Q = bh + bm exactly): hh + hm + mh + mm + lh (five; bl unused).  SP = 2 (the
// early-sweep mode: S taken as its two leading pieces, Q two pieces): hh + hm + mh
// (three; al, bl unused; dropped m m ~2^-18, S's own rounding 2^-17).
template <int MB, int NP, int SP, int NB>
__device__ __forceinline__ void sweep_products(f32x4 (&acc)[MB][NB], int j, const u32x4 (&ah)[MB],
                                               const u32x4 (&am)[MB], const u32x4 (&al)[MB],
                                               const u32x4& bh, const u32x4& bm,
                                               const u32x4& bl) {
  if constexpr (SP == 2) {
    static_assert(NP == 2, "two-piece S pairs with two-piece Q");
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(ah[mb], bm, acc[mb][j]);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(am[mb], bh, acc[mb][j]);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(ah[mb], bh, acc[mb][j]);
    return;
  }
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(am[mb], bm, acc[mb][j]);
  if constexpr (NP == 3) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(ah[mb], bl, acc[mb][j]);
  }
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(al[mb], bh, acc[mb][j]);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(ah[mb], bm, acc[mb][j]);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(am[mb], bh, acc[mb][j]);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(ah[mb], bh, acc[mb][j]);
}

// ---------------------------------------------------------------- sweep v2
// S image: S re-laid once per solve (sweep_prepare_kernel) in MFMA A-operand
// order so that every wave streams one contiguous run of HBM:
//   [64-row block rb][k-group g (32 k)][m-block mb (4)][half h (2)][lane][16 B],
// lane l of (rb, g, mb, h) holding S[64 rb + 16 mb + l%16][32 g + 8 (l/16) + 4 h .. +3].
// One (rb, g) chunk is 8 KiB; rows are padded to a multiple of 256 and columns
// to a multiple of 32 with zeros (no masking, no range checks in the sweep).
// Row-major S read 16 rows x 128 B per wave-instruction streamed at ~4 TB/s
// (knock-out: S loads + split alone 65 us at d = 8192); the image is read in
// 1-KiB contiguous wave-instructions.
constexpr int SI_RB = 64;    // rows per image row block (one wave)
constexpr int SI_BR = 256;   // rows per sweep2 block (4 waves)

__host__ __device__ inline int64_t si_rows(int64_t d) { return cdiv(d, SI_BR) * SI_BR; }
__host__ __device__ inline int64_t si_groups(int64_t d) { return cdiv(d, 32); }
size_t si_bytes(int64_t d) { return (size_t)si_rows(d) * si_groups(d) * 32 * 4; }

// One thread per (rb, g, mb, lane): reads 32 contiguous bytes of one row (64 for
// a float64 S), writes the two 16-B halves (h = 0, 1) 1 KiB apart (d = 8192: 88 us
// = 6.1 TB/s of read + write; an LDS-transposed variant with whole-row reads took
// 131 us).  The image is of
//   S + shift I - V_D diag(lam_D) V_D^T
// with the shift and the optional deflation (r locked / dominant eigenpairs, V_D
// column-major with ldv) formed in DOUBLE from S's own values and rounded to fp32
// once: the deflated entries then carry fp32 rounding relative to THEIR size, not
// to the dominant eigenvalues' (for a float64 S - the reference's dtype - this is
// what keeps the small eigenvectors at float64 parity; an fp32 chain of fmas
// would round every intermediate at |S_ij|).  shift: the solver's indefinite-input
// shift (capi.hip), 0 otherwise.
template <typename T>
__global__ __launch_bounds__(256) void sweep_prepare_kernel(const T* __restrict__ S, int64_t lds,
                                                            int64_t d, int64_t ng, int64_t nunits,
                                                            f32x4* __restrict__ SI,
                                                            u32x4* __restrict__ SH,
                                                            const float* __restrict__ Vd,
                                                            int64_t ldv,
                                                            const float* __restrict__ lamd, int r,
                                                            double shift) {
  const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (u >= nunits) return;
  const int lane = (int)(u & 63);
  const int mb = (int)((u >> 6) & 3);
  const int64_t t = u >> 8;  // rb * ng + g
  const int64_t rb = t / ng, g = t - rb * ng;
  const int64_t row = SI_RB * rb + 16 * mb + (lane & 15);
  const int64_t k = 32 * g + 8 * (lane >> 4);
  f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = {0.f, 0.f, 0.f, 0.f};
  if (row < d) {
    const T* src = S + row * lds + k;
    if (r == 0 && shift == 0.0 && std::is_same<T, float>::value) {  // plain copy
      if (k + 8 <= d) {
        v0 = *reinterpret_cast<const f32x4*>(src);
        v1 = *reinterpret_cast<const f32x4*>(src + 4);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (k + e < d) v0[e] = (float)src[e];
          if (k + 4 + e < d) v1[e] = (float)src[4 + e];
        }
      }
    } else {
      double v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (k + e < d) ? (double)src[e] : 0.0;
      if (row >= k && row < k + 8) v[row - k] += shift;
      for (int q = 0; q < r; ++q) {
        const float* vq = Vd + (int64_t)q * ldv;
        const double a = -(double)lamd[q] * (double)vq[row];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (k + e < d) v[e] = fma(a, (double)vq[k + e], v[e]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v0[e] = (float)v[e];
        v1[e] = (float)v[4 + e];
      }
    }
  }
  f32x4* dst = SI + ((t * 4 + mb) * 2) * 64 + lane;
  dst[0] = v0;
  dst[64] = v1;
  // two-piece image (same addressing): the h and m pieces of these 8 values, the
  // early sweeps' operand - read as is, no split in the sweep
  u32x4 h, m, l;
  split8(v0, v1, h, m, l);
  u32x4* dh = SH + ((t * 4 + mb) * 2) * 64 + lane;
  dh[0] = h;
  dh[64] = m;
}

// Sweep kernel v2: independent waves, no LDS, no barriers.
//
// Each wave owns 64 rows (MB = 4 m-blocks) of the S image and one split-K
// slice of k-groups.  Per k-group it loads its 8 KiB of S (8 x 1 KiB, one
// contiguous run from HBM) and the group's Q image fragments (NB x 3 x 1 KiB
// from L2: the XCD-aware slice order keeps an XCD on one slice of the image),
// splits S into h/m/l in registers and issues MB * NB * 6 MFMAs.  Q reuse is
// MB m-blocks per fragment, so the image is read from L2 p*6/256 times as many
// bytes as S from HBM (1.9x at p = 80), but there is no block-wide lock-step:
// the four waves of a CU (one per SIMD, up to 512 registers each) stream
// independently, each with a D-deep register ring of S and Q fragments.
// PROBE (knock-out builds for attribution, never launched by the library): bit 0
// drops the MFMAs, bit 1 the S loads, bit 2 the Q loads (results are garbage).
// PRE: SI is the two-piece image (sweep_prepare_kernel's SH: h | m per half slot)
// and the products are the three of SP = 2 - the early-sweep mode, no split.
// per / sb (every sweep kernel): one launch may cover sb.n problems of the same shape
// (the batched worker solves, capi.hip solve_batch): logical blocks [i per, (i + 1) per)
// are problem i's, and every pointer of problem i is problem 0's plus sb.off[i] bytes
// (the solver workspaces are equally carved slices of one allocation).  One problem:
// per = the grid, sb.n = 1.
template <int NB, int NP, int PROBE = 0, bool PRE = false>
__global__ __launch_bounds__(256, 1) void sweep2_kernel(const f32x4* __restrict__ SI, int64_t d,
                                                        const u32x4* __restrict__ QS,
                                                        int64_t ngrp, float* __restrict__ Y,
                                                        int64_t ldy, float alpha,
                                                        float* __restrict__ part, int per,
                                                        const SweepBatch sb) {
  constexpr int MB = 4;
  // logical block ids are XCD-contiguous (xcd_logical), so one problem's blocks share
  // an XCD's L2
  const int gl = xcd_logical(blockIdx.x, gridDim.x);
  const int prob = gl / per, lid = gl - prob * per;
  if (prob) {
    const int64_t po = sb.off[prob];
    SI = reinterpret_cast<const f32x4*>(reinterpret_cast<const char*>(SI) + po);
    QS = reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(QS) + po);
    Y = reinterpret_cast<float*>(reinterpret_cast<char*>(Y) + po);
    part = reinterpret_cast<float*>(reinterpret_cast<char*>(part) + po);
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, gq = lane >> 4;
  const int bx = (int)cdiv(d, SI_BR);
  const int ks = per / bx;
  const int sl = lid / bx;
  const int64_t rb = (int64_t)(lid - sl * bx) * (SI_BR / SI_RB) + wave;
  const int64_t row0 = rb * SI_RB;
  const int64_t c0 = ngrp * sl / ks, c1 = ngrp * (sl + 1) / ks;

  f32x4 acc[MB][NB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[mb][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Register rings: S rows of 3 groups (the split runs one group ahead of the
  // MFMAs, so S is needed two bodies after its load is issued), Q fragments of
  // 2 groups, S pieces of 2 groups (the MFMAs of group g read set g & 1 while
  // the split of group g + 1 fills the other, interleaved with them).
  const f32x4* sw = SI + rb * ngrp * (MB * 2 * 64) + lane;
  f32x4 sr[3][MB][2];
  u32x4 qf[2][NB][NP];
  u32x4 pc[2][3][MB];
  auto clampg = [&](int64_t g) { return g < c1 ? g : c1 - 1; };
  auto load_s = [&](int b, int64_t g) {
    const f32x4* sg = sw + clampg(g) * (MB * 2 * 64);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if constexpr (PROBE & 2)
          sr[b][mb][h] = f32x4{(float)g, (float)mb, (float)h, (float)lane};
        else
          sr[b][mb][h] = sg[(mb * 2 + h) * 64];
      }
  };
  auto load_q = [&](int b, int64_t g) {
    const u32x4* qg = QS + clampg(g) * (NB * NP * 64) + lane;
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int p3 = 0; p3 < NP; ++p3) {
        if constexpr (PROBE & 4)
          qf[b][j][p3] = u32x4{(unsigned)g, (unsigned)j, (unsigned)p3, (unsigned)lane};
        else
          qf[b][j][p3] = qg[(j * NP + p3) * 64];
      }
  };
  auto split_into = [&](int ps, int b) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      if constexpr (PRE) {
        pc[ps][0][mb] = __builtin_bit_cast(u32x4, sr[b][mb][0]);
        pc[ps][1][mb] = __builtin_bit_cast(u32x4, sr[b][mb][1]);
        pc[ps][2][mb] = pc[ps][1][mb];  // unused by the SP = 2 products
      } else {
        split8(sr[b][mb][0], sr[b][mb][1], pc[ps][0][mb], pc[ps][1][mb], pc[ps][2][mb]);
      }
    }
  };
  // Body of group g: S slot of g + 1 is SB1 = (g + 1) % 3, Q slot / piece set
  // QB = g & 1.  The tail loads and splits clamped copies of the last group.
  auto body = [&](auto SBc, auto QBc, int64_t g) {
    constexpr int SB1 = decltype(SBc)::value, QB = decltype(QBc)::value;
    const u32x4(&ah)[MB] = pc[QB][0];
    const u32x4(&am)[MB] = pc[QB][1];
    const u32x4(&al)[MB] = pc[QB][2];
    split_into(QB ^ 1, SB1);
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const u32x4 bh = qf[QB][j][0], bm = qf[QB][j][1], bl = qf[QB][j][NP - 1];
      if constexpr (PROBE & 1) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          acc[mb][j][0] += __uint_as_float((ah[mb][0] ^ am[mb][1] ^ al[mb][2] ^ bh[0] ^ bm[1] ^ bl[2]) & 0x3fffffffu);
        continue;
      }
      sweep_products<MB, NP, PRE ? 2 : 3>(acc, j, ah, am, al, bh, bm, bl);
    }
    load_q(QB, g + 2);   // the Q slot just consumed
    load_s(SB1, g + 4);  // the S slot just split
    // Keep the refills here: at this register pressure the scheduler otherwise
    // sinks the loads next to their use (a vmcnt(0) per group).
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;

  if (c0 < c1) {
    load_s(0, c0);
    load_q(0, c0);
    load_s(1, c0 + 1);
    load_q(1, c0 + 1);
    load_s(2, c0 + 2);
    __builtin_amdgcn_sched_barrier(0);
    split_into(0, 0);  // S(c0) -> piece set 0; slot 0 then takes S(c0 + 3)
    load_s(0, c0 + 3);
    __builtin_amdgcn_sched_barrier(0);
    // Six bodies per trip: S slot of g + 1 = (g + 1) % 3, Q slot = g & 1.
    int64_t g = c0;
    for (; g + 6 <= c1; g += 6) {
      body(I1{}, I0{}, g);
      body(I2{}, I1{}, g + 1);
      body(I0{}, I0{}, g + 2);
      body(I1{}, I1{}, g + 3);
      body(I2{}, I0{}, g + 4);
      body(I0{}, I1{}, g + 5);
    }
    if (g < c1) body(I1{}, I0{}, g);
    if (g + 1 < c1) body(I2{}, I1{}, g + 1);
    if (g + 2 < c1) body(I0{}, I0{}, g + 2);
    if (g + 3 < c1) body(I1{}, I1{}, g + 3);
    if (g + 4 < c1) body(I2{}, I0{}, g + 4);
  }

  constexpr int P = 16 * NB;
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
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

// Sweep kernel v3: v2's S image stream with the Q image shared through LDS.
//
// v2 loads every Q fragment into every wave (1.9x the S bytes through the CU's
// load path at p = 80; knock-outs: S + Q loads alone 62 us vs S alone 47 us).
// Here the four waves of a block DMA each k-group's Q image (3 NB KiB, 1-KiB
// pieces spread over the waves) into a (D + 1)-slot LDS ring with
// buffer_load ... lds, issued D groups ahead together with the S registers, and
// read the fragments back with conflict-free ds_read_b128: Q traffic drops to
// p*6/1024 of the S bytes.  One raw s_barrier per group publishes the slot
// (the DMA of group g is older than the S loads of group g, so the wait for
// those covers it); the slot refilled at group g was last read at g - 1.
__device__ __forceinline__ void sw_dma16(const __amdgpu_buffer_rsrc_t rsrc, int voff,
                                         const void* lds_dst) {
  // uniform, but the compiler may compute it in VGPRs (packed 16-bit slot arithmetic)
  const unsigned m0v = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void*)lds_dst);
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :
               : "v"(voff), "s"(rsrc), "s"(m0v)
               : "memory", "m0");
}

// body(integral_constant<B>, g + B) for B = B0 .. D - 1 (tail: only while g + B < c1).
template <int B, int D>
struct UnrollBodies {
  template <class F>
  static __device__ __forceinline__ void run(F& f, int64_t g, int64_t c1, bool tail) {
    if (!tail || g + B < c1) f(std::integral_constant<int, B>{}, g + B);
    UnrollBodies<B + 1, D>::run(f, g, c1, tail);
  }
};
template <int D>
struct UnrollBodies<D, D> {
  template <class F>
  static __device__ __forceinline__ void run(F&, int64_t, int64_t, bool) {}
};

// MBW: 16-row m-blocks per wave (4: 64 rows, one image row block; 2: half of one,
// so a block covers 128 rows and the grid needs half the split-K slices).
// HALF (with PRE): S and Q both as their leading bf16 piece alone, one product per
// fragment pair (~2^-9 relative: the solver's first sweeps, residual > 1e-2) - half
// the S bytes of the PRE mode (the h slots of the two-piece image) and half the Q
// image pieces.
template <int NB, int NP, int D, int OCC = 1, bool PRE = false, int MBW = 4, bool HALF = false>
__global__ __launch_bounds__(256, OCC) void sweep3_kernel(const f32x4* __restrict__ SI, int64_t d,
                                                        const u32x4* __restrict__ QS,
                                                        int64_t ngrp, float* __restrict__ Y,
                                                        int64_t ldy, float alpha,
                                                        float* __restrict__ part, int per,
                                                        const SweepBatch sb) {
  // logical block ids are XCD-contiguous (xcd_logical), so one problem's blocks share
  // an XCD's L2
  const int gl = xcd_logical(blockIdx.x, gridDim.x);
  const int prob = gl / per, lid = gl - prob * per;
  if (prob) {
    const int64_t po = sb.off[prob];
    SI = reinterpret_cast<const f32x4*>(reinterpret_cast<const char*>(SI) + po);
    QS = reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(QS) + po);
    Y = reinterpret_cast<float*>(reinterpret_cast<char*>(Y) + po);
    part = reinterpret_cast<float*>(reinterpret_cast<char*>(part) + po);
  }
  constexpr int MB = MBW;
  static_assert(MB == 2 || MB == 4, "m-blocks per wave");
  static_assert(!HALF || PRE, "the one-piece mode reads the two-piece image");
  constexpr int QU = NP * NB;        // 1-KiB Q image pieces per k-group
  constexpr int U = HALF ? NB : QU;  // of those, staged (HALF: the h piece of each block)
  constexpr int SPC = HALF ? 1 : 2;  // S image slots loaded per m-block
  constexpr int ND = (U + 3) / 4;    // DMAs per wave per group (tail pieces repeated)
  constexpr int SLOT = U * 1024;     // bytes per ring slot
  constexpr int NS = D + 1;          // ring slots
  static_assert(NS * SLOT <= 160 * 1024, "Q ring exceeds LDS");
  __shared__ __attribute__((aligned(16))) unsigned char qlds[NS * SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, gq = lane >> 4;
  const int bx = (int)cdiv(d, 4 * 16 * MB);
  const int ks = per / bx;
  const int sl = lid / bx;
  const int64_t rb = (int64_t)(lid - sl * bx) * 4 + wave;  // this wave's 16 MB rows
  const int64_t row0 = rb * 16 * MB;
  const int64_t c0 = ngrp * sl / ks, c1 = ngrp * (sl + 1) / ks;

  f32x4 acc[MB][NB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[mb][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<u32x4*>(QS), 0, (int)(ngrp * QU * 1024), 0x00020000);
  // image row block row0 / 64, starting at its m-block (row0 % 64) / 16
  const f32x4* sw = SI + (row0 / SI_RB) * ngrp * (4 * 2 * 64) + ((row0 % SI_RB) / 16) * 2 * 64 + lane;
  f32x4 sr[D][MB][2];
  auto load = [&](int b, int64_t g) {
    // Q pieces first: the compiler's wait for this group's S registers then
    // also covers them.
    unsigned char* slot = qlds + (int)(g % NS) * SLOT;
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      const int u = wave + 4 * i < U ? wave + 4 * i : U - 1;
      const int64_t src = HALF ? (g * NB + u) * NP : g * U + u;
      sw_dma16(qrs, (int)(src * 1024) + lane * 16, slot + u * 1024);
    }
    const f32x4* sg = sw + g * (4 * 2 * 64);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int h = 0; h < SPC; ++h) sr[b][mb][h] = sg[(mb * 2 + h) * 64];
  };
  auto body = [&](auto Bc, int64_t g) {
    constexpr int B = decltype(Bc)::value;
    // Everything issued before the D - 1 younger groups has landed: this
    // group's Q pieces (every wave's, after the barrier) and S registers.
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"((D - 1) * (ND + SPC * MB))
                 : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    u32x4 ah[MB], am[MB], al[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      if constexpr (HALF) {
        ah[mb] = __builtin_bit_cast(u32x4, sr[B][mb][0]);
        am[mb] = ah[mb];
        al[mb] = ah[mb];
      } else if constexpr (PRE) {
        ah[mb] = __builtin_bit_cast(u32x4, sr[B][mb][0]);
        am[mb] = __builtin_bit_cast(u32x4, sr[B][mb][1]);
        al[mb] = am[mb];  // unused by the SP = 2 products
      } else {
        split8(sr[B][mb][0], sr[B][mb][1], ah[mb], am[mb], al[mb]);
      }
    }
    const u32x4* qs = reinterpret_cast<const u32x4*>(qlds + (int)(g % NS) * SLOT) + lane;
    if constexpr (HALF) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const u32x4 bh = qs[j * 64];
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(ah[mb], bh, acc[mb][j]);
      }
    } else
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const u32x4 bh = qs[(j * NP + 0) * 64], bm = qs[(j * NP + 1) * 64];
      const u32x4 bl = qs[(j * NP + NP - 1) * 64];
      sweep_products<MB, NP, PRE ? 2 : 3>(acc, j, ah, am, al, bh, bm, bl);
    }
    // Refill D groups ahead (clamped: the tail re-loads the last group into its
    // own slot, which holds the same bytes, so no reader sees a change).
    const int64_t pf = g + D < c1 ? g + D : c1 - 1;
    load(B, pf);
    __builtin_amdgcn_sched_barrier(0);
  };

  if (c0 < c1) {
#pragma unroll
    for (int b = 0; b < D; ++b) load(b, c0 + b < c1 ? c0 + b : c1 - 1);
    __builtin_amdgcn_sched_barrier(0);
    // D bodies per trip (register set B takes groups c0 + B mod D), then the
    // fewer than D groups left
    int64_t g = c0;
    for (; g + D <= c1; g += D) UnrollBodies<0, D>::run(body, g, c1, false);
    UnrollBodies<0, D - 1>::run(body, g, c1, true);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the block's LDS

  constexpr int P = 16 * NB;
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
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

// Slabs summed in slice order (deterministic), four columns per thread (p % 16
// == 0; Y 16-byte aligned with ldy % 4 == 0, else one column per thread).
template <int V>
__global__ __launch_bounds__(256) void sweep_reduce_kernel(const float* __restrict__ part, int ks,
                                                           int64_t d, int p, float alpha,
                                                           float* __restrict__ Y, int64_t ldy, int per,
                                                           const SweepBatch sb) {
  using fv = std::conditional_t<V == 1, float, f32x4>;
  const int prob = blockIdx.x / per, bid = blockIdx.x - prob * per;
  if (prob) {
    part = reinterpret_cast<const float*>(reinterpret_cast<const char*>(part) + sb.off[prob]);
    Y = reinterpret_cast<float*>(reinterpret_cast<char*>(Y) + sb.off[prob]);
  }
  const int64_t idx = ((int64_t)bid * 256 + threadIdx.x) * V;
  if (idx >= d * p) return;
  const int64_t m = idx / p;
  const int n = (int)(idx - m * p);
  fv s = *reinterpret_cast<const fv*>(part + idx);
#pragma unroll 8
  for (int k = 1; k < ks; ++k) s += *reinterpret_cast<const fv*>(part + (int64_t)k * d * p + idx);
  *reinterpret_cast<fv*>(Y + m * ldy + n) = alpha * s;
}

// Split-K reduction of one sweep fused with the solver's basis step and the next
// sweep's Q image: replaces sweep_reduce_kernel + rr_power_kernel / cheb_step_kernel
// + split_q_kernel (three launches and their kernel boundaries per sweep).  One
// block per 8-row octet of the image (4 per k-group), 2p threads (rounded up to
// whole waves).  Phase 1 (row-major, one float4 of columns per thread, all ks slab
// loads issued together): Y = alpha sum_s part_s in slab order (ks == 1: Y as the
// sweep wrote it), the step, the new basis rounded to h + m when the next sweep
// takes two pieces (as split_q_kernel<2> rounds it), staged in LDS; phase 2
// (split_q_kernel's mapping, p threads): the octet's image units.
template <int NP>
__global__ __launch_bounds__(256) void sweep_finish_kernel(const float* __restrict__ part, int ks,
                                                           int64_t d, int p, float alpha,
                                                           float* __restrict__ Y, int64_t ldy,
                                                           SweepStep st, int nb,
                                                           u32x4* __restrict__ QS, int per,
                                                           const SweepBatch sb) {
  __shared__ float qt[8][132];
  const int prob = blockIdx.x / per, bid = blockIdx.x - prob * per;
  if (prob) {
    const int64_t po = sb.off[prob];
    part = reinterpret_cast<const float*>(reinterpret_cast<const char*>(part) + po);
    Y = reinterpret_cast<float*>(reinterpret_cast<char*>(Y) + po);
    QS = reinterpret_cast<u32x4*>(reinterpret_cast<char*>(QS) + po);
    st.Q = reinterpret_cast<float*>(reinterpret_cast<char*>(st.Q) + po);
    st.T = reinterpret_cast<float*>(reinterpret_cast<char*>(st.T) + po);
    st.cs = reinterpret_cast<const float*>(reinterpret_cast<const char*>(st.cs) + po);
    st.lam = reinterpret_cast<const float*>(reinterpret_cast<const char*>(st.lam) + po);
  }
  if (sb.n > 1) {  // this problem's own step constants
    st.kind = sb.kind[prob];
    st.tau = sb.tau[prob];
    st.thr = sb.thr[prob];
    st.a = sb.a[prob];
    st.cc = sb.cc[prob];
    st.gamma = sb.gamma[prob];
  }
  const int64_t g = bid >> 2;
  const int o = bid & 3;
  const int pq = p >> 2;
  const int u = threadIdx.x;
  if (u < 8 * pq) {
    const int rr = u / pq, c4 = (u - rr * pq) * 4;
    const int64_t r = 32 * g + 8 * o + rr;
    f32x4 qn = {0.f, 0.f, 0.f, 0.f};
    if (r < d) {
      f32x4 y;
      if (ks > 1) {
        const float* pp = part + r * p + c4;
        const int64_t sd = d * p;
        f32x4 v[8];
        y = *reinterpret_cast<const f32x4*>(pp);
        for (int k0 = 1; k0 < ks; k0 += 8) {  // loads of a group issued together
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (k0 + k < ks) v[k] = *reinterpret_cast<const f32x4*>(pp + (k0 + k) * sd);
#pragma unroll
          for (int k = 0; k < 8; ++k)  // fixed order: deterministic
            if (k0 + k < ks) y += v[k];
        }
        y *= alpha;
#ifdef DEIG_AB_SWEEP_ALWAYS_Y
        st.write_y = 1;  // measurement builds: the r05 behaviour (every sweep stores Y)
#endif
        if (st.write_y) *reinterpret_cast<f32x4*>(Y + r * ldy + c4) = y;
      } else {
        y = *reinterpret_cast<const f32x4*>(Y + r * ldy + c4);
      }
      f32x4* qp = reinterpret_cast<f32x4*>(st.Q + r * st.ldq + c4);
      const f32x4 q = *qp;
      qn = q;
      if (st.kind == 1) {
        const float l0 = fabsf(st.lam[0]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float c = st.cs[c4 + e];
          if (c > 0.f && fabsf(st.lam[c4 + e]) >= st.tau * l0) qn[e] = y[e] * c;
        }
      } else {
        f32x4* tp = reinterpret_cast<f32x4*>(st.T + r * p + c4);
        // degree 1 (gamma == 0) must not read T: uninitialised workspace then
        const f32x4 t = st.gamma != 0.f ? *tp : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (st.lam[c4 + e] >= st.thr) qn[e] = st.a * (y[e] - st.cc * q[e]) - st.gamma * t[e];
        *tp = q;
      }
      if (NP == 2) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const uint32_t h = cvt2(qn[2 * e], qn[2 * e + 1]);
          const uint32_t m = cvt2(qn[2 * e] - lo_f(h), qn[2 * e + 1] - hi_f(h));
          qn[2 * e] = lo_f(h) + lo_f(m);
          qn[2 * e + 1] = hi_f(h) + hi_f(m);
        }
      }
      *qp = qn;
    }
    *reinterpret_cast<f32x4*>(&qt[rr][c4]) = qn;
  }
  __syncthreads();
  if (u < p) {
    const int j = u >> 4, n = u;
    const f32x4 a = {qt[0][n], qt[1][n], qt[2][n], qt[3][n]};
    const f32x4 b = {qt[4][n], qt[5][n], qt[6][n], qt[7][n]};
    u32x4 hi, mi, lo;
    split8(a, b, hi, mi, lo);
    const int64_t tt = g * nb + j;
    const int lane = 16 * o + (u & 15);
    QS[(tt * NP + 0) * 64 + lane] = hi;
    QS[(tt * NP + 1) * 64 + lane] = mi;
    if constexpr (NP == 3) QS[(tt * NP + 2) * 64 + lane] = lo;
  }
}

// Split-K slices: about one block per CU, >= 4 K-steps per slice (r01g: two
// blocks per CU and finer slices measured slower).
int sweep_ks(int64_t d) {
  const int64_t bx = cdiv(d, SI_BR), nsteps = cdiv(d, SW_KS);
  int64_t ks = cdiv((int64_t)num_cus(), bx);
  const int64_t cap = nsteps / 4 > 1 ? nsteps / 4 : 1;
  if (ks > cap) ks = cap;
  if (ks < 1) ks = 1;
  return (int)ks;
}

// m-blocks per wave of the v3 kernel: 2 for the early-sweep mode up to p = 80
// (128-row blocks: half the split-K slices, so half the slab bytes the sweep writes
// and its epilogue reads; rocprof d = 8192: p = 80 47.2 vs 50.6 us, p = 64 45.4 vs
// 47.9, per sweep in the chain 52.4 vs 58.0), else 4 (p = 128: 272 vs 249 us per
// sweep - there the Q fragment reuse of 64-row waves wins; with the split in the
// sweep no gain either).  Ring depths 5-8 measured the same as 3
// (profiles/r02n_sweep_mb.log), so the ring is 3 deep.
int sweep_mb(bool pre, int nb) { return (pre && nb <= 5) ? 2 : 4; }
#ifdef DEIG_AB_SWEEP_DEPTH
constexpr int kSweepDepth = DEIG_AB_SWEEP_DEPTH;
#else
constexpr int kSweepDepth = 3;
#endif
#ifdef DEIG_AB_SWEEP_HALF_DEPTH
constexpr int kSweepDepthHalf = DEIG_AB_SWEEP_HALF_DEPTH;
#else
constexpr int kSweepDepthHalf = 3;
#endif

// Split-K slices of a v3 launch with mb m-blocks per wave (rows per block 64 mb).
int sweep_ks_mb(int64_t d, int mb) {
  if (mb == 4) return sweep_ks(d);
  const int64_t bx = cdiv(d, 64 * mb), nsteps = cdiv(d, SW_KS);
  int64_t ks = cdiv((int64_t)num_cus(), bx);
  const int64_t cap = nsteps / 4 > 1 ? nsteps / 4 : 1;
  if (ks > cap) ks = cap;
  if (ks < 1) ks = 1;
  const int64_t kmax = sweep_ks(d);  // the workspace holds sweep_ks(d) slabs
  return (int)(ks < kmax ? ks : kmax);
}

// Q image: 3 bf16 pieces per value
size_t qs_bytes(int64_t d, int p) { return (size_t)cdiv(d, SW_KS) * SW_KS * p * 6; }

// One launch: sb.n problems of `per` blocks each.
struct Grid {
  int per;
  const SweepBatch* sb;
  dim3 dim() const { return dim3((unsigned)(per * sb->n)); }
};

template <int NB, int NP, bool PRE>
void launch_v2(Grid g, hipStream_t st, const f32x4* SI, int64_t d, const u32x4* QS, float* Y,
               int64_t ldy, float alpha, float* part) {
  const int64_t ng = si_groups(d);
  hipLaunchKernelGGL((sweep2_kernel<NB, NP, 0, PRE>), g.dim(), dim3(256), 0, st, SI, d, QS, ng, Y,
                     ldy, alpha, part, g.per, *g.sb);
}

template <int NB, int NP, bool PRE, bool HALF = false>
void launch_v3(Grid g, hipStream_t st, const f32x4* SI, int64_t d, const u32x4* QS, float* Y,
               int64_t ldy, float alpha, float* part) {
  const int64_t ng = si_groups(d);
  constexpr int D = HALF ? kSweepDepthHalf : kSweepDepth;
  if (sweep_mb(PRE, NB) == 2)
    hipLaunchKernelGGL((sweep3_kernel<NB, NP, D, 1, PRE, 2, HALF>), g.dim(), dim3(256), 0, st,
                       SI, d, QS, ng, Y, ldy, alpha, part, g.per, *g.sb);
  else
    hipLaunchKernelGGL((sweep3_kernel<NB, NP, D, 1, PRE, 4, HALF>), g.dim(), dim3(256), 0, st,
                       SI, d, QS, ng, Y, ldy, alpha, part, g.per, *g.sb);
}

// The one-piece mode (v3 only, p >= 64: nb 4 .. 8).
void launch_half(int nb, Grid grid, hipStream_t st, const f32x4* SI, int64_t d, const u32x4* QS,
                 float* Y, int64_t ldy, float alpha, float* part) {
  switch (nb) {
    case 4: launch_v3<4, 2, true, true>(grid, st, SI, d, QS, Y, ldy, alpha, part); return;
    case 5: launch_v3<5, 2, true, true>(grid, st, SI, d, QS, Y, ldy, alpha, part); return;
    case 6: launch_v3<6, 2, true, true>(grid, st, SI, d, QS, Y, ldy, alpha, part); return;
    case 7: launch_v3<7, 2, true, true>(grid, st, SI, d, QS, Y, ldy, alpha, part); return;
    default: launch_v3<8, 2, true, true>(grid, st, SI, d, QS, Y, ldy, alpha, part); return;
  }
}

// v2 (sweep3 = false) or v3 with NP Q pieces, NB = p / 16 column blocks; PRE: the
// two-piece S image (three products).
template <int NP, bool PRE = false>
void launch_image(bool v3, int nb, Grid grid, hipStream_t st, const f32x4* SI, int64_t d,
                  const u32x4* QS, float* Y, int64_t ldy, float alpha, float* part) {
#define DEIG_NB_CASE(N_)                                                   \
  case N_:                                                                 \
    if (v3)                                                                \
      launch_v3<N_, NP, PRE>(grid, st, SI, d, QS, Y, ldy, alpha, part);    \
    else                                                                   \
      launch_v2<N_, NP, PRE>(grid, st, SI, d, QS, Y, ldy, alpha, part);    \
    return;
  switch (nb) {
    DEIG_NB_CASE(1) DEIG_NB_CASE(2) DEIG_NB_CASE(3) DEIG_NB_CASE(4)
    DEIG_NB_CASE(5) DEIG_NB_CASE(6) DEIG_NB_CASE(7)
    default: DEIG_NB_CASE(8)
  }
#undef DEIG_NB_CASE
}

// Workspace: [Q image][split-K slabs][S image][two-piece S image].
struct SweepWs {
  u32x4* QS;
  float* part;
  f32x4* SI;
  u32x4* SH;
  size_t total;
};
SweepWs sweep_carve(void* ws, int64_t d, int p) {
  SweepWs w;
  char* base = static_cast<char*>(ws);
  size_t off = 0;
  w.QS = reinterpret_cast<u32x4*>(base + off);
  off = align_up(off + qs_bytes(d, p), 256);
  w.part = reinterpret_cast<float*>(base + off);
  const int ks = sweep_ks(d);
  if (ks > 1) off = align_up(off + (size_t)ks * d * p * sizeof(float), 256);
  w.SI = reinterpret_cast<f32x4*>(base + off);
  off += si_bytes(d);
  w.SH = reinterpret_cast<u32x4*>(base + off);
  off += si_bytes(d);
  w.total = off;
  return w;
}

// Q pieces in round_q mode (the dropped piece of Q: split_q_kernel<2>).
constexpr int kRoundPieces = 2;

}  // namespace

size_t sweep_workspace_bytes(int64_t d, int p) { return sweep_carve(nullptr, d, p).total; }

int sweep_prepare(const void* S, int stype, int64_t d, int64_t lds, int p, void* ws,
                  size_t ws_bytes, hipStream_t st, const float* Vd, int64_t ldv, const float* lamd,
                  int r, double shift) {
  DEIG_REQUIRE(r == 0 || (Vd && lamd && ldv >= d), "sweep: bad deflation arguments (r=%d)", r);
  DEIG_REQUIRE(stype == DEIG_F32 || stype == DEIG_F64, "sweep: unknown element type %d", stype);
  DEIG_REQUIRE(d >= 1 && lds >= d && lds % 4 == 0 && S && aligned16(S),
               "sweep: S must be 16-byte aligned with lds >= d, lds %% 4 == 0");
  const SweepWs w = sweep_carve(ws, d, p);
  if (!ws || ws_bytes < w.total)
    return fail(DEIG_EWORKSPACE, "sweep: workspace %zu < %zu", ws_bytes, w.total);
  const int64_t ng = si_groups(d);
  const int64_t nunits = si_rows(d) / SI_RB * ng * 4 * 64;
  const dim3 grid((unsigned)cdiv(nunits, 256));
  if (stype == DEIG_F64)
    hipLaunchKernelGGL(sweep_prepare_kernel<double>, grid, dim3(256), 0, st,
                       static_cast<const double*>(S), lds, d, ng, nunits, w.SI, w.SH, Vd, ldv,
                       lamd, r, shift);
  else
    hipLaunchKernelGGL(sweep_prepare_kernel<float>, grid, dim3(256), 0, st,
                       static_cast<const float*>(S), lds, d, ng, nunits, w.SI, w.SH, Vd, ldv,
                       lamd, r, shift);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

int sweep_apply(const float* Q, int64_t d, int p, int64_t ldq, float* Y, int64_t ldy, float alpha,
                void* ws, size_t ws_bytes, hipStream_t st, int mode, const SweepStep* step,
                bool q_ready, bool kernel_only, const SweepBatch* batch) {
  SweepBatch one{};
  one.n = 1;
  const SweepBatch* sb = batch ? batch : &one;
  DEIG_REQUIRE(sb->n >= 1 && sb->n <= kMaxSweepBatch && sb->off[0] == 0,
               "sweep: batch of %d problems (1..%d, off[0] = 0)", sb->n, kMaxSweepBatch);
  const bool round_q = mode >= 1;
  DEIG_REQUIRE(d >= 1 && p >= 16 && p <= 128 && p % 16 == 0,
               "sweep: need d >= 1 and p in {16, 32, ..., 128} (p=%d)", p);
  DEIG_REQUIRE(ldq >= p && ldy >= p, "sweep: bad leading dims");
  DEIG_REQUIRE(Q && Y, "sweep: null Q / Y");
  const SweepWs w = sweep_carve(ws, d, p);
  if (!ws || ws_bytes < w.total)
    return fail(DEIG_EWORKSPACE, "sweep: workspace %zu < %zu", ws_bytes, w.total);
  const int nb = p / 16;
  const int64_t ngrp = 2 * cdiv(d, SW_KS);
  const int np = round_q ? kRoundPieces : 3;
  // kSweepHalf (3) where the v3 kernel runs (p >= 64), else the two-piece mode
  const bool half = mode == kSweepHalf && nb >= 4;
  const bool pre = (mode == kSweepFast || mode == kSweepHalf) && np == 2;
  const dim3 qgrid((unsigned)cdiv(ngrp * nb * 64, 256));
  // q_ready: the previous sweep's finish kernel already wrote this Q's image
  if (!q_ready) {
    if (np == 2)
      hipLaunchKernelGGL(split_q_kernel<2>, dim3(qgrid.x * sb->n), dim3(256), 0, st,
                         const_cast<float*>(Q), ldq, d, nb, ngrp, w.QS, (int)qgrid.x, *sb);
    else
      hipLaunchKernelGGL(split_q_kernel<3>, dim3(qgrid.x * sb->n), dim3(256), 0, st,
                         const_cast<float*>(Q), ldq, d, nb, ngrp, w.QS, (int)qgrid.x, *sb);
    DEIG_HIP_CHECK(hipGetLastError());
  }
  // v3 (LDS-shared Q ring): above p = 80 (v2's register rings spill) and for the
  // early-sweep mode from p = 64 (no split in the sweep, so the shared Q pays;
  // rocprof, d = 8192: p = 80 50.6 vs 55.3 us, p = 64 47.2 vs 48.3; p = 32 at
  // d = 3072 11.4 vs 11.0, profiles/r02l_sweep_v3pre.log; v2 stays faster with the
  // split in the sweep)
  const bool v3 = nb > 5 || (pre && nb >= 4);
  const int mbw = v3 ? sweep_mb(pre, nb) : 4;
  const int64_t bx = cdiv(d, mbw == 4 ? SI_BR : 64 * mbw);
  // a batch keeps the single problem's slicing: bit-identical to separate solves (and
  // fewer slices for a batch that fills the chip measured no faster: c1 7.85 vs 7.85,
  // c1g 14.9 vs 15.3 M samples/s, profiles/r04f_bench_*)
  const int ks = sweep_ks_mb(d, mbw);
  const Grid grid{(int)(bx * ks), sb};
  if (half)
    launch_half(nb, grid, st, reinterpret_cast<const f32x4*>(w.SH), d, w.QS, Y, ldy, alpha, w.part);
  else if (pre)
    launch_image<2, true>(v3, nb, grid, st, reinterpret_cast<const f32x4*>(w.SH), d, w.QS, Y, ldy,
                          alpha, w.part);
  else if (np == 2)
    launch_image<2>(v3, nb, grid, st, w.SI, d, w.QS, Y, ldy, alpha, w.part);
  else
    launch_image<3>(v3, nb, grid, st, w.SI, d, w.QS, Y, ldy, alpha, w.part);
  DEIG_HIP_CHECK(hipGetLastError());
  if (kernel_only) return DEIG_OK;
  if (step) {
    DEIG_REQUIRE(ldy % 4 == 0 && aligned16(Y) && step->ldq % 4 == 0 && aligned16(step->Q) &&
                     (step->kind == 1 || step->kind == 2),
                 "sweep: fused step needs 16-byte aligned Y / Q rows");
    const int nnp = step->next_mode >= kSweepRoundQ ? kRoundPieces : 3;
    const float* pp = ks > 1 ? w.part : nullptr;
    const int fper = (int)(4 * ngrp);
    const dim3 fgrid((unsigned)(fper * sb->n)), fblk((unsigned)((2 * p + 63) / 64 * 64));
    if (nnp == 2)
      hipLaunchKernelGGL(sweep_finish_kernel<2>, fgrid, fblk, 0, st, pp, ks, d, p, alpha, Y, ldy,
                         *step, nb, w.QS, fper, *sb);
    else
      hipLaunchKernelGGL(sweep_finish_kernel<3>, fgrid, fblk, 0, st, pp, ks, d, p, alpha, Y, ldy,
                         *step, nb, w.QS, fper, *sb);
    DEIG_HIP_CHECK(hipGetLastError());
    return DEIG_OK;
  }
  if (ks > 1) {
    if (ldy % 4 == 0 && aligned16(Y)) {
      const int rper = (int)cdiv(d * p / 4, 256);
      hipLaunchKernelGGL(sweep_reduce_kernel<4>, dim3((unsigned)(rper * sb->n)), dim3(256), 0, st,
                         w.part, ks, d, p, alpha, Y, ldy, rper, *sb);
    } else {
      const int rper = (int)cdiv(d * p, 256);
      hipLaunchKernelGGL(sweep_reduce_kernel<1>, dim3((unsigned)(rper * sb->n)), dim3(256), 0, st,
                         w.part, ks, d, p, alpha, Y, ldy, rper, *sb);
    }
    DEIG_HIP_CHECK(hipGetLastError());
  }
  return DEIG_OK;
}

}  // namespace deig
