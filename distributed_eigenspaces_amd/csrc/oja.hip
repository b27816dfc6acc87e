// Mini-batch Oja steps for the online / streaming variant (BASELINE.json config 4):
//   V <- orth(V + eta/b * Xb^T (Xb V)),   orth = Cholesky-QR2.
// Not present in the reference (parity unpinned; judged by sin(theta) against
// the one-shot float64 oracle and ref_cpu.oja_epoch).  Two paths, bf16x3 split
// products in both: the two-pass v3 (any shape) reads Xb twice (Xb V and Xb^T T),
// two launches per batch (oja_nn_kernel, oja_tn_kernel), K split over the waves of a
// block and summed in LDS (no slab passes), each pass writing the next one's MFMA
// operand image (T's for TN, V's for the next batch's NN); the resident v4
// (oja_blk_kernel, config 4's shape) runs a whole run of batches in one launch with
// each workgroup's block of Xb held in registers - Xb read once per batch.
#include <algorithm>

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

// (*err set: a v4 hand-off timed out - the basis is poisoned with NaN, never returned
// silently wrong)
__global__ __launch_bounds__(256) void rowpad_to_col(const float* __restrict__ Vr, int64_t d,
                                                     int k, int kp, float* __restrict__ V,
                                                     int64_t ldv, const unsigned* __restrict__ err) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * k) return;
  const int j = (int)(idx / d);
  const int64_t r = idx - (int64_t)j * d;
  V[r + (int64_t)j * ldv] = *err ? __builtin_nanf("") : Vr[r * kp + j];
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

template <int KP, bool INV = true>
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
    // one v_rsq_f32 (1 ulp) instead of the correctly rounded sqrt and division
    // sequences: this single wave's latency chain is its cost
    dinv[j] = __builtin_amdgcn_rsqf(v);
    const float ljj = v * dinv[j];
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
  if constexpr (!INV) {  // L itself (kp x kp, identity-padded beyond k) for trsm_img_kernel
    if (r < kp)
#pragma unroll
      for (int c = 0; c < KP; ++c)
        if (c < kp) Rinv[r * kp + c] = a[c];
    return;
  }
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


// ---------------------------------------------------------------- v3 passes
// bf16 operands for the split products of the NN pass (as the covariance and the
// sweeps: x = hi + lo, three bf16 MFMA products hi hi + hi lo + lo hi per fp32
// product, exact products summed in fp32: ~2^-16 relative).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t cvt2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
__device__ __forceinline__ float lo_f(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float hi_f(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }

// 8 fp32 -> (hi, lo) bf16x8 pairs.
__device__ __forceinline__ void split8(const f32x4& a, const f32x4& b, bf16x8& hi, bf16x8& lo) {
  const float x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  u32x4 h, l;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const uint32_t hh = cvt2(x[2 * p], x[2 * p + 1]);
    h[p] = hh;
    l[p] = cvt2(x[2 * p] - lo_f(hh), x[2 * p + 1] - hi_f(hh));
  }
  hi = __builtin_bit_cast(bf16x8, h);
  lo = __builtin_bit_cast(bf16x8, l);
}

// The MFMA B-operand image of a row-padded d x kp matrix M (row stride kp): for
// k-step ks (rows 32 ks ..), column block nb and piece h (hi, lo), lane l holds
// M[32 ks + 8 (l >> 4) + 0..7][16 nb + (l & 15)] as 8 bf16 - 16 B, one 1-KiB
// load per wave and fragment.  Rows >= rows are zeros.
__device__ __forceinline__ int64_t img_index(int ks, int nb, int h, int lane, int NB) {
  return (((int64_t)ks * NB + nb) * 2 + h) * 64 + lane;
}

__global__ __launch_bounds__(256) void img_kernel(const float* __restrict__ M, int64_t rows, int kp,
                                                  int nks, u32x4* __restrict__ img) {
  const int NB = kp / 16;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (ks, nb, lane)
  if (idx >= (int64_t)nks * NB * 64) return;
  const int lane = (int)(idx & 63);
  const int64_t q = idx >> 6;
  const int nb = (int)(q % NB), ks = (int)(q / NB);
  const int64_t r0 = 32 * (int64_t)ks + 8 * (lane >> 4);
  const int col = 16 * nb + (lane & 15);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = r0 + j < rows ? M[(r0 + j) * kp + col] : 0.f;
  bf16x8 hi, lo;
  split8(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, hi, lo);
  img[img_index(ks, nb, 0, lane, NB)] = __builtin_bit_cast(u32x4, hi);
  img[img_index(ks, nb, 1, lane, NB)] = __builtin_bit_cast(u32x4, lo);
}

// V_out = V_in L^-T (the CholQR apply as a triangular solve: y L^T = v per row,
// L from chol_rinv_kernel<KP, false>) and, with img != nullptr, V_out's NN operand
// image (img_kernel's layout, fused).  One block per 32 rows (one image k-step); 8
// lanes per row split each step's dot product (lane s takes the terms t = s mod 8) and
// meet by xor shuffles, so every lane of the row knows y_i.  r04: replaces the
// explicit inverse, the apply skinny pass and img_kernel.
template <int KP>
__global__ __launch_bounds__(256) void trsm_img_kernel(const float* __restrict__ Vin, const float* __restrict__ L,
                                                       int64_t d, int kp, float* __restrict__ Vout,
                                                       u32x4* __restrict__ img) {
  __shared__ float Ls[KP][KP + 1];
  __shared__ float dv[KP];
  __shared__ float Ys[32][KP + 1];
  const int t = threadIdx.x, rr = t >> 3, sub = t & 7;
  const int64_t r0 = (int64_t)blockIdx.x * 32, row = r0 + rr;
  for (int u = t; u < KP * KP; u += 256) {
    const int i = u / KP, c = u - i * KP;
    Ls[i][c] = (i < kp && c < kp) ? L[i * kp + c] : (i == c ? 1.f : 0.f);
  }
  for (int u = t; u < 32 * KP; u += 256) {
    const int i = u / KP, c = u - i * KP;
    const int64_t rw = r0 + i;
    Ys[i][c] = (rw < d && c < kp) ? Vin[rw * kp + c] : 0.f;
  }
  __syncthreads();
  if (t < KP) dv[t] = 1.0f / Ls[t][t];
  __syncthreads();
  float y[KP / 8];
#pragma unroll
  for (int tt = 0; tt < KP / 8; ++tt) y[tt] = 0.f;
#pragma unroll
  for (int i = 0; i < KP; ++i) {
    float part = 0.f;
#pragma unroll
    for (int tt = 0; tt < (i + 7) / 8; ++tt)
      if (8 * tt + sub < i) part = fmaf(Ls[i][8 * tt + sub], y[tt], part);
    part += __shfl_xor(part, 1, 64);
    part += __shfl_xor(part, 2, 64);
    part += __shfl_xor(part, 4, 64);
    const float yi = (Ys[rr][i] - part) * dv[i];
    if ((i & 7) == sub) y[i / 8] = yi;
  }
  __syncthreads();  // every lane's reads of Ys are done
#pragma unroll
  for (int tt = 0; tt < KP / 8; ++tt) {
    const int c = 8 * tt + sub;
    Ys[rr][c] = y[tt];
    if (row < d && c < kp) Vout[row * kp + c] = y[tt];
  }
  if (!img) return;
  __syncthreads();
  const int NB = kp / 16;
  if (t < NB * 64) {  // image entries of k-step blockIdx.x: rows 8 (ln >> 4) .., column 16 nb + (ln & 15)
    const int ln = t & 63, nb = t >> 6;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = Ys[8 * (ln >> 4) + j][16 * nb + (ln & 15)];
    bf16x8 hi, lo;
    split8(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, hi, lo);
    img[img_index(blockIdx.x, nb, 0, ln, NB)] = __builtin_bit_cast(u32x4, hi);
    img[img_index(blockIdx.x, nb, 1, ln, NB)] = __builtin_bit_cast(u32x4, lo);
  }
}

// Measurement builds only (tools/ab.py build; the shipped library is variant 0):
// -DDEIG_AB_OJA_VARIANT=N knocks parts out of the NN (N % 8) / TN ((N / 8) % 8)
// passes - 1: no X loads, 2: no operand-image loads, 4: no MFMAs - and picks the
// prefetch depth ((N / 64) % 4: 4, 2, 6, 8 k-steps); (N / 256) % 2 = 1: the TN
// pass without its XCD-aware block order.
#ifdef DEIG_AB_OJA_VARIANT
constexpr int kOjaAB = DEIG_AB_OJA_VARIANT;
#else
constexpr int kOjaAB = 0;
#endif
constexpr int kOjaPF = ((kOjaAB / 64) % 4) == 0 ? 4 : ((kOjaAB / 64) % 4) == 1 ? 2 : ((kOjaAB / 64) % 4) == 2 ? 6 : 8;

// NN: T = Xb V (b x kp), written as the TN pass's B-operand image (img_kernel's
// layout; an 8-row group never straddles two blocks).  One 512-thread block per 16 rows of Xb,
// its 8 waves split K (= d) into 8 slices and their 16 x kp partial tiles are summed
// in LDS in wave order (deterministic, no slab pass).  A operand straight from HBM:
// lane l holds row r0 + (l & 15), features 32 ks + 8 (l >> 4) .. + 7 (two float4
// loads; the 16 rows x 128 B of a wave-instruction pair are whole lines), split to
// hi / lo in registers; B from the V image (img_kernel), L2-resident.  Loads run
// PF k-steps ahead of the MFMAs (register ring).
template <int NB, int KO = kOjaAB % 8>
__global__ __launch_bounds__(512) void oja_nn_kernel(const float* __restrict__ X, int64_t ldx, int64_t b,
                                                     int d, int nks, const u32x4* __restrict__ vimg,
                                                     u32x4* __restrict__ timg) {
  constexpr int PF = kOjaPF;
  constexpr int KP = 16 * NB;
  __shared__ f32x4 red[8][NB][64];
  __shared__ float tt[16][KP + 1];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t r0 = (int64_t)blockIdx.x * 16;
  const int64_t row = r0 + (lane & 15);
  // loads are never predicated (the compiler's counted waits stay deep): rows >= b
  // and features >= d read clamped in-range addresses; the V image is zero past d
  // and rows >= b are zeroed below
  const float* xr = X + (row < b ? row : b - 1) * ldx;
  const int NKS = nks;
  const int per = (nks + 7) / 8;
  const int ks0 = wave * per, ks1 = min(nks, ks0 + per);
  f32x4 acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 xa[PF], xb[PF];
  u32x4 bh[PF][NB], bl[PF][NB];
  auto load = [&](int ks, int slot) {
    const int k = 32 * ks + 8 * (lane >> 4);
    if constexpr (KO & 1) {
      xa[slot] = f32x4{(float)k, 1.f, 2.f, 3.f};
      xb[slot] = f32x4{(float)ks, 1.f, 2.f, 3.f};
    } else {
      xa[slot] = *reinterpret_cast<const f32x4*>(xr + min(k, d - 4));
      xb[slot] = *reinterpret_cast<const f32x4*>(xr + min(k + 4, d - 4));
    }
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      if constexpr (KO & 2) {
        bh[slot][nb] = u32x4{(unsigned)ks, 1u, 2u, (unsigned)lane};
        bl[slot][nb] = u32x4{(unsigned)k, 1u, 2u, (unsigned)lane};
      } else {
        bh[slot][nb] = vimg[img_index(ks, nb, 0, lane, NB)];
        bl[slot][nb] = vimg[img_index(ks, nb, 1, lane, NB)];
      }
    }
  };
  auto step = [&](int u) {
    bf16x8 ahi, alo;
    split8(xa[u], xb[u], ahi, alo);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      if constexpr (KO & 4) {  // keep the operands live without the MFMAs
        const u32x4 a = __builtin_bit_cast(u32x4, ahi) ^ __builtin_bit_cast(u32x4, alo);
        const u32x4 q = a ^ bh[u][nb] ^ bl[u][nb];
        acc[nb] += __builtin_bit_cast(f32x4, q & u32x4{0x3f800000u, 0x3f800000u, 0x3f800000u, 0x3f800000u});
      } else {
        const bf16x8 bhi = __builtin_bit_cast(bf16x8, bh[u][nb]);
        const bf16x8 blo = __builtin_bit_cast(bf16x8, bl[u][nb]);
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bhi, acc[nb], 0, 0, 0);
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, blo, acc[nb], 0, 0, 0);
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bhi, acc[nb], 0, 0, 0);
      }
    }
  };
#pragma unroll
  for (int u = 0; u < PF; ++u) load(min(ks0 + u, NKS - 1), u);  // unconditional, in range
  // steady state without conditions (so that the compiler's counted waits keep PF
  // k-steps of loads in flight), then the guarded tail
  int ks = ks0;
  for (; ks + 2 * PF <= ks1; ks += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      step(u);
      load(ks + u + PF, u);
    }
  }
  for (; ks < ks1; ks += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      if (ks + u < ks1) {
        step(u);
        if (ks + u + PF < ks1) load(ks + u + PF, u);
      }
    }
  }
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) red[wave][nb][lane] = acc[nb];
  __syncthreads();
  const int t = threadIdx.x;
  if (t < NB * 64) {
    const int nb = t >> 6, ln = t & 63;
    f32x4 sum = red[0][nb][ln];
#pragma unroll
    for (int w = 1; w < 8; ++w) sum += red[w][nb][ln];
    // C/D map of 16x16: row 4 (lane >> 4) + reg, column lane & 15
#pragma unroll
    for (int i = 0; i < 4; ++i)
      tt[4 * (ln >> 4) + i][16 * nb + (ln & 15)] = r0 + 4 * (ln >> 4) + i < b ? sum[i] : 0.f;
  }
  __syncthreads();
  if (t < 2 * KP) {  // image entries of these 16 rows: k-step r0 / 32, groups (r0 % 32) / 8 + gi
    const int gi = t / KP, col = t % KP;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = tt[8 * gi + j][col];
    bf16x8 hi, lo;
    split8(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, hi, lo);
    const int ln = (col & 15) + 16 * ((int)(r0 & 31) / 8 + gi);
    timg[img_index((int)(r0 / 32), col / 16, 0, ln, NB)] = __builtin_bit_cast(u32x4, hi);
    timg[img_index((int)(r0 / 32), col / 16, 1, ln, NB)] = __builtin_bit_cast(u32x4, lo);
  }
}

// TN: V += c Xb^T T (V row-padded d x kp, updated in place) and the next NN's V
// image.  One 512-thread block per 16 features; its 8 waves split the b rows and
// their 16 x kp partials are summed in LDS in wave order (no slab pass).  The A
// operand (Xb^T) needs 8 consecutive ROWS of one feature per lane: the wave loads
// 32 rows x 16 features with float4 loads (whole 64-B row segments) and transposes
// them through its own LDS region ([feature][row], TS floats a row); B is the T
// image (img_kernel).  An 8-feature group of the V image never straddles two
// blocks (16 | 32), so each block writes its own image entries.
template <int NB, int KO = (kOjaAB / 8) % 8>
__global__ __launch_bounds__(512) void oja_tn_kernel(const float* __restrict__ X, int64_t ldx, int64_t b,
                                                     int d, int nkr, const u32x4* __restrict__ timg,
                                                     float c, float* __restrict__ V,
                                                     u32x4* __restrict__ vimg) {
  constexpr int TS = 36;
  constexpr int KP = 16 * NB;
  __shared__ __attribute__((aligned(16))) float tr[8][16 * TS];
  __shared__ f32x4 red[8][NB][64];
  __shared__ float vt[16][KP + 1];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware: the two blocks of a 32-feature (128-B) row segment run on one XCD
  // and share its L2 line (round-robin dispatch would split every pair over two)
  const int f0 = ((kOjaAB / 256) % 2 ? (int)blockIdx.x : xcd_logical(blockIdx.x, gridDim.x)) * 16;
  const int fl = 4 * (lane & 3);  // this lane's 4 features (load mapping)
  // unpredicated loads (see oja_nn_kernel): features >= d and rows >= b read clamped
  // in-range addresses; their products are dropped (f >= d) or meet zero T rows
  const float* xb_ = X + min(f0 + fl, d - 4);
  const int NKS = nkr;
  const int per = (nkr + 7) / 8;
  const int ks0 = wave * per, ks1 = min(nkr, ks0 + per);
  float* T = tr[wave];
  f32x4 acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // loads run PF k-steps (32 rows each) ahead of their use (register ring): one
  // k-step in flight per wave was latency-bound (16 KiB per CU)
  constexpr int PF = kOjaPF;
  f32x4 xa[PF], xb[PF];
  u32x4 bh[PF][NB], bl[PF][NB];
  auto load = [&](int ks, int slot) {
    const int64_t r = 32 * (int64_t)ks + (lane >> 2);
    if constexpr (KO & 1) {
      xa[slot] = f32x4{(float)r, 1.f, 2.f, 3.f};
      xb[slot] = f32x4{(float)ks, 1.f, 2.f, 3.f};
    } else {
      xa[slot] = *reinterpret_cast<const f32x4*>(xb_ + min(r, b - 1) * ldx);
      xb[slot] = *reinterpret_cast<const f32x4*>(xb_ + min(r + 16, b - 1) * ldx);
    }
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      if constexpr (KO & 2) {
        bh[slot][nb] = u32x4{(unsigned)ks, 1u, 2u, (unsigned)lane};
        bl[slot][nb] = u32x4{(unsigned)r, 1u, 2u, (unsigned)lane};
      } else {
        bh[slot][nb] = timg[img_index(ks, nb, 0, lane, NB)];
        bl[slot][nb] = timg[img_index(ks, nb, 1, lane, NB)];
      }
    }
  };
  const int rr = lane >> 2;
  auto step = [&](int u) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      T[(fl + e) * TS + rr] = xa[u][e];
      T[(fl + e) * TS + rr + 16] = xb[u][e];
    }
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(T + (lane & 15) * TS + 8 * (lane >> 4));
    const f32x4 a1 = *reinterpret_cast<const f32x4*>(T + (lane & 15) * TS + 8 * (lane >> 4) + 4);
    bf16x8 ahi, alo;
    split8(a0, a1, ahi, alo);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      if constexpr (KO & 4) {  // keep the operands live without the MFMAs
        const u32x4 a = __builtin_bit_cast(u32x4, ahi) ^ __builtin_bit_cast(u32x4, alo);
        const u32x4 q = a ^ bh[u][nb] ^ bl[u][nb];
        acc[nb] += __builtin_bit_cast(f32x4, q & u32x4{0x3f800000u, 0x3f800000u, 0x3f800000u, 0x3f800000u});
      } else {
        const bf16x8 bhi = __builtin_bit_cast(bf16x8, bh[u][nb]);
        const bf16x8 blo = __builtin_bit_cast(bf16x8, bl[u][nb]);
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bhi, acc[nb], 0, 0, 0);
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, blo, acc[nb], 0, 0, 0);
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bhi, acc[nb], 0, 0, 0);
      }
    }
  };
#pragma unroll
  for (int u = 0; u < PF; ++u) load(min(ks0 + u, NKS - 1), u);  // unconditional, in range
  // steady state without conditions (the compiler's counted waits then keep PF
  // k-steps of loads in flight), then the guarded tail
  int ks = ks0;
  for (; ks + 2 * PF <= ks1; ks += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      step(u);
      load(ks + u + PF, u);
    }
  }
  for (; ks < ks1; ks += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      if (ks + u < ks1) {
        step(u);
        if (ks + u + PF < ks1) load(ks + u + PF, u);
      }
    }
  }
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) red[wave][nb][lane] = acc[nb];
  __syncthreads();
  const int t = threadIdx.x;
  if (t < NB * 64) {
    const int nb = t >> 6, ln = t & 63;
    f32x4 sum = red[0][nb][ln];
#pragma unroll
    for (int w = 1; w < 8; ++w) sum += red[w][nb][ln];
    const int col = 16 * nb + (ln & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int fr = 4 * (ln >> 4) + i;
      const int f = f0 + fr;
      float v = 0.f;
      if (f < d) {
        v = fmaf(c, sum[i], V[(int64_t)f * KP + col]);
        V[(int64_t)f * KP + col] = v;
      }
      vt[fr][col] = v;
    }
  }
  __syncthreads();
  // image entries of these 16 features: k-step f0 / 32, groups (f0 % 32) / 8 + gi
  if (t < 2 * KP) {
    const int gi = t / KP, col = t % KP;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = vt[8 * gi + j][col];
    bf16x8 hi, lo;
    split8(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, hi, lo);
    const int ln = (col & 15) + 16 * ((f0 & 31) / 8 + gi);
    vimg[img_index(f0 / 32, col / 16, 0, ln, NB)] = __builtin_bit_cast(u32x4, hi);
    vimg[img_index(f0 / 32, col / 16, 1, ln, NB)] = __builtin_bit_cast(u32x4, lo);
  }
}

// ---------------------------------------------------------------- v4: one launch
// Block-resident Oja (config 4's shape: b = 4096, d = 512 c <= 3072, kp <= 32).  One
// persistent launch runs a run of batches; 256 workgroups (one per CU, 8 waves) tile
// the batch as a 16 x 16 grid of X blocks - workgroup (i, j) owns rows
// R_i = [256 i, 256 i + 256) and features F_j = [FB j, FB j + FB), FB = d / 16 - and
// keeps its block in registers (wave w: rows 32 w .. 32 w + 31 as MFMA A fragments,
// 96 VGPRs at FB = 192), so Xb is read from HBM ONCE per batch (the two-pass v3
// reads it twice) and the next batch's block is prefetched while the basis update
// finishes.  Per batch, with V_j = V[F_j], T = Xb V:
//   1. P_ij = X_ij V_j (256 x kp; V_j's image staged in LDS), written to ppart;
//   A. row group i: all 16 P_i. partials written;
//   2. T rows R_i[16 j .. +16) = sum_j' P_ij' (fixed order), written as the TN operand
//      image (timg);
//   B. row group i: T_i complete;
//   3. Q_ij = X_ij^T T_i (FB x kp: the block transposed per wave through LDS, the
//      8 waves' row-step partials summed in LDS in wave order), written to qpart;
//   C. column group j: all 16 Q_.j partials written;
//   4. (one wave) V[F_j] slice += c sum_i' Q_i'j (fixed order) and its image entries;
//   D. column group j: V_j's image complete.
// Hand-offs (MI355X_MICROARCH.md visibility table, first row): payloads stored
// write-through (sc1) and drained (vmcnt(0), then the workgroup barrier), ONE lane adds
// to the group's counter, ONE lane polls it (relaxed agent loads), the payload is
// read with sc1 loads only.  Column group j lives on one XCD (its C / D hand-offs stay
// in that L2); row groups span all eight.  Counters start each launch at zero (the
// last block out resets them) and every
// spin is bounded (2 s): a timeout sets *err, every later wait returns at once, and
// the final copy-out poisons V with NaN - a failure is loud, never a hang.
constexpr int OB_G = 256, OB_NR = 16, OB_NF = 16, OB_RB = 256, OB_TS = 36;
constexpr int OB_CNT_LINE = 32;  // one counter per 128-B line
// Loads in flight in the two 16-partial reductions (steps 2 and 4): all 16 issued
// before the fixed-order sum (r05; 4 before) - one L2 / fabric round trip per lane
// instead of four, same sums bit for bit.
#ifdef DEIG_AB_OJA_RED_UNROLL
constexpr int kOjaRedUnroll = DEIG_AB_OJA_RED_UNROLL;
#else
constexpr int kOjaRedUnroll = 16;
#endif

struct OjaBlk {
  const float* X;  // first batch of the run
  int64_t ldx;
  int64_t b;
  int d, kp, nbatch;
  float coef;      // eta / b
  float* V;        // row-padded d x kp, updated in place
  u32x4* vimg;     // V's image (NN B operand)
  u32x4* timg;     // T's image (TN B operand)
  float* ppart;    // [16 j][b / 4][kp][4]
  float* qpart;    // [16 i][d / 4][kp][4]
  unsigned* cnt;   // [4 phases][16 groups] x OB_CNT_LINE, then the exit count
  unsigned* err;
  unsigned long long* trace;  // measurement builds only (DEIG_AB_OJA_TRACE)
};
// Measurement builds only (-DDEIG_AB_OJA_TRACE, tools/oja_trace.py): per block and batch
// 16 wall_clock64 stamps at the phase boundaries, in a buffer after the workspace.
#ifdef DEIG_AB_OJA_TRACE
#define OB_STAMP(slot, cond) \
  if (cond) a.trace[((int64_t)blockIdx.x * 64 + (bt & 63)) * 16 + (slot)] = wall_clock64()
#else
#define OB_STAMP(slot, cond)
#endif

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ob_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// 16-B write-through store / L1-bypassing load (aux 16 = sc1)
__device__ __forceinline__ void ob_st(const __amdgpu_buffer_rsrc_t& r, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 16);
}
__device__ __forceinline__ u32x4 ob_ld(const __amdgpu_buffer_rsrc_t& r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16);
}
__device__ __forceinline__ void ob_signal(unsigned* c) {
  __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Spin bound of one hand-off wait in wall_clock64 ticks (100 MHz): 2 s.  Test builds
// only (-DDEIG_AB_OJA_SPIN_TICKS=0, tests/test_gpu_oja_timeout.py) shrink it so that
// waits time out and the timeout report (deig_oja_error) can be exercised.
#ifdef DEIG_AB_OJA_SPIN_TICKS
constexpr uint64_t kOjaSpinTicks = DEIG_AB_OJA_SPIN_TICKS;
#else
constexpr uint64_t kOjaSpinTicks = 200000000ull;
#endif
// One lane: wait until *c >= target (bounded; see above).
__device__ __forceinline__ void ob_wait(unsigned* c, unsigned target, unsigned* err) {
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    if (wall_clock64() - t0 >= kOjaSpinTicks) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}
__device__ __forceinline__ void ob_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <int NB, int NKS>
__global__ __launch_bounds__(512) void oja_blk_kernel(OjaBlk a) {
  constexpr int KP = 16 * NB;
  constexpr int FB = 32 * NKS;
  constexpr int VL_N = NKS * NB * 2 * 64;  // u32x4 of V_j's image
  constexpr int NFT = 2 * NKS;              // feature tiles of the block
  // feature tiles per step-3 reduction chunk: the largest even divisor of NFT up to 6
  constexpr int CH = NFT <= 6 ? NFT : NFT % 6 == 0 ? 6 : NFT % 4 == 0 ? 4 : 2;
  static_assert(NFT % CH == 0 && CH % 2 == 0, "step-3 chunks are whole k-steps");
  // red (step 3's cross-wave sums) and vl (step 1's V_j image) are never live together
  __shared__ f32x4 red[8][CH][NB][64];
  static_assert(sizeof(red) >= VL_N * sizeof(u32x4), "vl aliases red");
  u32x4* vl = reinterpret_cast<u32x4*>(&red[0][0][0][0]);
  __shared__ __attribute__((aligned(16))) float xt[8][32 * OB_TS];
  __shared__ float tt[16][KP + 1];
  __shared__ unsigned step3_done, step4_done;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = threadIdx.x;
  // column group j on one XCD: blocks b, b + 8, ... (XCD b & 7) take j = 2 x + s / 16
  const int x = blockIdx.x & 7, sl = blockIdx.x >> 3;
  const int j = 2 * x + (sl >> 4), i = sl & 15;
  const int R0 = OB_RB * i, F0 = FB * j;
  const int64_t b = a.b;
  const int d = a.d;
  unsigned* cA = a.cnt + (0 * 16 + i) * OB_CNT_LINE;
  unsigned* cB = a.cnt + (1 * 16 + i) * OB_CNT_LINE;
  unsigned* cC = a.cnt + (2 * 16 + j) * OB_CNT_LINE;
  unsigned* cD = a.cnt + (3 * 16 + j) * OB_CNT_LINE;
  const __amdgpu_buffer_rsrc_t rv = ob_rsrc(a.vimg, (uint32_t)((d / 32) * NB * 2 * 64 * 16));
  const __amdgpu_buffer_rsrc_t rt = ob_rsrc(a.timg, (uint32_t)((b / 32) * NB * 2 * 64 * 16));
  const __amdgpu_buffer_rsrc_t rp = ob_rsrc(a.ppart, (uint32_t)(16 * b * KP * 4));
  const __amdgpu_buffer_rsrc_t rq = ob_rsrc(a.qpart, (uint32_t)(16 * (int64_t)d * KP * 4));

  // this wave's X: rows R0 + 32 w + 16 rt + (lane & 15), features F0 + 32 ks + 8 (lane >> 4) + 4 h
  f32x4 xr[2][NKS][2];
  auto load_x_ks = [&](int bt, int ks) {
    const float* xb = a.X + (int64_t)bt * b * a.ldx;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const float* row = xb + (int64_t)(R0 + 32 * wave + 16 * r + (lane & 15)) * a.ldx + F0 + 8 * (lane >> 4);
      xr[r][ks][0] = *reinterpret_cast<const f32x4*>(row + 32 * ks);
      xr[r][ks][1] = *reinterpret_cast<const f32x4*>(row + 32 * ks + 4);
    }
  };
  auto load_x = [&](int bt) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) load_x_ks(bt, ks);
  };
  load_x(0);
  for (int bt = 0; bt < a.nbatch; ++bt) {
    const unsigned target = 16u * (unsigned)(bt + 1);
    const bool more = bt + 1 < a.nbatch;
    // ---- V_j's image -> LDS (written by the previous batch's step 4, or before the launch)
    for (int u = t; u < VL_N; u += 512)  // k-steps F0 / 32 .. are contiguous in the image
      vl[u] = ob_ld(rv, (uint32_t)(((int64_t)(F0 / 32) * NB * 2 * 64 + u) * 16));
    __syncthreads();
    OB_STAMP(0, t == 0);
    // ---- 1. P = X_ij V_j
    {
      f32x4 acc[2][NB];
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[r][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          bf16x8 ahi, alo;
          split8(xr[r][ks][0], xr[r][ks][1], ahi, alo);
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) {
            const bf16x8 bhi = __builtin_bit_cast(bf16x8, vl[((ks * NB + nb) * 2 + 0) * 64 + lane]);
            const bf16x8 blo = __builtin_bit_cast(bf16x8, vl[((ks * NB + nb) * 2 + 1) * 64 + lane]);
            acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bhi, acc[r][nb], 0, 0, 0);
            acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, blo, acc[r][nb], 0, 0, 0);
            acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bhi, acc[r][nb], 0, 0, 0);
          }
        }
      }
      // rows 4 (lane >> 4) + e of the tile, column 16 nb + (lane & 15): [j][row / 4][col][4]
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const int64_t rq = (R0 + 32 * wave + 16 * r) / 4 + (lane >> 4);
          const int col = 16 * nb + (lane & 15);
          ob_st(rp, (uint32_t)((((int64_t)j * (b / 4) + rq) * KP + col) * 16),
                __builtin_bit_cast(u32x4, acc[r][nb]));
        }
    }
    ob_drain();
    __syncthreads();
    OB_STAMP(1, t == 0);
    if (t == 0) {
      ob_signal(cA);
      ob_wait(cA, target, a.err);
    }
    __syncthreads();
    OB_STAMP(2, t == 0);
    // ---- 2. T rows R0 + 16 j .. + 15 = sum_j' P_ij'
    if (t < 4 * KP) {
      const int rql = t / KP, col = t - rql * KP;
      const int64_t rq = (R0 + 16 * j) / 4 + rql;
      f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll kOjaRedUnroll
      for (int jj = 0; jj < OB_NF; ++jj)
        s += __builtin_bit_cast(f32x4, ob_ld(rp, (uint32_t)((((int64_t)jj * (b / 4) + rq) * KP + col) * 16)));
#pragma unroll
      for (int e = 0; e < 4; ++e) tt[4 * rql + e][col] = s[e];
    }
    __syncthreads();
    if (t < 2 * KP) {
      const int gi = t / KP, col = t - gi * KP;
      float v[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) v[jj] = tt[8 * gi + jj][col];
      bf16x8 hi, lo;
      split8(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, hi, lo);
      const int r0 = R0 + 16 * j;
      const int ln = (col & 15) + 16 * ((r0 & 31) / 8 + gi);
      ob_st(rt, (uint32_t)(img_index(r0 / 32, col / 16, 0, ln, NB) * 16), __builtin_bit_cast(u32x4, hi));
      ob_st(rt, (uint32_t)(img_index(r0 / 32, col / 16, 1, ln, NB) * 16), __builtin_bit_cast(u32x4, lo));
    }
    ob_drain();
    __syncthreads();
    OB_STAMP(3, t == 0);
    if (t == 0) {
      ob_signal(cB);
      ob_wait(cB, target, a.err);
    }
    __syncthreads();
    OB_STAMP(4, t == 0);
    // ---- 3. Q_ij = X_ij^T T_i: wave w takes row step w (its own rows) for every
    // feature tile; its T_i fragments straight to registers
    {
      bf16x8 th[NB], tlo[NB];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        th[nb] = __builtin_bit_cast(bf16x8, ob_ld(rt, (uint32_t)(img_index(R0 / 32 + wave, nb, 0, lane, NB) * 16)));
        tlo[nb] = __builtin_bit_cast(bf16x8, ob_ld(rt, (uint32_t)(img_index(R0 / 32 + wave, nb, 1, lane, NB) * 16)));
      }
#ifdef DEIG_AB_OJA_TRACE
      if (wave == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // T fragments landed
#endif
      OB_STAMP(10, t == 0);
      float* T = xt[wave];
      if (t == 0) step3_done = step4_done = 0;  // arrival counters (barriers follow)
      // CH feature tiles (CH / 2 k-steps) at a time: their products, then the 8 row
      // steps' partials summed in wave order
#pragma unroll
      for (int c0 = 0; c0 < NFT; c0 += CH) {
        f32x4 acc[CH][NB];
#pragma unroll
        for (int kc = 0; kc < CH / 2; ++kc) {
          const int ks = c0 / 2 + kc;
          // this wave's 32 rows x 32 features of k-step ks, transposed: T[f][row]
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int e = 0; e < 4; ++e)
                T[(8 * (lane >> 4) + 4 * h + e) * OB_TS + 16 * r + (lane & 15)] = xr[r][ks][h][e];
          // waves 0-5: this k-step of the next batch's block streams from here on (its
          // registers are free once staged); waves 6, 7 publish Q and run step 4
          // first, and their drains would wait for it
          if (wave < 6 && more) load_x_ks(bt + 1, ks);
#pragma unroll
          for (int f2 = 0; f2 < 2; ++f2) {
            const f32x4 a0 = *reinterpret_cast<const f32x4*>(T + (16 * f2 + (lane & 15)) * OB_TS + 8 * (lane >> 4));
            const f32x4 a1 = *reinterpret_cast<const f32x4*>(T + (16 * f2 + (lane & 15)) * OB_TS + 8 * (lane >> 4) + 4);
            bf16x8 ahi, alo;
            split8(a0, a1, ahi, alo);
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
              f32x4 c = {0.f, 0.f, 0.f, 0.f};
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, th[nb], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, tlo[nb], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, th[nb], c, 0, 0, 0);
              acc[2 * kc + f2][nb] = c;
            }
          }
        }
#pragma unroll
        for (int ft = 0; ft < CH; ++ft)
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) red[wave][ft][nb][lane] = acc[ft][nb];
        OB_STAMP(11 + 2 * (c0 / CH), t == 0 && c0 / CH < 2);
        __syncthreads();
        OB_STAMP(12 + 2 * (c0 / CH), t == 0 && c0 / CH < 2);
        for (int u = t - 384; u >= 0 && u < CH * NB * 64; u += 128) {  // waves 6, 7
          const int ln = u & 63, nb = (u >> 6) % NB, ft = (u >> 6) / NB;
          f32x4 sm = red[0][ft][nb][ln];
#pragma unroll
          for (int w = 1; w < 8; ++w) sm += red[w][ft][nb][ln];
          const int64_t fq = (F0 + 16 * (c0 + ft)) / 4 + (ln >> 4);
          const int col = 16 * nb + (ln & 15);
          ob_st(rq, (uint32_t)((((int64_t)i * (d / 4) + fq) * KP + col) * 16), __builtin_bit_cast(u32x4, sm));
        }
        __syncthreads();
      }
    }
    OB_STAMP(5, t == 0);
    if (wave >= 6) {
      // Q published by waves 6, 7 only: both drained, the second to arrive signals
      ob_drain();
      if (lane == 0 && atomicAdd(&step3_done, 1u) == 1u) ob_signal(cC);
      // ---- 4. (waves 6, 7) V[F_j] group of 8 features g = i + 16 (wave - 6) (< FB / 8)
      if (lane == 0) ob_wait(cC, target, a.err);
      __builtin_amdgcn_wave_barrier();
      OB_STAMP(6, lane == 0 && wave == 7);
      const int col = lane >> 1, q = lane & 1;
      const int g = i + OB_NR * (wave - 6);
      if (g < FB / 8) {
        f32x4 sm = {0.f, 0.f, 0.f, 0.f};
        const int64_t fq = (F0 + 8 * g) / 4 + q;
        // this lane's V entries first (independent of the partials: their loads
        // overlap the partials' instead of following the sum)
        float vo[4] = {0.f, 0.f, 0.f, 0.f};
        if (col < KP) {
#pragma unroll
          for (int e = 0; e < 4; ++e) vo[e] = a.V[(4 * fq + e) * KP + col];
#pragma unroll kOjaRedUnroll
          for (int ii = 0; ii < OB_NR; ++ii)
            sm += __builtin_bit_cast(f32x4, ob_ld(rq, (uint32_t)((((int64_t)ii * (d / 4) + fq) * KP + col) * 16)));
        }
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t f = 4 * fq + e;
          v[e] = 0.f;
          if (col < KP) {
            v[e] = fmaf(a.coef, sm[e], vo[e]);
            a.V[f * KP + col] = v[e];
          }
        }
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = __shfl_xor(v[e], 1, 64);
        // the group's 8 features in order: lane q = 0 holds 0..3, its partner 4..7
        const f32x4 first = q ? f32x4{o[0], o[1], o[2], o[3]} : f32x4{v[0], v[1], v[2], v[3]};
        const f32x4 second = q ? f32x4{v[0], v[1], v[2], v[3]} : f32x4{o[0], o[1], o[2], o[3]};
        bf16x8 hh, ll;
        split8(first, second, hh, ll);
        if (col < KP) {
          const int f8 = F0 + 8 * g;
          const int ln = (col & 15) + 16 * ((f8 & 31) / 8);
          ob_st(rv, (uint32_t)(img_index(f8 / 32, col / 16, q, ln, NB) * 16),
                __builtin_bit_cast(u32x4, q ? ll : hh));
        }
      }
      ob_drain();
      OB_STAMP(7, lane == 0 && wave == 7);
      if (lane == 0 && atomicAdd(&step4_done, 1u) == 1u) ob_signal(cD);
      if (more) load_x(bt + 1);
    }
    OB_STAMP(8, t == 0);
    if (more) {
      if (t == 0) ob_wait(cD, target, a.err);
      __syncthreads();
    }
    OB_STAMP(9, t == 0);
  }
#ifndef DEIG_AB_OJA_COOP
  // The hand-off counters are left at zero for the next launch on this workspace
  // (no memset and its kernel boundary between runs): every block drains its own
  // counter atomics (vmcnt(0): performed, not just issued), then counts itself out;
  // the last one out - every other block is past all of its waits and signals -
  // zeroes the counters and the exit count.
  ob_drain();
  __syncthreads();
  if (t == 0) {
    unsigned* ce = a.cnt + 4 * 16 * OB_CNT_LINE;
    if (__hip_atomic_fetch_add(ce, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == OB_G - 1u) {
      for (int c = 0; c < 4 * 16; ++c)
        __hip_atomic_store(a.cnt + c * OB_CNT_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ce, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
#endif
}

struct OjaWs {
  unsigned *cnt, *err;  // v4 hand-off counters (zero between launches) and timeout word
  float *Vr, *Vr2, *G, *Rinv, *slab;
  u32x4 *vimg, *timg;  // bf16 operand images of V (NN) and T (TN)
  float *ppart, *qpart;  // v4 partials
  unsigned long long* trace;
  size_t slab_bytes;
};
// [4 phases][16 groups] hand-off counters + the exit count, one per 128-B line
constexpr size_t OB_CNT_BYTES = (4 * 16 + 1) * OB_CNT_LINE * sizeof(unsigned);

OjaWs carve_oja(void* ws, size_t cap, int64_t b, int64_t d, int kp, size_t* total) {
  Carve c(ws, cap);
  OjaWs o;
  // the counters first: the per-launch memset starts at the allocation and is a
  // multiple of 16 B (cdna_hip_programming.md Guideline 16, Re-initialise every call)
  o.cnt = c.take<unsigned>(OB_CNT_BYTES / sizeof(unsigned));
  o.err = c.take<unsigned>(OB_CNT_LINE);
  o.Vr = c.take<float>((size_t)d * kp);
  o.Vr2 = c.take<float>((size_t)d * kp);
  o.G = c.take<float>((size_t)kp * kp);
  o.Rinv = c.take<float>((size_t)kp * kp);
  o.vimg = c.take<u32x4>((size_t)cdiv(d, 32) * (kp / 16) * 2 * 64);
  o.timg = c.take<u32x4>((size_t)cdiv(b, 32) * (kp / 16) * 2 * 64);
  // CholQR's two skinny products (the NN / TN passes reduce in LDS: no slabs)
  size_t sb = skinny_workspace_bytes(kp, kp, d);
  const size_t s4 = skinny_workspace_bytes(d, kp, kp);
  if (s4 > sb) sb = s4;
  o.slab = c.take<float>(sb / sizeof(float) + 1);
  o.slab_bytes = sb;
  o.ppart = c.take<float>((size_t)OB_NF * b * kp);
  o.qpart = c.take<float>((size_t)OB_NR * d * kp);
#ifdef DEIG_AB_OJA_TRACE
  o.trace = c.take<unsigned long long>((size_t)OB_G * 64 * 16);
#else
  o.trace = nullptr;
#endif
  *total = c.off;
  return o;
}

// Cholesky-QR of the row-padded d x kp basis `in` (`scratch` has the same size) with
// `passes` passes (2 = CholQR2, orthonormal to fp32 rounding; 1 = one pass, used
// between batches where only the span and a bounded condition number matter);
// the result is in *result (in or scratch: one buffer swap per pass).
// The apply is a triangular solve (trsm_img_kernel) with L from the one-wave
// Cholesky; with_img: the last pass also writes the result's NN operand image.
int cholqr(float* in, float* scratch, const OjaWs& o, int64_t d, int k, int kp, hipStream_t st,
           int passes, float** result, bool with_img) {
  int rc;
  float* cur = in;
  float* nxt = scratch;
  for (int pass = 0; pass < passes; ++pass) {
    if ((rc = skinny_launch(true, cur, kp, cur, kp, o.G, kp, kp, kp, d, 1.f, 0.f, o.slab,
                            o.slab_bytes, st)))
      return rc;
    u32x4* img = (with_img && pass + 1 == passes) ? o.vimg : nullptr;
    const dim3 g((unsigned)cdiv(d, 32));
    if (kp <= 16) {
      hipLaunchKernelGGL((chol_rinv_kernel<16, false>), dim3(1), dim3(64), 0, st, o.G, k, kp, o.Rinv);
      hipLaunchKernelGGL(trsm_img_kernel<16>, g, dim3(256), 0, st, cur, o.Rinv, d, kp, nxt, img);
    } else if (kp <= 32) {
      hipLaunchKernelGGL((chol_rinv_kernel<32, false>), dim3(1), dim3(64), 0, st, o.G, k, kp, o.Rinv);
      hipLaunchKernelGGL(trsm_img_kernel<32>, g, dim3(256), 0, st, cur, o.Rinv, d, kp, nxt, img);
    } else if (kp <= 48) {
      hipLaunchKernelGGL((chol_rinv_kernel<48, false>), dim3(1), dim3(64), 0, st, o.G, k, kp, o.Rinv);
      hipLaunchKernelGGL(trsm_img_kernel<48>, g, dim3(256), 0, st, cur, o.Rinv, d, kp, nxt, img);
    } else {
      hipLaunchKernelGGL((chol_rinv_kernel<64, false>), dim3(1), dim3(64), 0, st, o.G, k, kp, o.Rinv);
      hipLaunchKernelGGL(trsm_img_kernel<64>, g, dim3(256), 0, st, cur, o.Rinv, d, kp, nxt, img);
    }
    DEIG_HIP_CHECK(hipGetLastError());
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
// v4 (oja_blk_kernel) shape: one 4096-row batch on a 16 x 16 grid of X blocks held
// in registers (d = 512 c <= 3072, kp <= 32), 256 co-resident workgroups.
bool oja_blk_eligible(int64_t b, int64_t d, int64_t ldx, int kp) {
  return b == (int64_t)OB_NR * OB_RB && d % 512 == 0 && d >= 512 && d <= 3072 && kp <= 32 &&
         ldx % 4 == 0 && num_cus() >= OB_G;
}

// The resident kernel's workgroups wait on each other, so all OB_G of them must be
// resident at once.  r05 measured the cooperative launch (hipLaunchCooperativeKernel)
// at ~12 us of idle device time on each side of every run (profiles/r05p_c4_*): it
// drains the queue first.  Its only service is the launch-time check of the grid
// against the occupancy query (MI355X_MICROARCH.md, cost table 'coop-launch'), so the
// same check is made here once per kernel instance - one workgroup of 512 threads per
// CU on >= OB_G CUs - and the grid goes out as a plain launch.  A device whose CUs are
// held by other work can still delay some workgroups: the 2-s spin bound turns that
// into NaN output (see above), never a hang.
template <int NB, int NKS>
bool oja_blk_fits() {
  static const bool ok = [] {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, oja_blk_kernel<NB, NKS>, 512, 0) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return n >= 1 && num_cus() >= OB_G;
  }();
  return ok;
}

template <int NB>
hipError_t launch_oja_blk(int nks, const OjaBlk& a, hipStream_t st) {
#ifndef DEIG_AB_OJA_COOP
  switch (nks) {
#define DEIG_OJA_NKS(x)                                                                         \
  case x:                                                                                       \
    if (!oja_blk_fits<NB, x>()) return hipErrorCooperativeLaunchTooLarge;                      \
    hipLaunchKernelGGL((oja_blk_kernel<NB, x>), dim3(OB_G), dim3(512), 0, st, a);               \
    return hipGetLastError();
    DEIG_OJA_NKS(1) DEIG_OJA_NKS(2) DEIG_OJA_NKS(3) DEIG_OJA_NKS(4) DEIG_OJA_NKS(5) DEIG_OJA_NKS(6)
#undef DEIG_OJA_NKS
    default:
      return hipErrorInvalidValue;
  }
#else
  const void* fn = nullptr;
  switch (nks) {
#define DEIG_OJA_NKS(x) \
  case x:               \
    fn = reinterpret_cast<const void*>(&oja_blk_kernel<NB, x>); \
    break;
    DEIG_OJA_NKS(1) DEIG_OJA_NKS(2) DEIG_OJA_NKS(3) DEIG_OJA_NKS(4) DEIG_OJA_NKS(5) DEIG_OJA_NKS(6)
#undef DEIG_OJA_NKS
    default:
      return hipErrorInvalidValue;
  }
  OjaBlk arg = a;
  void* args[] = {&arg};
  return hipLaunchCooperativeKernel(fn, dim3(OB_G), dim3(512), args, 0, st);
#endif
}

int oja_steps_launch(const float* X, int64_t nb, int64_t b, int64_t d, int64_t ldx, float eta,
                     float* V, int k, int64_t ldv, int orth_every, void* ws, size_t ws_bytes,
                     hipStream_t st, int algo) {
  DEIG_REQUIRE(nb >= 1 && b >= 1 && d >= 4 && d % 4 == 0,
               "oja: need nb >= 1, b >= 1 and d %% 4 == 0");
  DEIG_REQUIRE(k >= 1 && k <= 64 && k <= d, "oja: need 1 <= k <= min(64, d)");
  DEIG_REQUIRE(ldx >= d && ldx % 4 == 0 && ldv >= d, "oja: bad leading dims");
  DEIG_REQUIRE(orth_every >= 1, "oja: orth_every must be >= 1");
  DEIG_REQUIRE(algo == DEIG_OJA_AUTO || algo == DEIG_OJA_TWO_PASS || algo == DEIG_OJA_RESIDENT,
               "oja: unknown algo %d", algo);
  const int kp = (int)cdiv(k, 16) * 16;
  size_t total = 0;
  OjaWs o = carve_oja(ws, ws_bytes, b, d, kp, &total);
  if (!ws || total > ws_bytes)
    return fail(DEIG_EWORKSPACE, "oja: workspace %zu < %zu", ws_bytes, total);
  bool blk = algo != DEIG_OJA_TWO_PASS && oja_blk_eligible(b, d, ldx, kp);
  if (algo == DEIG_OJA_RESIDENT && !blk)
    return fail(DEIG_EINVAL, "oja: the resident path needs b = 4096, d = 512 c <= 3072, k <= 32 "
                             "and %d CUs (got b %lld, d %lld, k %d)", OB_G, (long long)b, (long long)d, k);
  int rc;
  DEIG_HIP_CHECK(hipMemsetAsync(o.err, 0, sizeof(unsigned), st));
  // the basis lives in `cur` (o.Vr or o.Vr2: each CholQR pass swaps the two)
  float* cur = o.Vr;
  float* spare = o.Vr2;
  hipLaunchKernelGGL(col_to_rowpad, dim3((unsigned)cdiv(d * kp, 256)), dim3(256), 0, st, V, ldv, d,
                     k, kp, cur);
  DEIG_HIP_CHECK(hipGetLastError());
  const int NB = kp / 16;
  const int nks = (int)cdiv(d, 32), nkr = (int)cdiv(b, 32);
  auto build_vimg = [&](const float* Vr) -> int {
    hipLaunchKernelGGL(img_kernel, dim3((unsigned)cdiv((int64_t)nks * NB * 64, 256)), dim3(256), 0, st, Vr,
                       d, kp, nks, o.vimg);
    DEIG_HIP_CHECK(hipGetLastError());
    return DEIG_OK;
  };
  if ((rc = build_vimg(cur))) return rc;
  // runs of batches between two re-orthonormalisations (after batch i when
  // (i + 1) % orth_every == 0, and after the last): intermediate ones only bound the
  // basis' condition number (the span is what the update carries) - one CholQR pass;
  // the last one is CholQR2
  for (int64_t i0 = 0; i0 < nb;) {
    const int64_t i1 = std::min(nb, (i0 / orth_every + 1) * orth_every);
    if (blk) {
#ifndef DEIG_AB_OJA_COOP
      // zeroed once per call: each launch leaves them at zero for the next
      if (i0 == 0) DEIG_HIP_CHECK(hipMemsetAsync(o.cnt, 0, OB_CNT_BYTES, st));
#else
      DEIG_HIP_CHECK(hipMemsetAsync(o.cnt, 0, OB_CNT_BYTES, st));
#endif
      OjaBlk a;
      a.X = X + i0 * b * ldx;
      a.ldx = ldx;
      a.b = b;
      a.d = (int)d;
      a.kp = kp;
      a.nbatch = (int)(i1 - i0);
      a.coef = eta / (float)b;
      a.V = cur;
      a.vimg = o.vimg;
      a.timg = o.timg;
      a.ppart = o.ppart;
      a.qpart = o.qpart;
      a.cnt = o.cnt;
      a.err = o.err;
      a.trace = o.trace;
      const hipError_t le = NB == 1 ? launch_oja_blk<1>((int)(d / 512), a, st)
                                    : launch_oja_blk<2>((int)(d / 512), a, st);
      if (le != hipSuccess) {
        (void)hipGetLastError();
        // the grid cannot be co-resident (CUs held by other work, a partitioned
        // device): DEIG_OJA_RESIDENT reports it, AUTO runs this and every later run
        // on the two-pass kernels (the same arithmetic, to within 1e-5)
        if (algo == DEIG_OJA_RESIDENT)
          return fail(DEIG_EHIP, "oja: the resident kernel's grid cannot be co-resident: %s",
                      hipGetErrorString(le));
        blk = false;
      }
    }
    if (!blk) {
      for (int64_t i = i0; i < i1; ++i) {
        const float* Xb = X + i * b * ldx;
        // T = Xb V (as the TN pass's operand image, every row of its nkr k-steps
        // written, zeros past b), then V += eta/b Xb^T T (and V's image)
        switch (NB) {
#define DEIG_OJA_NB(x)                                                                           \
  case x:                                                                                        \
    hipLaunchKernelGGL(oja_nn_kernel<x>, dim3((unsigned)(2 * nkr)), dim3(512), 0, st, Xb, ldx, b, \
                       (int)d, nks, o.vimg, o.timg);                                             \
    hipLaunchKernelGGL(oja_tn_kernel<x>, dim3((unsigned)cdiv(d, 16)), dim3(512), 0, st, Xb, ldx, b, \
                       (int)d, nkr, o.timg, eta / (float)b, cur, o.vimg);                        \
    break;
          DEIG_OJA_NB(1) DEIG_OJA_NB(2) DEIG_OJA_NB(3) DEIG_OJA_NB(4)
#undef DEIG_OJA_NB
          default:
            return fail(DEIG_EINVAL, "oja: k = %d > 64", k);
        }
        DEIG_HIP_CHECK(hipGetLastError());
      }
    }
    const int passes = i1 == nb ? 2 : 1;
    float* res = cur;
    if ((rc = cholqr(cur, spare, o, d, k, kp, st, passes, &res, i1 < nb))) return rc;
    spare = res == cur ? spare : cur;
    cur = res;
    i0 = i1;
  }
  hipLaunchKernelGGL(rowpad_to_col, dim3((unsigned)cdiv(d * k, 256)), dim3(256), 0, st, cur, d, k,
                     kp, V, ldv, o.err);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

// The timeout word of the last oja_steps_launch on this workspace (set by a resident
// hand-off that waited past its bound; V was then written as NaN).  Synchronises st.
int oja_error(const void* ws, size_t ws_bytes, int64_t b, int64_t d, int k, hipStream_t st) {
  DEIG_REQUIRE(k >= 1 && k <= 64 && b >= 1 && d >= 4, "oja_error: bad shape");
  const int kp = (int)cdiv(k, 16) * 16;
  size_t total = 0;
  OjaWs o = carve_oja(const_cast<void*>(ws), ws_bytes, b, d, kp, &total);
  if (!ws || total > ws_bytes)
    return fail(DEIG_EWORKSPACE, "oja_error: workspace %zu < %zu", ws_bytes, total);
  unsigned e = 0;
  DEIG_HIP_CHECK(hipMemcpyAsync(&e, o.err, sizeof(e), hipMemcpyDeviceToHost, st));
  DEIG_HIP_CHECK(hipStreamSynchronize(st));
  if (e)
    return fail(DEIG_ETIMEOUT, "oja: a resident hand-off waited past its bound (CUs held by other "
                               "work?); V was written as NaN");
  return DEIG_OK;
}

int oja_launch(const float* Xb, int64_t b, int64_t d, int64_t ldx, float eta, float* V, int k,
               int64_t ldv, void* ws, size_t ws_bytes, hipStream_t st) {
  return oja_steps_launch(Xb, 1, b, d, ldx, eta, V, k, ldv, 1, ws, ws_bytes, st, DEIG_OJA_AUTO);
}

}  // namespace deig
