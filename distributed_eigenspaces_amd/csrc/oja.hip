// Mini-batch Oja steps for the online / streaming variant (BASELINE.json config 4):
//   V <- orth(V + eta/b * Xb^T (Xb V)),   orth = Cholesky-QR2.
// Not present in the reference (parity unpinned; judged by sin(theta) against
// the one-shot float64 oracle and ref_cpu.oja_epoch).  Xb is read twice (Xb V
// and Xb^T T), each pass at ~k/2 flop/B (HBM-bound for k <= 32): two launches per
// batch (oja_nn_kernel, oja_tn_kernel), bf16x3 split products, K split over the
// waves of a block and summed in LDS (no slab passes); each pass writes the next
// one's MFMA operand image (T's for TN, V's for the next batch's NN).
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

// Measurement builds only (tools/oja_ab.py; the shipped library is variant 0):
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

struct OjaWs {
  float *Vr, *Vr2, *G, *Rinv, *slab;
  u32x4 *vimg, *timg;  // bf16 operand images of V (NN) and T (TN)
  size_t slab_bytes;
};

OjaWs carve_oja(void* ws, size_t cap, int64_t b, int64_t d, int kp, size_t* total) {
  Carve c(ws, cap);
  OjaWs o;
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
  const int NB = kp / 16;
  const int nks = (int)cdiv(d, 32), nkr = (int)cdiv(b, 32);
  auto build_vimg = [&](const float* Vr) -> int {
    hipLaunchKernelGGL(img_kernel, dim3((unsigned)cdiv((int64_t)nks * NB * 64, 256)), dim3(256), 0, st, Vr,
                       d, kp, nks, o.vimg);
    DEIG_HIP_CHECK(hipGetLastError());
    return DEIG_OK;
  };
  if ((rc = build_vimg(cur))) return rc;
  for (int64_t i = 0; i < nb; ++i) {
    const float* Xb = X + i * b * ldx;
    // T = Xb V (as the TN pass's operand image, every row of its nkr k-steps written,
    // zeros past b), then V += eta/b Xb^T T (and V's image)
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
    // intermediate re-orthonormalisations only bound the basis' condition number
    // (the span is what the update carries): one CholQR pass; the last one is CholQR2
    const int passes = (i + 1 == nb) ? 2 : ((i + 1) % orth_every == 0 ? 1 : 0);
    if (passes) {
      float* res = cur;
      if ((rc = cholqr(cur, spare, o, d, k, kp, st, passes, &res))) return rc;
      spare = res == cur ? spare : cur;
      cur = res;
      if (i + 1 < nb && (rc = build_vimg(cur))) return rc;
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
