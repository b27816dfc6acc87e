// Exact covariance of uint8 samples on CDNA4 int8 MFMA (fused
// ingest):  S = alpha * V^T V  with V the n x d feature matrix of
//   DEIG_U8_RAW  : v = x (one byte per feature, d bytes of each row);
//   DEIG_U8_GRAY3: v = (r + g + b) / 3 for interleaved pixels (3 bytes per feature) -
//                  the reference's grayscale + flatten, distributed.py:170-173
//                  (data.mean(axis=3), reshape to 1024) followed by :59-70.
// The reference computes in float64 from the uint8 CIFAR bytes (load_data.py:18-33);
// here every product and sum is EXACT (integers), so S is the exact result rounded
// once (fp64; fp32 within 1 ulp of the correctly rounded value, u8_finalize_kernel)
// - no accumulation error at all,
// which an fp32 SYRK of uncentered 0..255 data cannot offer (its rounding noise
// ~5e-7 max|S| alone moves a CIFAR-like top-k basis by ~3e-4 in ||P - P_ref||_F).
//
// Integer decomposition (all operands int8, v_mfma_i32_16x16x64_i8, int32 acc):
//   raw : y = x - 128 (= x ^ 0x80 as int8);
//         sum x_i x_j = sum y_i y_j + 128 (Y_i + Y_j) + 128^2 n,   Y = column sums of y
//   gray: s = r + g + b in [0, 765], t = s - 384 in [-384, 381] = 16 h + l,
//         h = t >> 4 in [-24, 23], l = t & 15, w = h + l in [-24, 38]  (three planes);
//         sum t_i t_j = 240 P_hh + 16 P_ww - 15 P_ll   (P_ww - P_hh - P_ll = the cross term)
//         sum s_i s_j = sum t_i t_j + 384 (T_i + T_j) + 384^2 n,   T = column sums of t,
//         and v = s / 3 gives the factor 1/9.
// Pipeline: u8_prep_kernel (X -> int8 planes in MFMA operand order + int64 column
// sums), u8_syrk_kernel (128 x 128 lower tiles x K segments x planes, LDS double
// buffer, int32 MFMA accumulators, int64 atomic adds: exact and order independent,
// hence deterministic), u8_finalize_kernel (combine planes + corrections in int64,
// one double rounding, both triangles from the same value: bit-exact symmetry).
#include "deig_internal.hpp"

namespace deig {
namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int KB = 64;        // rows per K-step (one MFMA 16x16x64 depth)
constexpr int TB = 128;       // output tile edge (features)
constexpr int FPAD = 128;     // features padded to a multiple of this
constexpr int SYRK_THR = 256;  // 4 waves, 2 x 2 wave tiles of 64 x 64
constexpr int PREP_THR = 256;  // prep: 4 waves (one 16-row group each), 4 features per lane
constexpr int MAX_SEG_KB = 1024;  // <= 65536 rows per item: int32 accumulators cannot overflow
constexpr int PREP_YB = 128;

inline int u8_planes(int mode) { return mode == DEIG_U8_GRAY3 ? 3 : 1; }

// Image: plane-major, then [kb][g = 16-row group][feature][16 bytes = rows 16g..16g+15].
__host__ __device__ inline int64_t img_off(int64_t plane, int64_t kb, int g, int64_t f, int64_t nkb,
                                           int64_t fpad) {
  return (((plane * nkb + kb) * 4 + g) * fpad + f) * 16;
}

// 4 x 4 byte transpose: r[q] holds byte u = feature u of row q; out[u] holds byte q =
// row q of feature u.
__device__ __forceinline__ void tr4(const uint32_t r[4], uint32_t out[4]) {
  const uint32_t lo01 = __builtin_amdgcn_perm(r[1], r[0], 0x05010400u);
  const uint32_t hi01 = __builtin_amdgcn_perm(r[1], r[0], 0x07030602u);
  const uint32_t lo23 = __builtin_amdgcn_perm(r[3], r[2], 0x05010400u);
  const uint32_t hi23 = __builtin_amdgcn_perm(r[3], r[2], 0x07030602u);
  out[0] = __builtin_amdgcn_perm(lo23, lo01, 0x05040100u);
  out[1] = __builtin_amdgcn_perm(lo23, lo01, 0x07060302u);
  out[2] = __builtin_amdgcn_perm(hi23, hi01, 0x05040100u);
  out[3] = __builtin_amdgcn_perm(hi23, hi01, 0x07060302u);
}

__device__ __forceinline__ int sbyte(uint32_t v, int u) { return (int)(int8_t)(v >> (8 * u)); }

// grid (fpad / 256, YB), 4 waves: lane owns features f .. f + 3 (f = 256 bx + 4 lane)
// and wave g the 16-row group g of row blocks kb = by, by + YB, ...; per group it
// loads one dword (raw) or three (gray) per row, forms the int8 plane values,
// transposes 4 x 4 byte blocks and writes 16 B per feature and plane (coalesced
// across lanes).  The 4 waves' column sums meet in LDS: one atomic per feature and
// block.  (One wave walking all 4 groups: 44 us for a c1 worker shard, r03s.)
template <int MODE>
__global__ __launch_bounds__(PREP_THR) void u8_prep_kernel(const uint8_t* __restrict__ X,
                                                           int64_t n, int64_t ldx, int d,
                                                           int64_t fpad, int64_t nkb,
                                                           uint8_t* __restrict__ img,
                                                           unsigned long long* __restrict__ colsum,
                                                           int nt, int* __restrict__ order) {
  constexpr int NP = MODE == DEIG_U8_GRAY3 ? 3 : 1;
  __shared__ long long cs[4][256];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  if (blockIdx.x == 0 && blockIdx.y == 0) {  // the tile order: lower triangle, row-major
    for (int i = threadIdx.x; i < nt * (nt + 1) / 2; i += PREP_THR) {
      int ti = (int)((sqrtf(8.f * (float)i + 1.f) - 1.f) * 0.5f);
      while (ti * (ti + 1) / 2 > i) --ti;
      while ((ti + 1) * (ti + 2) / 2 <= i) ++ti;
      order[i] = ti | ((i - ti * (ti + 1) / 2) << 16);
    }
  }
  const int f = blockIdx.x * 256 + lane * 4;
  const bool fin = f < d;  // d % 4 == 0: the 4 features are all in or all out
  int csum[4] = {0, 0, 0, 0};
  for (int64_t kb = blockIdx.y; kb < nkb; kb += gridDim.y) {
    {
      uint32_t rows[NP][16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = kb * KB + g * 16 + r;
        const bool ok = fin && row < n;
        if (MODE == DEIG_U8_RAW) {
          const uint32_t x = ok ? *reinterpret_cast<const uint32_t*>(X + row * ldx + f) : 0x80808080u;
          const uint32_t y = x ^ 0x80808080u;  // int8 (x - 128); padding rows -> 0
          rows[0][r] = y;
#pragma unroll
          for (int u = 0; u < 4; ++u) csum[u] += sbyte(y, u);
        } else {
          uint32_t b[3] = {0u, 0u, 0u};
          if (ok) {
            const uint32_t* p = reinterpret_cast<const uint32_t*>(X + row * ldx + 3 * (int64_t)f);
            b[0] = p[0];
            b[1] = p[1];
            b[2] = p[2];
          }
          uint32_t ph = 0, pl = 0, pw = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            int s = 0;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              const int byte = 3 * u + c;
              s += (int)((b[byte >> 2] >> (8 * (byte & 3))) & 0xffu);
            }
            const int t = ok ? s - 384 : 0;  // padding rows contribute nothing
            const int h = t >> 4, l = t & 15, w = h + l;
            csum[u] += t;
            ph |= ((uint32_t)h & 0xffu) << (8 * u);
            pl |= ((uint32_t)l & 0xffu) << (8 * u);
            pw |= ((uint32_t)w & 0xffu) << (8 * u);
          }
          rows[0][r] = ph;
          rows[NP > 1 ? 1 : 0][r] = pl;
          rows[NP > 2 ? 2 : 0][r] = pw;
        }
      }
      if (f >= fpad) continue;  // (uniform per wave: fpad % 256 == 0 or the last lanes)
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) {
        uint32_t col[4][4];  // [feature u][dword q]
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t t4[4];
          tr4(&rows[pl][4 * q], t4);
#pragma unroll
          for (int u = 0; u < 4; ++u) col[u][q] = t4[u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          *reinterpret_cast<u32x4*>(img + img_off(pl, kb, g, f + u, nkb, fpad)) =
              u32x4{col[u][0], col[u][1], col[u][2], col[u][3]};
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) cs[g][4 * lane + u] = csum[u];
  __syncthreads();
  const int t = threadIdx.x;  // feature 256 bx + t
  const int64_t ft = (int64_t)blockIdx.x * 256 + t;
  if (ft < d) {
    const long long v = ((cs[0][t] + cs[1][t]) + cs[2][t]) + cs[3][t];
    atomicAdd(colsum + ft, (unsigned long long)v);
  }
}

struct U8Sched {
  const uint8_t* img;
  unsigned long long* G;  // planes x fpad x fpad int64 (two's complement), lower tiles
  const int* order;       // lower tile list: ti | tj << 16
  int64_t nkb, fpad;
  int T, nseg;
  // direct epilogue (raw mode, one K segment): S written from the accumulators
  const unsigned long long* colsum;
  int64_t d, n, div, lds, lds64;
  double alpha;
  float* S;
  double* S64;
};

// One item = (plane, lower tile, K segment).  LDS: 2 stages x (A panel, B panel),
// each panel = 4 row groups x 128 features x 16 B = 8 KiB, the same bytes as the
// image's [kb][g][f0 .. f0+127] runs.  Wave (wi, wj) owns rows 64 wi.. and columns
// 64 wj.. of the tile: 4 x 4 MFMA blocks, lane l reads the A fragment of feature
// 16 a + (l & 15), row group l >> 4 (16 consecutive rows = 16 bytes).
// DIRECT (raw mode, the whole K range in one item: n <= 65536 rows, so the int32
// accumulators are the exact sums): the epilogue adds the mean terms in int64,
// scales once in double (as u8_finalize_kernel) and stores S[i][j] and S[j][i] -
// no int64 image, no memset, no atomics, no finalize pass (c1 worker shard: the
// image path's memset + atomics + finalize were most of its 0.30 ms, r03s).
template <bool DIRECT>
__global__ __launch_bounds__(SYRK_THR, 2) void u8_syrk_kernel(U8Sched s) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[2][2][4 * TB * 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = tid >> 6, wi = wave >> 1, wj = wave & 1;
  const int item = blockIdx.x;
  const int plane = blockIdx.y;
  const int tile = item % s.T, seg = item / s.T;
  const int tt = s.order[tile];
  const int ti = tt & 0xffff, tj = tt >> 16;
  const bool diag = ti == tj;
  const bool active = !(diag && wi < wj);  // the upper block of a diagonal tile is a mirror
  const int64_t k0 = s.nkb * seg / s.nseg, k1 = s.nkb * (seg + 1) / s.nseg;
  const int64_t i0 = (int64_t)ti * TB, j0 = (int64_t)tj * TB;

  // staging: thread t moves 16 B chunks c = t and t + 256 of each panel (512 chunks
  // = 4 groups x 128 features)
  auto load = [&](int64_t kb, u32x4 (&ra)[2], u32x4 (&rb)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = tid + h * SYRK_THR;
      const int g = c >> 7, fl = c & 127;
      // (unconditional: a diagonal tile loads its panel twice - a branch around the B
      // loads would make the compiler's counted waits conservative)
      ra[h] = *reinterpret_cast<const u32x4*>(s.img + img_off(plane, kb, g, i0 + fl, s.nkb, s.fpad));
      rb[h] = *reinterpret_cast<const u32x4*>(s.img + img_off(plane, kb, g, j0 + fl, s.nkb, s.fpad));
    }
  };
  auto put = [&](int st, const u32x4 (&ra)[2], const u32x4 (&rb)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = tid + h * SYRK_THR;
      *reinterpret_cast<u32x4*>(&lds[st][0][c * 16]) = ra[h];
      *reinterpret_cast<u32x4*>(&lds[st][1][c * 16]) = rb[h];
    }
  };

  i32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = i32x4{0, 0, 0, 0};

  if (k0 >= k1) return;  // (whole block: an empty K segment adds nothing)
  // K loop: LDS double buffer fed from a PF-deep register ring - the loads of k-step
  // kk + PF are issued while kk's MFMAs run, so each load has PF - 1 steps to land
  // (one step ahead, a c1 worker shard took 149 us: every step waited out a global
  // load latency).  Loads are unpredicated (clamped to the last k-step) so that the
  // compiler's counted waits keep the ring in flight; PF even: stage = u & 1.
  constexpr int PF = 4;
  u32x4 ra[PF][2], rb[PF][2];
  auto clampk = [&](int64_t kb) { return kb < k1 ? kb : k1 - 1; };
#pragma unroll
  for (int u = 0; u < PF; ++u) load(clampk(k0 + u), ra[u], rb[u]);
  put(0, ra[0], rb[0]);
  __syncthreads();
  const int g = lane >> 4, c = lane & 15;
  auto body = [&](int64_t kk, int u) {
    load(clampk(kk + PF), ra[u], rb[u]);  // slot u's k-step is already in LDS
    const int st = u & 1;
    if (active) {
      const uint8_t* pa = &lds[st][0][0];
      const uint8_t* pb = diag ? pa : &lds[st][1][0];
      i32x4 fa[4], fb[4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
        fa[a] = *reinterpret_cast<const i32x4*>(pa + (g * TB + 64 * wi + 16 * a + c) * 16);
#pragma unroll
      for (int b = 0; b < 4; ++b)
        fb[b] = *reinterpret_cast<const i32x4*>(pb + (g * TB + 64 * wj + 16 * b + c) * 16);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[a], fb[b], acc[a][b], 0, 0, 0);
    }
    put(st ^ 1, ra[(u + 1) % PF], rb[(u + 1) % PF]);  // k-step kk + 1 (a clamped copy past k1)
    __syncthreads();
  };
  int64_t kb = k0;
  for (; kb + PF <= k1; kb += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) body(kb + u, u);
  }
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (kb + u < k1) body(kb + u, u);
  if (!DIRECT && !active) return;  // (the direct epilogue has barriers: every wave stays)
  // C/D map (gfx950, dtype independent): column = lane & 15, row = 4 (lane >> 4) + reg
  if constexpr (DIRECT) {
    // every column sum loaded up front at clamped indices (a load inside the i < d
    // branch waited out its latency alone: 16 serialised loads per wave)
    long long cjv[4], civ[4][4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int64_t j = j0 + 64 * wj + 16 * b + (lane & 15);
      cjv[b] = (long long)s.colsum[j < s.d ? j : s.d - 1];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t i = i0 + 64 * wi + 16 * a + 4 * (lane >> 4) + r;
        civ[a][r] = (long long)s.colsum[i < s.d ? i : s.d - 1];
      }
    // values of this wave's 64 x 64 block (float for S; S64 stored here, scattered)
    float vf[4][4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t i = i0 + 64 * wi + 16 * a + 4 * (lane >> 4) + r;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int64_t j = j0 + 64 * wj + 16 * b + (lane & 15);
          const long long v64 =
              (long long)acc[a][b][r] + 128ll * (civ[a][r] + cjv[b]) + 16384ll * s.n;
          const double v = s.div > 0 ? (double)v64 / (double)s.div : s.alpha * (double)v64;
          vf[a][b][r] = (float)v;
          if (s.S64 && active && i < s.d && j < s.d && !(diag && j > i)) {
            s.S64[i * s.lds64 + j] = v;
            s.S64[j * s.lds64 + i] = v;
          }
        }
      }
    if (s.S) {
      // S[i][j]: 16 consecutive j per row and instruction
      if (active)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int64_t i = i0 + 64 * wi + 16 * a + 4 * (lane >> 4) + r;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const int64_t j = j0 + 64 * wj + 16 * b + (lane & 15);
              if (i < s.d && j < s.d && !(diag && j > i)) s.S[i * s.lds + j] = vf[a][b][r];
            }
          }
      // the mirror S[j][i] through LDS, one 64-row half of the tile at a time: the
      // stage buffers (32 KiB, free after the K loop's last barrier) hold the half as
      // 64 x 128 floats, columns XOR-swizzled by the row; then 16 threads per S row
      // write 64 contiguous floats (float4 each).  (Stored straight from the
      // accumulators, every mirror instruction scattered 4-byte writes over 64 rows:
      // r04 A/B in one process on the c1 worker shard, 99.7 vs 102.5 us per covariance,
      // bit-identical, profiles/r04b_u8_mirror_ab.log.)
      float* T = reinterpret_cast<float*>(&lds[0][0][0]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (active && wi == h)
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int il = 16 * a + 4 * (lane >> 4) + r;
#pragma unroll
              for (int b = 0; b < 4; ++b) {
                const int jl = 64 * wj + 16 * b + (lane & 15);
                T[il * 128 + (jl ^ (il & 31))] = vf[a][b][r];
              }
            }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int task = it * SYRK_THR + tid;  // (S row j0 + jl, rows i4 .. i4 + 3 of the half)
          const int jl = task >> 4, i4 = (task & 15) * 4;
          const int64_t j = j0 + jl;
          const int64_t ib = i0 + 64 * h + i4;
          if (j < s.d) {
            float x[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] = T[(i4 + e) * 128 + (jl ^ ((i4 + e) & 31))];
            float* dst = s.S + j * s.lds + ib;
            if (!diag && ib + 3 < s.d && (reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
              *reinterpret_cast<f32x4*>(dst) = f32x4{x[0], x[1], x[2], x[3]};
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (ib + e < s.d && (!diag || j < ib + e)) dst[e] = x[e];
            }
          }
        }
        __syncthreads();
      }
    }
    return;
  }
  unsigned long long* Gp = s.G + (int64_t)plane * s.fpad * s.fpad;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t i = i0 + 64 * wi + 16 * a + 4 * (lane >> 4) + r;
        const int64_t j = j0 + 64 * wj + 16 * b + (lane & 15);
        if (diag && j > i) continue;
        atomicAdd(Gp + i * s.fpad + j, (unsigned long long)(long long)acc[a][b][r]);
      }
}

// One thread per S entry: the lower-triangle value of (max(i,j), min(i,j)) from
// the exact int64 sums, scaled in double, stored to both triangles.  div > 0 (alpha
// == 1/n, the reference's /= n): v = a / (div * 9 for gray), ONE rounding of the
// exact quotient (div * 9 is exact); else alpha * a (/ 9).  The fp32 S is that
// double rounded to float: the correctly rounded value except in the ~2^-29 of
// cases where the double lands on a float tie (then 1 ulp).
template <int MODE>
__global__ __launch_bounds__(256) void u8_finalize_kernel(const unsigned long long* __restrict__ G,
                                                          const unsigned long long* __restrict__ colsum,
                                                          int64_t fpad, int64_t d, int64_t n,
                                                          double alpha, int64_t div,
                                                          float* __restrict__ S,
                                                          int64_t lds, double* __restrict__ S64,
                                                          int64_t lds64) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * d) return;
  const int64_t r = idx / d, c = idx - r * d;
  const int64_t i = r > c ? r : c, j = r > c ? c : r;
  const long long ci = (long long)colsum[i], cj = (long long)colsum[j];
  long long a;
  double v;
  if (MODE == DEIG_U8_RAW) {
    a = (long long)G[i * fpad + j] + 128ll * (ci + cj) + 16384ll * n;
    v = div > 0 ? (double)a / (double)div : alpha * (double)a;
  } else {
    const int64_t pl = fpad * fpad;
    const long long phh = (long long)G[i * fpad + j];
    const long long pll = (long long)G[pl + i * fpad + j];
    const long long pww = (long long)G[2 * pl + i * fpad + j];
    a = 240ll * phh + 16ll * pww - 15ll * pll + 384ll * (ci + cj) + 147456ll * n;
    v = div > 0 ? (double)a / (9.0 * (double)div) : alpha * (double)a / 9.0;
  }
  if (S) S[r * lds + c] = (float)v;
  if (S64) S64[r * lds64 + c] = v;
}

struct U8Layout {
  int64_t fpad, nkb, nt, T;
  int planes;
  size_t off_order, off_col, off_G, off_img, total;
};

U8Layout u8_layout(int64_t n, int64_t d, int mode) {
  U8Layout L;
  L.planes = u8_planes(mode);
  L.fpad = cdiv(d, FPAD) * FPAD;
  L.nkb = cdiv(n, KB);
  L.nt = L.fpad / TB;
  L.T = L.nt * (L.nt + 1) / 2;
  size_t off = 0;
  L.off_order = off;
  off = align_up(off + sizeof(int) * (size_t)L.T, 256);
  L.off_col = off;
  off = align_up(off + sizeof(unsigned long long) * (size_t)L.fpad, 256);
  L.off_G = off;
  off = align_up(off + sizeof(unsigned long long) * (size_t)L.planes * L.fpad * L.fpad, 256);
  L.off_img = off;
  off += (size_t)L.planes * L.nkb * KB * L.fpad;
  L.total = off;
  return L;
}

}  // namespace

size_t syrk_u8_workspace_bytes(int64_t n, int64_t d, int mode) {
  if (n < 1 || d < 1) return 0;
  return u8_layout(n, d, mode).total;
}

int syrk_u8_launch(const uint8_t* X, int64_t n, int64_t d, int64_t ldx, int mode, double alpha,
                   float* S, int64_t lds, double* S64, int64_t lds64, void* ws, size_t ws_bytes,
                   hipStream_t stream) {
  DEIG_REQUIRE(mode == DEIG_U8_RAW || mode == DEIG_U8_GRAY3, "syrk_u8: unknown mode %d", mode);
  DEIG_REQUIRE(n >= 1, "syrk_u8: n must be >= 1 (got %lld)", (long long)n);
  DEIG_REQUIRE(d >= 4 && d % 4 == 0 && d <= (1 << 15),
               "syrk_u8: d must be a multiple of 4 in [4, 32768] (got %lld)", (long long)d);
  const int64_t need = mode == DEIG_U8_RAW ? d : 3 * d;
  DEIG_REQUIRE(ldx >= need && ldx % 4 == 0, "syrk_u8: ldx must be >= %lld bytes and a multiple of 4",
               (long long)need);
  DEIG_REQUIRE(X && (reinterpret_cast<uintptr_t>(X) & 3u) == 0, "syrk_u8: X must be 4-byte aligned");
  DEIG_REQUIRE(S || S64, "syrk_u8: need S and/or S64");
  DEIG_REQUIRE(!S || lds >= d, "syrk_u8: lds must be >= d");
  DEIG_REQUIRE(!S64 || lds64 >= d, "syrk_u8: lds64 must be >= d");
  DEIG_REQUIRE(n <= (int64_t(1) << 40), "syrk_u8: n too large");
  const U8Layout L = u8_layout(n, d, mode);
  if (!ws || ws_bytes < L.total)
    return fail(DEIG_EWORKSPACE, "syrk_u8: workspace %zu bytes < required %zu", ws_bytes, L.total);
  char* base = static_cast<char*>(ws);
  int* order = reinterpret_cast<int*>(base + L.off_order);
  unsigned long long* col = reinterpret_cast<unsigned long long*>(base + L.off_col);
  unsigned long long* G = reinterpret_cast<unsigned long long*>(base + L.off_G);
  uint8_t* img = reinterpret_cast<uint8_t*>(base + L.off_img);
  const int G_ = num_cus();
  // direct epilogue: raw mode, one K segment (int32 exact), enough tiles to fill half
  // the chip (config 1: 300 tiles of a 3072-feature worker shard)
  const bool direct = mode == DEIG_U8_RAW && L.nkb <= MAX_SEG_KB && 2 * L.T >= G_;
  DEIG_HIP_CHECK(hipMemsetAsync(col, 0, sizeof(unsigned long long) * L.fpad, stream));
  if (!direct)
    DEIG_HIP_CHECK(hipMemsetAsync(G, 0, sizeof(unsigned long long) * L.planes * L.fpad * L.fpad, stream));
  const int yb = (int)(L.nkb < PREP_YB ? L.nkb : PREP_YB);
  const dim3 pg((unsigned)(L.fpad / 256 + (L.fpad % 256 ? 1 : 0)), (unsigned)yb);
  if (mode == DEIG_U8_RAW)
    hipLaunchKernelGGL(u8_prep_kernel<DEIG_U8_RAW>, pg, dim3(PREP_THR), 0, stream, X, n, ldx,
                       (int)d, L.fpad, L.nkb, img, col, (int)L.nt, order);
  else
    hipLaunchKernelGGL(u8_prep_kernel<DEIG_U8_GRAY3>, pg, dim3(PREP_THR), 0, stream, X, n, ldx,
                       (int)d, L.fpad, L.nkb, img, col, (int)L.nt, order);
  DEIG_HIP_CHECK(hipGetLastError());
  // K segments: enough items to fill the chip twice over, each <= MAX_SEG_KB row
  // blocks (int32 accumulators) and >= 4 (amortise the staging prologue).
  int64_t nseg = direct ? 1 : cdiv(2 * G_, L.T * L.planes);
  const int64_t min_seg = cdiv(L.nkb, MAX_SEG_KB);
  if (nseg < min_seg) nseg = min_seg;
  if (!direct && nseg > cdiv(L.nkb, 4)) nseg = cdiv(L.nkb, 4) > min_seg ? cdiv(L.nkb, 4) : min_seg;
  if (nseg < 1) nseg = 1;
  U8Sched s;
  s.img = img;
  s.G = G;
  s.order = order;
  s.nkb = L.nkb;
  s.fpad = L.fpad;
  s.T = (int)L.T;
  s.nseg = (int)nseg;
  const int64_t div = (alpha == 1.0 / (double)n && n < (int64_t(1) << 48)) ? n : 0;
  s.colsum = col;
  s.d = d;
  s.n = n;
  s.div = div;
  s.alpha = alpha;
  s.S = S;
  s.lds = lds;
  s.S64 = S64;
  s.lds64 = lds64;
  if (direct) {
    hipLaunchKernelGGL(u8_syrk_kernel<true>, dim3((unsigned)L.T, 1u), dim3(SYRK_THR), 0, stream, s);
    DEIG_HIP_CHECK(hipGetLastError());
    return DEIG_OK;
  }
  hipLaunchKernelGGL(u8_syrk_kernel<false>, dim3((unsigned)(L.T * nseg), (unsigned)L.planes),
                     dim3(SYRK_THR), 0, stream, s);
  DEIG_HIP_CHECK(hipGetLastError());
  const dim3 fg((unsigned)cdiv(d * d, 256));
  if (mode == DEIG_U8_RAW)
    hipLaunchKernelGGL(u8_finalize_kernel<DEIG_U8_RAW>, fg, dim3(256), 0, stream, G, col, L.fpad, d,
                       n, alpha, div, S, lds, S64, lds64);
  else
    hipLaunchKernelGGL(u8_finalize_kernel<DEIG_U8_GRAY3>, fg, dim3(256), 0, stream, G, col, L.fpad,
                       d, n, alpha, div, S, lds, S64, lds64);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

}  // namespace deig
