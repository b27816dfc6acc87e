// Covariance SYRK on CDNA4 fp32 MFMA:  S = alpha * X^T X  (X: n x d row-major).
//
// Replaces SlaveNode.compute_sigma_hat_ (distributed.py:59-70), whose
// np.dot(x.T, x) on a transposed view lands in OpenBLAS dsyrk: one triangle is
// computed and mirrored, so the result is bit-exactly symmetric.  Same here:
// only lower-triangle 256x256 tiles are computed; off-diagonal tiles are written
// twice (tile + transpose) from the same registers.
//
// Kernel shape (one 512-thread workgroup per CU, 8 waves as 2 (i) x 4 (j)):
//   * tile 256 (i) x 256 (j); wave tile 128 x 64 = 4 x 2 blocks of
//     v_mfma_f32_32x32x2_f32 (exact f32 fma chain, 64 FLOP/clk/SIMD);
//   * K-tile = 32 rows of X.  The two 256-column panels of those rows (1 KiB per
//     row) are DMA'd HBM -> LDS with buffer_load ... lds (16 B per lane, one row
//     per wave-instruction, out-of-range rows/columns read as 0 through the
//     buffer descriptor's range check); two LDS buffers = 128 KiB;
//   * operand reads: the wave's 128 i-columns are interleaved so that lane l's
//     four MFMA blocks read 4 consecutive floats (one ds_read_b128, conflict
//     free) and its two j-blocks read 2 consecutive floats (one ds_read_b64):
//     block mb row r <-> i = 4r + mb, block nb col c <-> j = 2c + nb.
//
// Work decomposition over G = #CU persistent blocks (no atomics, deterministic):
//   T = nt(nt+1)/2 lower tiles, q = T / G, R = T % G.
//   phase m < q : block b computes tile m*G + xcd(b) over all K  -> direct store
//   remainder   : the R*NK (tile, K-tile) work items are cut into G equal
//                 contiguous ranges; each block's range spans <= 2 tiles, whose
//                 fp32 partials go to slab slots 2b, 2b+1; syrk_reduce_kernel sums
//                 a tile's slabs in block order, scales, and stores both triangles.
// In a phase every block walks the same rows of X at the same pace, so a row
// panel is fetched from HBM once and re-read by the other ~T/nt tiles from
// L2 / Infinity Cache.
#include "deig_internal.hpp"

namespace deig {
namespace {

constexpr int BT = 256;          // tile edge
constexpr int BK = 32;           // rows of X per K-tile
constexpr int NTHR = 512;        // 8 waves
constexpr int PANEL = BK * BT;   // floats per panel buffer (32 KiB)
constexpr int SLAB = BT * BT;    // floats per partial slab (256 KiB)
// The MFMA accumulators are flushed into an fp32 slab every FLUSH_KT K-tiles
// (4096 rows): a plain fp32 chain over all n rows would carry ~eps*sqrt(n/3)
// relative error on the diagonal (5e-5 at n = 2^21); two-level summation keeps
// it ~2e-6 and stays deterministic.
constexpr int FLUSH_KT = 128;

struct Sched {
  const float* X;
  float* S;
  float* part;   // 2 remainder slabs per block
  float* accs;   // 1 flush slab per block (phase tiles)
  int64_t n, ldx, lds;
  int64_t NK;  // K-tiles per tile
  int64_t Wr;  // remainder work items (R * NK)
  int d, nt, T, G, q, R;
  float alpha;
};

__device__ __forceinline__ void tile_coords(int t, int& ti, int& tj) {
  int r = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
  while (r * (r + 1) / 2 > t) --r;
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  ti = r;
  tj = t - r * (r + 1) / 2;
}

// First block whose remainder range contains work position pos.
__device__ __forceinline__ int64_t block_of(int64_t pos, int64_t Wr, int G) {
  return ((pos + 1) * (int64_t)G + Wr - 1) / Wr - 1;
}

typedef int i32x4 __attribute__((ext_vector_type(4)));

// Raw buffer descriptor (gfx950): base, stride 0, num_records bytes, dword format.
__device__ __forceinline__ i32x4 make_rsrc(const void* base, int nrec) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  i32x4 r;
  r[0] = (int)(uint32_t)a;
  r[1] = (int)((uint32_t)(a >> 32) & 0xffffu);
  r[2] = nrec;
  r[3] = 0x00020000;
  return r;
}

// buffer_load_dwordx4 ... lds: 16 B per lane into LDS at (m0 + 16 * lane).
// Issued from inline asm on purpose: hipcc cannot tell which LDS bytes an
// LDS-DMA writes and would otherwise put vmcnt(0) in front of every ds_read of
// the *other* buffer, serialising the prefetch with the MFMA loop.  The only
// wait on these loads is the explicit vmcnt(0) before the K-tile barrier.
__device__ __forceinline__ void dma16(i32x4 rsrc, int voff, const float* lds_dst) {
  const unsigned m0v = (unsigned)(uintptr_t)(lds_void*)lds_dst;
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :
               : "v"(voff), "s"(rsrc), "s"(m0v)
               : "memory", "m0");
}

// DMA the two 256-column panels of K-tile kt into LDS.  One buffer descriptor
// per K-tile (SGPRs) whose range ends after the last valid row, so rows >= n and
// the over-read past the end of X return 0.  Only the lane offset lives in a
// VGPR; it is laundered through an empty asm so the per-row offsets are
// recomputed here instead of being hoisted (and held) across the K loop.
__device__ __forceinline__ void stage(const Sched& s, int64_t kt, int i0, int j0, bool diag,
                                      float* A, float* B, int wave, int lane16) {
  const int64_t r0 = kt * BK;
  int64_t rows = s.n - r0;
  rows = rows < BK ? rows : BK;
  const i32x4 rsrc = make_rsrc(s.X + r0 * s.ldx, (int)(rows * s.ldx * 4));
  int l16 = lane16;
  asm volatile("" : "+v"(l16));
#pragma unroll
  for (int rr = 0; rr < BK / 8; ++rr) {
    const int row = wave * (BK / 8) + rr;
    const int base = (int)(row * s.ldx) * 4;
    dma16(rsrc, l16 + base + i0 * 4, A + row * BT);
    if (!diag) dma16(rsrc, l16 + base + j0 * 4, B + row * BT);
  }
}

__device__ __forceinline__ void kt_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

__device__ __forceinline__ void compute(const float* A, const float* B, f32x16 (&acc)[4][2],
                                        int wi, int wj, int lane) {
  const int c = lane & 31, h = lane >> 5;
  const float* pa = A + h * BT + 128 * wi + 4 * c;
  const float* pb = B + h * BT + 64 * wj + 2 * c;
#pragma unroll
  for (int ks = 0; ks < BK / 2; ++ks) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(pa + 2 * ks * BT);
    const f32x2 b = *reinterpret_cast<const f32x2*>(pb + 2 * ks * BT);
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
        acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mb], b[nb], acc[mb][nb], 0, 0, 0);
    }
  }
}

__device__ __forceinline__ float* slab_ptr(float* slab, int wave, int mb, int nb, int g, int lane) {
  return slab + ((((wave * 4 + mb) * 2 + nb) * 4 + g) * 64 + lane) * 4;
}

// acc (+ slab if !first) -> slab; acc = 0.  Register-order image, 16 B per lane.
__device__ __forceinline__ void flush(float* slab, bool first, f32x16 (&acc)[4][2], int wave,
                                      int lane) {
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4* ptr = reinterpret_cast<f32x4*>(slab_ptr(slab, wave, mb, nb, g, lane));
        f32x4 v = {acc[mb][nb][4 * g], acc[mb][nb][4 * g + 1], acc[mb][nb][4 * g + 2],
                   acc[mb][nb][4 * g + 3]};
        if (!first) v += *ptr;
        *ptr = v;
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[mb][nb][4 * g + e] = 0.f;
      }
}

// acc += slab (the flushed part of this segment), before the epilogue.
__device__ __forceinline__ void unflush(const float* slab, f32x16 (&acc)[4][2], int wave,
                                        int lane) {
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(slab_ptr(const_cast<float*>(slab), wave, mb, nb, g, lane));
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[mb][nb][4 * g + e] += v[e];
      }
}

// One (tile, K-range) segment.  mode 0: direct store (full K); mode 1: partial slab.
__device__ void segment(const Sched& s, float* lds, int tile, int64_t k0, int64_t k1, int slot,
                        bool partial) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wi = wave >> 2, wj = wave & 3;
  const int lane16 = lane * 16;
  int ti, tj;
  tile_coords(tile, ti, tj);
  const int i0 = ti * BT, j0 = tj * BT;
  const bool diag = (ti == tj);

  f32x16 acc[4][2];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mb][nb][r] = 0.0f;

  // LDS: [buf][A|B][BK][BT]; buffer toggled by a scalar offset.
  float* slab = partial ? s.part + (int64_t)slot * SLAB : s.accs + (int64_t)blockIdx.x * SLAB;
  bool flushed = false;
  if (k0 < k1) {
    stage(s, k0, i0, j0, diag, lds, lds + PANEL, wave, lane16);
    kt_barrier();
    int cur = 0;
    int since = 0;
    for (int64_t kt = k0; kt < k1; ++kt) {
      float* Ac = lds + cur * (2 * PANEL);
      float* An = lds + (cur ^ 1) * (2 * PANEL);
      if (kt + 1 < k1) stage(s, kt + 1, i0, j0, diag, An, An + PANEL, wave, lane16);
      compute(Ac, diag ? Ac : Ac + PANEL, acc, wi, wj, lane);
      if (++since == FLUSH_KT && kt + 1 < k1) {
        flush(slab, !flushed, acc, wave, lane);
        flushed = true;
        since = 0;
      }
      kt_barrier();
      cur ^= 1;
    }
  }
  if (flushed) unflush(slab, acc, wave, lane);

  const int c = lane & 31, h = lane >> 5;
  if (partial) {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 v = {acc[mb][nb][4 * g], acc[mb][nb][4 * g + 1], acc[mb][nb][4 * g + 2],
                     acc[mb][nb][4 * g + 3]};
          *reinterpret_cast<f32x4*>(slab + ((((wave * 4 + mb) * 2 + nb) * 4 + g) * 64 + lane) * 4) =
              v;
        }
    return;
  }

  const float al = s.alpha;
  const int d = s.d;
  // row-major store S[i][j..j+1]
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rho = (r & 3) + 8 * (r >> 2) + 4 * h;
      const int i = i0 + 128 * wi + 4 * rho + mb;
      const int j = j0 + 64 * wj + 2 * c;
      if (i < d && j < d) {
        f32x2 v = {al * acc[mb][0][r], al * acc[mb][1][r]};
        *reinterpret_cast<f32x2*>(s.S + (int64_t)i * s.lds + j) = v;
      }
    }
  if (!diag) {
    // mirror S[j][i..i+3]
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rho = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int ib = i0 + 128 * wi + 4 * rho;
        const int j = j0 + 64 * wj + 2 * c + nb;
        if (ib < d && j < d) {
          f32x4 v = {al * acc[0][nb][r], al * acc[1][nb][r], al * acc[2][nb][r],
                     al * acc[3][nb][r]};
          *reinterpret_cast<f32x4*>(s.S + (int64_t)j * s.lds + ib) = v;
        }
      }
  }
}

__global__ __launch_bounds__(NTHR, 2) void syrk_kernel(Sched s) {
  __shared__ __attribute__((aligned(16))) float lds[4 * PANEL];
  const int b = blockIdx.x;
  const int L = xcd_logical(b, s.G);
  int64_t pos = 0, end = 0;
  if (s.R > 0) {
    pos = (int64_t)b * s.Wr / s.G;
    end = (int64_t)(b + 1) * s.Wr / s.G;
  }
  int m = 0, seg = 0;
  // One call site for segment(): phases first, then the remainder ranges.
  for (;;) {
    int tile, slot = 0;
    int64_t k0, k1;
    bool partial;
    if (m < s.q) {
      tile = m * s.G + L;
      k0 = 0;
      k1 = s.NK;
      partial = false;
      ++m;
    } else if (pos < end) {
      const int64_t r = pos / s.NK;
      k0 = pos - r * s.NK;
      k1 = k0 + (end - pos);
      if (k1 > s.NK) k1 = s.NK;
      tile = s.q * s.G + (int)r;
      slot = 2 * b + seg;
      partial = true;
      pos += k1 - k0;
      ++seg;
    } else {
      break;
    }
    segment(s, lds, tile, k0, k1, slot, partial);
  }
}

// grid (R, SLAB/4/256): one thread per float4 of a remainder tile's slab image.
__global__ __launch_bounds__(256) void syrk_reduce_kernel(Sched s) {
  const int r = blockIdx.x;
  const int f = blockIdx.y * 256 + threadIdx.x;  // float4 index in slab image
  const int lane = f & 63, g = (f >> 6) & 3, nb = (f >> 8) & 1, mb = (f >> 9) & 3, wave = f >> 11;
  const int wi = wave >> 2, wj = wave & 3, c = lane & 31, h = lane >> 5;
  int ti, tj;
  tile_coords(s.q * s.G + r, ti, tj);
  const bool diag = (ti == tj);

  const int64_t pos0 = (int64_t)r * s.NK, pos1 = pos0 + s.NK;
  const int64_t bf = block_of(pos0, s.Wr, s.G), bl = block_of(pos1 - 1, s.Wr, s.G);
  f32x4 sum = {0.f, 0.f, 0.f, 0.f};
  for (int64_t b = bf; b <= bl; ++b) {
    const int64_t sb = b * s.Wr / s.G, eb = (b + 1) * s.Wr / s.G;
    if (eb <= sb || eb <= pos0 || sb >= pos1) continue;
    const int64_t slot = 2 * b + (sb < pos0 ? 1 : 0);
    sum += *reinterpret_cast<const f32x4*>(s.part + slot * SLAB + (int64_t)f * 4);
  }
  const int i0 = ti * BT, j0 = tj * BT;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int rho = u + 8 * g + 4 * h;
    const int i = i0 + 128 * wi + 4 * rho + mb;
    const int j = j0 + 64 * wj + 2 * c + nb;
    if (i < s.d && j < s.d) {
      const float v = s.alpha * sum[u];
      s.S[(int64_t)i * s.lds + j] = v;
      if (!diag) s.S[(int64_t)j * s.lds + i] = v;
    }
  }
}

void make_sched(Sched& s, int64_t n, int64_t d, int G) {
  s.n = n;
  s.d = (int)d;
  s.nt = (int)cdiv(d, BT);
  s.T = s.nt * (s.nt + 1) / 2;
  s.G = G;
  s.q = s.T / G;
  s.R = s.T % G;
  s.NK = cdiv(n, BK);
  s.Wr = (int64_t)s.R * s.NK;
}

}  // namespace

// [G flush slabs][2G remainder slabs]
static size_t ws_bytes_for(const Sched& s) {
  return (size_t)(s.R > 0 ? 3 : 1) * s.G * SLAB * sizeof(float);
}

size_t syrk_workspace_bytes(int64_t n, int64_t d) {
  Sched s;
  make_sched(s, n, d, num_cus());
  return ws_bytes_for(s);
}

int syrk_launch(const float* X, int64_t n, int64_t d, int64_t ldx, float alpha, float* S,
                int64_t lds, void* ws, size_t ws_bytes, hipStream_t stream) {
  DEIG_REQUIRE(n >= 1, "syrk: n must be >= 1 (got %lld)", (long long)n);
  DEIG_REQUIRE(d >= 1 && d % 4 == 0, "syrk: d must be a positive multiple of 4 (got %lld)",
               (long long)d);
  DEIG_REQUIRE(d <= (1 << 20), "syrk: d too large (%lld)", (long long)d);
  DEIG_REQUIRE(ldx >= d && ldx % 4 == 0, "syrk: ldx must be >= d and a multiple of 4");
  DEIG_REQUIRE(lds >= d && lds % 4 == 0, "syrk: lds must be >= d and a multiple of 4");
  DEIG_REQUIRE((int64_t)BK * ldx * 4 < 0x7fffffffLL, "syrk: ldx too large for 32-bit offsets");
  DEIG_REQUIRE(X && S && aligned16(X) && aligned16(S), "syrk: X and S must be 16-byte aligned");
  Sched s;
  make_sched(s, n, d, num_cus());
  s.X = X;
  s.S = S;
  s.ldx = ldx;
  s.lds = lds;
  s.alpha = alpha;
  const size_t need = ws_bytes_for(s);
  if (ws_bytes < need || !ws)
    return fail(DEIG_EWORKSPACE, "syrk: workspace %zu bytes < required %zu", ws_bytes, need);
  s.accs = static_cast<float*>(ws);
  s.part = s.accs + (size_t)s.G * SLAB;
  hipLaunchKernelGGL(syrk_kernel, dim3(s.G), dim3(NTHR), 0, stream, s);
  DEIG_HIP_CHECK(hipGetLastError());
  if (s.R > 0) {
    hipLaunchKernelGGL(syrk_reduce_kernel, dim3(s.R, SLAB / 4 / 256), dim3(256), 0, stream, s);
    DEIG_HIP_CHECK(hipGetLastError());
  }
  return DEIG_OK;
}

}  // namespace deig
