// Covariance SYRK on CDNA4 bf16 MFMA with split fp32 operands ("split3"):
//   S = alpha * X^T X  (+ S if accumulating),  X: n x d fp32 row-major.
//
// Replaces SlaveNode.compute_sigma_hat_ (distributed.py:59-70; np.dot(x.T, x)
// on a transposed view -> OpenBLAS dsyrk, then /= n).  gfx950 has no xf32 MFMA
// and its f32 MFMA runs at 1/16 of the bf16 rate, so every fp32 sample is split
// once into x = hi + lo (hi = bf16(x), lo = bf16(x - hi); |x - hi - lo| <=
// 2^-17 |x|) and each product is formed from three bf16 MFMA products
//   x_a x_b ~ hi_a hi_b + hi_a lo_b + lo_a hi_b
// accumulated in fp32 (the bf16 products are exact in fp32).  The dropped
// lo_a lo_b term is ~2^-18 |x_a x_b|: negligible off the diagonal (zero-mean
// rounding residues), but it biases the diagonal by ~-3e-6 relative, so the
// split pass also accumulates sum_k lo_ik^2 per feature and a last kernel adds it
// to S[i][i].  Net error vs float64 ~1e-7 * max|S|, the same order as the
// fp32-MFMA kernel (syrk.hip), at 16/3 x its MFMA rate.
//
// Pipeline per row chunk (bounded workspace; chunks accumulate into S):
//   split_kernel   X (fp32, HBM) -> XP: bf16 hi/lo image in MFMA operand order,
//                  [32-row block][256-feature panel][slice = (octet, hi|lo)]
//                  [feature][8 rows] - a panel's K-tile is 32 contiguous KiB -
//                  rows padded with zeros to a multiple of 32, + lo^2 partials;
//   syrks_h_kernel persistent, one 512-thread block per CU, 256 x 256 lower
//                  tiles, v_mfma_f32_16x16x32_bf16, K-tile = 32 rows whose two
//                  panels (32 KiB each: 4 octets x {hi, lo} x 256 features x 16 B)
//                  are DMA'd L2/HBM -> LDS with buffer_load ... lds into two
//                  ring buffers restaged half a K-tile at a time (segment_h: 2
//                  phases per K-tile, waves 4-7 one barrier behind, counted
//                  vmcnt + raw s_barrier); conflict-free ds_read_b128 reads;
//                  (the r02-r03 K loops syrks_st_kernel / syrks_q_kernel / the
//                  non-fused syrks_kernel: ab/syrk_split_superseded.inc, A/B
//                  builds only)
//   syrks_reduce   split-K remainder tiles, summed in block order (deterministic);
//   diag_corr      S[i][i] += alpha * sum lo_i^2.
// Tile order: 8 x 4 super-tiles of the lower triangle, so the ~32 tiles an XCD
// runs concurrently share few panels in its L2.  Work decomposition (no
// atomics): q = T / G full phases of one tile per block; the R = T mod G
// remainder tiles are cut into nseg equal K segments run K-synchronously
// (segment-major item order) and summed in segment order by syrks_reduce.
#include <cmath>
#include <cstdlib>

#include "deig_internal.hpp"

namespace deig {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Two fp32 -> packed bf16 (element 0 in the low half), round to nearest even:
// one v_cvt_pk_bf16_f32.
__device__ __forceinline__ uint32_t cvt2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
__device__ __forceinline__ float lo_f(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float hi_f(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }

constexpr int BT = 256;                      // tile edge (features)
constexpr int ROWS_PAD = 32;                 // chunk rows are padded to this (2 k-steps)
constexpr int NTHR = 512;                    // 8 waves: 2 (i) x 4 (j), wave tile 128 x 64
constexpr int SLICE_B = BT * 16;             // (octet, hi|lo) slice of a panel: 4 KiB
constexpr int SLAB = BT * BT;                // floats per partial slab
constexpr int SPLIT_YB = 256;                // row groups of the split pass
constexpr int SUPER_H = 8, SUPER_W = 4;      // super-tile shape (tiles)
constexpr int BLOCK_B = 8 * SLICE_B;         // one panel of a 32-row block: 32 KiB
// Recommended XP image per chunk: a config-3 shard (2^21 x 8192) in one chunk on
// a 288 GB MI355X; callers with less room pass a smaller workspace and get chunks.
constexpr size_t DEFAULT_CHUNK_BYTES = size_t(64) << 30;

struct SSched {
  const unsigned char* XP;  // bf16 image of this chunk
  float* S;
  float* part;   // one slab per remainder item
  float* accs;   // 1 flush slab per block
  const int* order;  // tile order: ti | tj << 16
  int64_t lds, dp;
  int64_t NK;  // K-tiles in the chunk
  int nseg;    // K segments per remainder tile (items = R * nseg)
  int d, nt, T, G, q, R;
  float alpha;
  int beta;
  int flush_kt;  // K-tiles between two-level flushes of the accumulators
  int prio;      // 1: waves 4-7 run at s_setprio 1 (the arbitration losers otherwise)
  unsigned* pace;  // per-XCD arrival counters (128 B apart), zeroed per launch
  int pace_kt;     // K-tiles between two XCD pacing points (0: off)
  int xm;          // remainder: segments per XCD, XCD-major numbering (0: global)
  int rpace;       // remainder rounds paced too (segment_h only)
  // fused split (variant 163): X is staged as fp32 and split in LDS
  const float* X;
  int64_t ldx, nrows;
  float* corr;  // lo^2 partials: [segment][octet wave][dp]
};

// XCD pacing point of the full-tile phases: the ~G/8 blocks on one XCD run
// neighbouring tiles of one super-tile and read the same K rows of its panels, but
// drift apart over ~10^5 K-tiles until their shared panels no longer meet in the
// XCD's 4 MB L2.  Every pace_kt K-tiles one lane per block adds 1 to its XCD's
// counter and waits (bounded: 20 us of s_memrealtime, so a block that is not
// resident can only cost time, never a hang) until all of the XCD's blocks have
// arrived.  Relaxed atomics, no fence: nothing is published, so no L2 write-back.
// The result's wait (vmcnt(0)) also drains this wave's ring DMAs, which keeps the
// counted vmcnt waits exact.
// Chip-wide pacing (r05): in the full-tile phases every kChipPaceEvery-th XCD pacing
// point also waits for all G blocks on one more counter (same bounded spin), which
// keeps the eight XCDs within ~128 K-tiles (~128 MB of the XP image) of each other,
// so a panel's K-tile fetched from HBM by one XCD is still in the Infinity Cache when
// the other XCDs that use the panel read it.  Interleaved A/B at config 3 (one
// process, bit-identical, profiles/r05zb_syrk_chip_pacing_ab.log): 296.6 -> 283.7 ms
// per op at every 2nd point; every point 286.0, every 3rd 286.5, every 4th 294.0;
// chip-wide only (no XCD level) 292.5; XCD pacing off 327.8.  Remainder rounds with
// global item numbering are chip-paced too, against the round's item count (config 2,
// all remainder: 24.77 -> 24.54 ms; config 3 286.0 -> 284.8).  Config 5 (short K per
// tile) is unchanged.
constexpr int kChipPaceEvery = 2;
// flush stagger per XCD = flush_kt / kFlushStaggerDiv K-tiles (0: none)
#ifdef DEIG_AB_SYRK_FLUSH_STAGGER
constexpr int kFlushStaggerDiv = DEIG_AB_SYRK_FLUSH_STAGGER;
#else
constexpr int kFlushStaggerDiv = 16;
#endif

__device__ __noinline__ void xcd_pace(unsigned* ctr, unsigned target) {
  __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (wall_clock64() - t0 > 2000) break;
    __builtin_amdgcn_s_sleep(1);
  }
}


__device__ __forceinline__ i32x4 make_rsrc(const void* base, uint32_t nrec) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  i32x4 r;
  r[0] = (int)(uint32_t)a;
  r[1] = (int)((uint32_t)(a >> 32) & 0xffffu);
  r[2] = (int)nrec;
  r[3] = 0x00020000;
  return r;
}

// 16 B per lane HBM -> LDS at m0 + 16 * lane (see syrk.hip for why inline asm).
__device__ __forceinline__ void dma16(i32x4 rsrc, int voff, const void* lds_dst) {
  const unsigned m0v = (unsigned)(uintptr_t)(lds_void*)lds_dst;
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :
               : "v"(voff), "s"(rsrc), "s"(m0v)
               : "memory", "m0");
}

// A K-tile is KT MFMA k-steps (16 rows each); the LDS ring holds NST K-tiles.
// Panel slice sl = (octet sl/2, hi|lo sl%2) is 4 KiB = four 1-KiB DMA wave-
// instructions; a panel has 4*KT slices.  One wave issues 4*KT DMAs per stage
// off the diagonal (the flattened [A slices | B slices] list split over the 8
// waves) and 2*KT on it (A only) - the counted vmcnt waits rely on these counts.
template <int KT>
struct Geo {
  static constexpr int NSLICE = 4 * KT;
  static constexpr int PANEL_B = NSLICE * SLICE_B;
  static constexpr int BUF_B = 2 * PANEL_B;
  static constexpr int DMA = 4 * KT, DMA_DIAG = 2 * KT;
};

template <int KT>
__device__ __forceinline__ void stage(const SSched& s, int64_t kt, int i0, int j0, bool diag,
                                      unsigned char* buf, int wave, int lane16) {
  using G_ = Geo<KT>;
  // XP: [32-row block][panel][slice 0..7][256 features][16 B]; this K-tile is
  // slices s0 .. s0 + 4*KT - 1 of block kt*KT/2.
  const int64_t blk = kt * KT / 2;
  const int s0 = (int)((kt * KT) & 1) * 4;
  const i32x4 rsrc = make_rsrc(s.XP + blk * (int64_t)s.nt * BLOCK_B, (uint32_t)(s.nt * BLOCK_B));
  int l16 = lane16;
  asm volatile("" : "+v"(l16));
  if (!diag) {
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      const int c = wave * KT + u;  // slice in [A slices | B slices]
      const int pb = c / G_::NSLICE, sl = c % G_::NSLICE;
      const int g = (pb ? j0 : i0) / BT * BLOCK_B + (s0 + sl) * SLICE_B;
      unsigned char* dst = buf + pb * G_::PANEL_B + sl * SLICE_B;
#pragma unroll
      for (int p = 0; p < 4; ++p) dma16(rsrc, l16 + g + p * 1024, dst + p * 1024);
    }
  } else {
#pragma unroll
    for (int u = 0; u < 2 * KT; ++u) {
      const int idx = wave * 2 * KT + u;  // (slice, 1-KiB part) of panel A
      const int sl = idx >> 2, p = idx & 3;
      dma16(rsrc, l16 + i0 / BT * BLOCK_B + (s0 + sl) * SLICE_B + p * 1024,
            buf + sl * SLICE_B + p * 1024);
    }
  }
}

// ------------------------------------------------ fused split (variant 163)
// X is staged as it lies in HBM (fp32 rows) and split in LDS, so no XP image is
// written and re-read (the split pass moved 2 x 4nd bytes).  A K-tile is 32 rows;
// wave w owns octet w & 3 of panel w >> 2 (diagonal tiles: panel A twice): it
// DMAs those 8 rows x 256 features (8 x 1 KiB) into the 8 KiB that the octet's
// (hi, lo) slices occupy, and later overwrites them in place with the slices.
// The region is the wave's own, so the split needs no barrier of its own.
constexpr int OCT_B = 2 * SLICE_B;

// One descriptor per stage: base = the octet's first row, records = its rows
// below nrows (later rows read as out of range, and an out-of-range LDS-DMA
// writes zeros); voff = 16 * lane, or an out-of-range offset (2^30 + row offset
// >= every record count, as ldx <= 2^25) for lanes whose features are >= d.
__device__ __forceinline__ void stage_x(const SSched& s, int64_t kt, int f0, unsigned char* buf,
                                        int wave, int voff) {
  const int64_t row0 = kt * 32 + 8 * (wave & 3);
  int64_t rv = s.nrows - row0;
  rv = rv < 0 ? 0 : rv > 8 ? 8 : rv;
  const uint32_t ldx4 = (uint32_t)s.ldx * 4u;
  const i32x4 rsrc = make_rsrc(s.X + row0 * s.ldx + f0, (uint32_t)rv * ldx4);
  unsigned char* dst = buf + (wave >> 2) * Geo<2>::PANEL_B + (wave & 3) * OCT_B;
#pragma unroll
  for (int r = 0; r < 8; ++r) dma16(rsrc, voff + (int)(r * ldx4), dst + r * 1024);
}

// Split the wave's staged region in place.  Lane c holds features 2c, 2c + 1 (half
// h = 0) and 128 + 2c, 129 + 2c (h = 1) of the 8 rows; all 16 reads land before
// the first write (the slices overlap every staged row).  Rows >= nrows and
// features >= d are zeroed here (independent of what a dropped DMA left in LDS).
// SQ: also accumulate the dropped lo * lo diagonal term (as r^2, r = x - hi: the
// difference is ~2^-25 x^2) into sq[2h + e].
template <bool SQ>
__device__ __forceinline__ void convert_x(unsigned char* buf, int wave, int lane, int rv, int fv,
                                          float* sq) {
  unsigned char* R = buf + (wave >> 2) * Geo<2>::PANEL_B + (wave & 3) * OCT_B;
  f32x2 v[2][8];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int r = 0; r < 8; ++r)
      v[h][r] = *reinterpret_cast<const f32x2*>(R + r * 1024 + h * 512 + 8 * lane);
  if (rv < 8 || fv < 256) {  // wave-uniform: the ragged last K-tile / a panel past d
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (r >= rv || 128 * h + 2 * lane >= fv) v[h][r] = f32x2{0.f, 0.f};
  }
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      u32x4 hv, lv;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float x0 = v[h][2 * p][e], x1 = v[h][2 * p + 1][e];
        const uint32_t hh = cvt2(x0, x1);
        const float r0 = x0 - lo_f(hh), r1 = x1 - hi_f(hh);
        hv[p] = hh;
        lv[p] = cvt2(r0, r1);
        if (SQ) sq[2 * h + e] = fmaf(r0, r0, fmaf(r1, r1, sq[2 * h + e]));
      }
      const int f = 128 * h + 2 * lane + e;
      *reinterpret_cast<u32x4*>(R + f * 16) = hv;
      *reinterpret_cast<u32x4*>(R + SLICE_B + f * 16) = lv;
    }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Wait until this wave's DMAs of a stage have landed while `ahead` later stages
// (0 .. NST-2) may stay in flight.
template <int KT, int NST>
__device__ __forceinline__ void wait_stage(int ahead, bool diag) {
  static_assert(NST >= 2 && NST <= 5, "ring depth");
  constexpr int D = Geo<KT>::DMA, DD = Geo<KT>::DMA_DIAG;
  if (ahead <= 0) {
    wait_vm<0>();
  } else if (ahead == 1 || NST == 3) {
    if (diag) wait_vm<DD>(); else wait_vm<D>();
  } else if (ahead == 2 || NST == 4) {
    if (diag) wait_vm<2 * DD>(); else wait_vm<2 * D>();
  } else {
    if (diag) wait_vm<3 * DD>(); else wait_vm<3 * D>();
  }
}

// ---------------------------------------------------------------- accumulators
// A wave's 128 x 64 output tile in MFMA result registers, for two MFMA shapes:
//   MF = 32: v_mfma_f32_32x32x16_bf16, 4 x 2 blocks of f32x16;
//   MF = 16: v_mfma_f32_16x16x32_bf16, 8 x 4 blocks of f32x4.
// Both are viewed as 32 "quads": 4 consecutive rows ib..ib+3 of one column j,
// which is how they are flushed, spilled to slabs and stored.
template <int MF>
struct Acc;

template <>
struct Acc<32> {
  f32x16 a[4][2];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int r = 0; r < 16; ++r) a[mb][nb][r] = 0.f;
  }
  // quad q = (mb, nb, g): rows 32 mb + 8 g + 4 (lane / 32), column 32 nb + lane % 32
  __device__ __forceinline__ float at(int q, int u) const { return a[q >> 3][(q >> 2) & 1][4 * (q & 3) + u]; }
  __device__ __forceinline__ void set(int q, int u, float v) { a[q >> 3][(q >> 2) & 1][4 * (q & 3) + u] = v; }
  static __device__ __forceinline__ int qrow(int q, int lane) {
    return 32 * (q >> 3) + 8 * (q & 3) + 4 * (lane >> 5);
  }
  static __device__ __forceinline__ int qcol(int q, int lane) { return 32 * ((q >> 2) & 1) + (lane & 31); }

  // One K-tile of KT 16-row k-steps; operand slice of 8 k-values: octet 2 st + lane / 32.
  template <int KT>
  __device__ __forceinline__ void mma(const unsigned char* A, const unsigned char* B, int wi,
                                      int wj, int lane) {
    const int c = lane & 31, h = lane >> 5;
#pragma unroll
    for (int st = 0; st < KT; ++st) {
      const int o = 2 * st + h;
      const unsigned char* ph = A + ((o * 2) * BT + 128 * wi + c) * 16;
      const unsigned char* qh = B + ((o * 2) * BT + 64 * wj + c) * 16;
      bf16x8 ahi[4], alo[4], bhi[2], blo[2];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        ahi[mb] = *reinterpret_cast<const bf16x8*>(ph + (32 * mb) * 16);
        alo[mb] = *reinterpret_cast<const bf16x8*>(ph + (BT + 32 * mb) * 16);
      }
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        bhi[nb] = *reinterpret_cast<const bf16x8*>(qh + (32 * nb) * 16);
        blo[nb] = *reinterpret_cast<const bf16x8*>(qh + (BT + 32 * nb) * 16);
      }
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          a[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi[mb], bhi[nb], a[mb][nb], 0, 0, 0);
          a[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi[mb], blo[nb], a[mb][nb], 0, 0, 0);
          a[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(alo[mb], bhi[nb], a[mb][nb], 0, 0, 0);
        }
    }
  }
};

template <>
struct Acc<16> {
  f32x4 a[8][4];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) a[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // quad q = (mb, nb): rows 16 mb + 4 (lane / 16), column 16 nb + lane % 16
  __device__ __forceinline__ float at(int q, int u) const { return a[q >> 2][q & 3][u]; }
  __device__ __forceinline__ void set(int q, int u, float v) { a[q >> 2][q & 3][u] = v; }
  static __device__ __forceinline__ int qrow(int q, int lane) { return 16 * (q >> 2) + 4 * (lane >> 4); }
  static __device__ __forceinline__ int qcol(int q, int lane) { return 16 * (q & 3) + (lane & 15); }

  // One K-tile of KT 16-row k-steps = KT/2 32-deep MFMA steps; operand slice of
  // 8 k-values: octet 4 st + lane / 16 (conflict-free ds_read_b128 lane groups).
  template <int KT>
  __device__ __forceinline__ void mma(const unsigned char* A, const unsigned char* B, int wi,
                                      int wj, int lane) {
    static_assert(KT % 2 == 0, "16x16x32 needs 32-row K-tiles");
    const int c = lane & 15, g = lane >> 4;
#pragma unroll
    for (int st = 0; st < KT / 2; ++st) {
      const int o = 4 * st + g;
      const unsigned char* ph = A + ((o * 2) * BT + 128 * wi + c) * 16;
      const unsigned char* qh = B + ((o * 2) * BT + 64 * wj + c) * 16;
      bf16x8 bhi[4], blo[4];
      // A block mb + 1 is read while block mb's 12 MFMAs run (two A register
      // sets), so only the first read of a k-step exposes LDS latency.
      bf16x8 ahi = *reinterpret_cast<const bf16x8*>(ph);
      bf16x8 alo = *reinterpret_cast<const bf16x8*>(ph + BT * 16);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        bhi[nb] = *reinterpret_cast<const bf16x8*>(qh + (16 * nb) * 16);
        blo[nb] = *reinterpret_cast<const bf16x8*>(qh + (BT + 16 * nb) * 16);
      }
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) {
        bf16x8 nhi = ahi, nlo = alo;
        if (mb + 1 < 8) {
          nhi = *reinterpret_cast<const bf16x8*>(ph + (16 * (mb + 1)) * 16);
          nlo = *reinterpret_cast<const bf16x8*>(ph + (BT + 16 * (mb + 1)) * 16);
        }
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          a[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bhi[nb], a[mb][nb], 0, 0, 0);
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          a[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, blo[nb], a[mb][nb], 0, 0, 0);
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          a[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bhi[nb], a[mb][nb], 0, 0, 0);
        ahi = nhi;
        alo = nlo;
      }
      // Issue order for the scheduler: A0 + B reads, then per block the next
      // block's two A reads ahead of the current block's 12 MFMAs.
      __builtin_amdgcn_sched_group_barrier(0x100, 10, 0);
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) {
        if (mb + 1 < 8) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);
      }
    }
  }

};

constexpr int NQUAD = 32;

// Slab image: quad-major, 16 B per lane (the reduce kernel reads it back).
__device__ __forceinline__ f32x4* slab_at(float* slab, int wave, int q, int lane) {
  return reinterpret_cast<f32x4*>(slab + ((wave * NQUAD + q) * 64 + lane) * 4);
}

// The slab addresses are formed here from an opaque base: otherwise the compiler
// hoists all 32 of them out of the K loop and keeps 64 VGPRs live for them.
#ifdef DEIG_AB_SYRK_SERIAL_FLUSH
template <int MF>
__device__ __forceinline__ void flush(float* slab, bool first, Acc<MF>& acc, int wave, int lane) {
  asm volatile("" : "+v"(slab));
#pragma unroll
  for (int q = 0; q < NQUAD; ++q) {
    f32x4* ptr = slab_at(slab, wave, q, lane);
    f32x4 v = {acc.at(q, 0), acc.at(q, 1), acc.at(q, 2), acc.at(q, 3)};
    if (!first) v += *ptr;
    *ptr = v;
#pragma unroll
    for (int u = 0; u < 4; ++u) acc.set(q, u, 0.f);
  }
}
#else
// r06: buffer loads / stores in batches of kFlushBatch quads.  Through a generic
// pointer the slab accesses were flat_* operations, which the hardware may complete
// out of order, so each quad's read was its own vmcnt(0) round trip: 32 serial round
// trips per flush (~34 us per event at config 3).  Buffer operations complete in issue
// order, so a batch's reads are in flight together (its write-backs stay queued
// behind them).
#ifdef DEIG_AB_SYRK_FLUSH_BATCH
constexpr int kFlushBatch = DEIG_AB_SYRK_FLUSH_BATCH;
#else
constexpr int kFlushBatch = 4;
#endif
template <int MF>
__device__ __forceinline__ void flush(float* slab, bool first, Acc<MF>& acc, int wave, int lane) {
  asm volatile("" : "+v"(slab));
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(slab, (short)0, (int)(SLAB * sizeof(float)), 0x00020000);
  const int voff = (wave * NQUAD * 64 + lane) * 16;
  auto put = [&](int q, f32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, voff + q * 1024, 0, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc.set(q, u, 0.f);
  };
  if (first) {
#pragma unroll
    for (int q = 0; q < NQUAD; ++q) put(q, f32x4{acc.at(q, 0), acc.at(q, 1), acc.at(q, 2), acc.at(q, 3)});
    return;
  }
#pragma unroll
  for (int b = 0; b < NQUAD; b += kFlushBatch) {
    f32x4 v[kFlushBatch];
#pragma unroll
    for (int i = 0; i < kFlushBatch; ++i)
      v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff + (b + i) * 1024, 0, 0));
    __builtin_amdgcn_sched_barrier(0);  // the batch's reads issue together
#pragma unroll
    for (int i = 0; i < kFlushBatch; ++i) {
      const int q = b + i;
      put(q, v[i] + f32x4{acc.at(q, 0), acc.at(q, 1), acc.at(q, 2), acc.at(q, 3)});
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}
#endif

template <int MF>
__device__ __forceinline__ void unflush(float* slab, Acc<MF>& acc, int wave, int lane) {
  asm volatile("" : "+v"(slab));
#ifdef DEIG_AB_SYRK_SERIAL_FLUSH
#pragma unroll
  for (int q = 0; q < NQUAD; ++q) {
    const f32x4 v = *slab_at(slab, wave, q, lane);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc.set(q, u, acc.at(q, u) + v[u]);
  }
#else
  // buffer loads in batches (flat loads were one vmcnt(0) round trip each, see flush)
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(slab, (short)0, (int)(SLAB * sizeof(float)), 0x00020000);
  const int voff = (wave * NQUAD * 64 + lane) * 16;
#pragma unroll
  for (int b = 0; b < NQUAD; b += kFlushBatch) {
    f32x4 v[kFlushBatch];
#pragma unroll
    for (int i = 0; i < kFlushBatch; ++i)
      v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff + (b + i) * 1024, 0, 0));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < kFlushBatch; ++i)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc.set(b + i, u, acc.at(b + i, u) + v[i][u]);
  }
#endif
}

// Store 4 consecutive rows ib..ib+3 of column j (values = alpha * a[u] (+ S)),
// into S[i][j] and the mirror S[j][i].  Diagonal tiles keep only i >= j, so both
// triangles come from the same register (bit-exact symmetry).
__device__ __forceinline__ void store4(const SSched& s, int ib, int j, bool diag, const float* a) {
  if (ib >= s.d || j >= s.d) return;
  float v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    float* p = s.S + (int64_t)(ib + u) * s.lds + j;
    v[u] = s.alpha * a[u];
    if (s.beta && (!diag || ib + u >= j)) v[u] += *p;
  }
  if (!diag) {
#pragma unroll
    for (int u = 0; u < 4; ++u) s.S[(int64_t)(ib + u) * s.lds + j] = v[u];
    const f32x4 w = {v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(s.S + (int64_t)j * s.lds + ib) = w;
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (ib + u >= j) {
        s.S[(int64_t)(ib + u) * s.lds + j] = v[u];
        s.S[(int64_t)j * s.lds + ib + u] = v[u];
      }
  }
}

template <int MF, int KT, int NST, bool FX, bool SQ>
__device__ __forceinline__ void segment(const SSched& s, unsigned char* lds, int tile, int64_t k0, int64_t k1,
                        int slot, bool partial, int pace_j, int cseg) {
  static_assert(!FX || (KT == 2 && NST == 2), "fused split: 32-row K-tiles, two stages");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wi = wave >> 2, wj = wave & 3;
  const int lane16 = lane * 16;
  const int tt = __builtin_amdgcn_readfirstlane(s.order[tile]);
  const int ti = tt & 0xffff, tj = tt >> 16;
  const int i0 = ti * BT, j0 = tj * BT;
  const bool diag = (ti == tj);
  // fused split: this wave's panel origin, valid features in it, DMA lane offset
  const int fx0 = (wave >= 4 && !diag) ? j0 : i0;
  const int fv = s.d - fx0;
  const int xvoff = 4 * lane < fv ? lane16 : (1 << 30);
  // lo^2 of the diagonal: panel A's octets (waves 0-3) of diagonal tiles
  const bool sqw = SQ;
  float sq[4] = {0.f, 0.f, 0.f, 0.f};

  if (s.prio && wave >= 4) __builtin_amdgcn_s_setprio(1);
  Acc<MF> acc;
  acc.zero();
  float* slab = partial ? s.part + (int64_t)slot * SLAB : s.accs + (int64_t)blockIdx.x * SLAB;
  bool flushed = false;
  const int64_t nkt = k1 - k0;
  if (nkt > 0) {
    // Nothing else may be in flight on the VM counter while the ring runs (the
    // counted waits assume only DMAs): drain the previous segment's stores.
    wait_vm<0>();
    __syncthreads();  // the previous segment's last stage may still be read
    // Ring of NST stages; NST - 1 K-tiles are issued ahead of the one being
    // computed.  Stage t lives in buffer t % NST.
    constexpr int BUF_B = Geo<KT>::BUF_B;
    if constexpr (FX) {
      // fused: K-tile k0 staged and split (masked: it may be ragged) before the
      // loop; iteration t stages K-tile t + 1 after the barrier and splits it
      // inside K-tile t's MFMAs (its own region: a vmcnt wait, no barrier).
      stage_x(s, k0, fx0, lds, wave, xvoff);
      wait_vm<0>();
      const int64_t rv0 = s.nrows - (k0 * 32 + 8 * (wave & 3));
      convert_x<SQ>(lds, wave, lane, rv0 < 0 ? 0 : rv0 > 8 ? 8 : (int)rv0, fv, sq);
    } else {
      for (int t = 0; t < NST - 1 && t < nkt; ++t)
        stage<KT>(s, k0 + t, i0, j0, diag, lds + t * BUF_B, wave, lane16);
    }
    int cur = 0, nxt = NST - 1, since = 0, since_pace = 0;
    // pacing target: blocks on this XCD x arrival index
    const int xcd = blockIdx.x & 7;
    const unsigned nx = (unsigned)((s.G >> 3) + (xcd < (s.G & 7) ? 1 : 0));
    for (int64_t t = 0; t < nkt; ++t) {
      const int64_t left = nkt - 1 - t;
      if (pace_j >= 0 && ++since_pace == s.pace_kt) {
        since_pace = 0;
        ++pace_j;
        if (threadIdx.x == 0) xcd_pace(s.pace + 32 * xcd, (unsigned)pace_j * nx);
      }
      // RAW: this wave's DMAs of stage t landed (counted vmcnt), then a barrier
      // every reader passes.  WAR: stage t-1's ds_reads retired (lgkmcnt) before
      // the barrier, so its buffer can be restaged right after it.  A raw
      // s_barrier: __syncthreads() would drain the ring with vmcnt(0).
      // fused: every wave split its own region of stage t last iteration (its
      // ds_writes retire at the lgkmcnt wait), so the barrier publishes stage t.
      if (!FX) wait_stage<KT, NST>(left < NST - 2 ? (int)left : NST - 2, diag);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if constexpr (FX) {
        if (t + 1 < nkt) stage_x(s, k0 + t + 1, fx0, lds + nxt * BUF_B, wave, xvoff);
        // K-tile t's MFMAs, then this wave's split of K-tile t + 1 (its DMAs were
        // issued right after the barrier: the MFMAs cover their latency).  The
        // in-place split of the wave's own region needs no barrier of its own.
        unsigned char* bc = lds + cur * BUF_B;
        acc.template mma<KT>(bc, bc + Geo<KT>::PANEL_B, wi, wj, lane);
        if (t + 1 < nkt) {
          wait_vm<0>();
          const int64_t rv1 = s.nrows - ((k0 + t + 1) * 32 + 8 * (wave & 3));
          convert_x<SQ>(lds + nxt * BUF_B, wave, lane, rv1 < 0 ? 0 : rv1 > 8 ? 8 : (int)rv1, fv, sq);
        }
      } else {
        if (t + NST - 1 < nkt)
          stage<KT>(s, k0 + t + NST - 1, i0, j0, diag, lds + nxt * BUF_B, wave, lane16);
        unsigned char* bc = lds + cur * BUF_B;
        acc.template mma<KT>(bc, diag ? bc : bc + Geo<KT>::PANEL_B, wi, wj, lane);
      }
      if (++since == s.flush_kt && t + 1 < nkt) {
        flush<MF>(slab, !flushed, acc, wave, lane);
        wait_vm<0>();  // keep the slab traffic off the ring's counted waits
        flushed = true;
        since = 0;
      }
      cur = cur + 1 == NST ? 0 : cur + 1;
      nxt = nxt + 1 == NST ? 0 : nxt + 1;
    }
  }
  if (flushed) unflush<MF>(slab, acc, wave, lane);
  if (sqw) {  // [segment][octet wave][dp]; summed by diag_corr_kernel
    float* c = s.corr + (int64_t)(cseg * 4 + wave) * s.dp + i0;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      *reinterpret_cast<f32x2*>(c + 128 * h + 2 * lane) = f32x2{sq[2 * h], sq[2 * h + 1]};
  }

  if (partial) {
#pragma unroll
    for (int q = 0; q < NQUAD; ++q)
      *slab_at(slab, wave, q, lane) = f32x4{acc.at(q, 0), acc.at(q, 1), acc.at(q, 2), acc.at(q, 3)};
    return;
  }
#pragma unroll
  for (int q = 0; q < NQUAD; ++q) {
    const float a[4] = {acc.at(q, 0), acc.at(q, 1), acc.at(q, 2), acc.at(q, 3)};
    store4(s, i0 + 128 * wi + Acc<MF>::qrow(q, lane), j0 + 64 * wj + Acc<MF>::qcol(q, lane), diag, a);
  }
}

#ifdef DEIG_AB_SYRK_VARIANT
// the r03 K loops (staggered phases, quarter-refill ring): A/B builds only
#include "ab/syrk_split_superseded.inc"
#endif

// Pacing points of one segment: point j (1..n) waits for the XCD counter to reach
// base + j * mult (n = 0: none).
struct PaceSeq {
  int n;
  unsigned base, mult;
  unsigned gbase = 0;  // the chip-wide counter's target before this segment
  unsigned gmult = 0;  // blocks that pace chip-wide with this one (G, or a round's items)
  bool g = false;      // every kChipPaceEvery-th point is also chip-wide
};

// Blocks of this block's XCD (logical L) that run a remainder item in round u.
// Global numbering: item i = L + u G (the XCD's blocks are logical [L - b/8, + nx));
// XCD-major (s.xm > 0, G % 8 == 0): XCD x owns segments [x xm, (x + 1) xm) and its
// G / 8 blocks take their items j = l + u G / 8 (j = local segment * R + r).
__device__ __forceinline__ int rem_active(const SSched& s, int L, int u) {
  if (s.xm) {
    const int gx = s.G >> 3, left = s.R * s.xm - u * gx;
    return left < 0 ? 0 : (left < gx ? left : gx);
  }
  const int xcd = blockIdx.x & 7;
  const int nx = (s.G >> 3) + (xcd < (s.G & 7) ? 1 : 0);
  const int left = s.R * s.nseg - u * s.G - (L - (int)(blockIdx.x >> 3));
  return left < 0 ? 0 : (left < nx ? left : nx);
}

__device__ __forceinline__ int rem_rounds(const SSched& s, int L) {
  if (s.xm) {
    const int gx = s.G >> 3, l = L % gx, items = s.R * s.xm;
    return l < items ? (items - 1 - l) / gx + 1 : 0;
  }
  const int items = s.R * s.nseg;
  return L < items ? (items - 1 - L) / s.G + 1 : 0;
}

// Round u's item of block L: tile index, slot (= segment * R + r) and segment.
__device__ __forceinline__ void rem_item(const SSched& s, int L, int u, int& tile, int& slot, int& sg) {
  int r;
  if (s.xm) {
    const int gx = s.G >> 3, x = L / gx, j = L - x * gx + u * gx;
    const int sl = j / s.R;
    r = j - sl * s.R;
    sg = x * s.xm + sl;
  } else {
    const int i = L + u * s.G;
    sg = i / s.R;
    r = i - sg * s.R;
  }
  tile = s.q * s.G + r;
  slot = sg * s.R + r;
}

// ------------------------------------------------ half-refill ring (variant 30000)
// The staggered kernel's two phases per K-tile (variant 12100: 48-MFMA M parts, half
// the barriers of four phases) on segment_q's ring: phase h reads A quarters 2h and
// 2h + 1 (and B in phase 0), and each region is restaged with K-tile t + 2 as soon as
// both wave groups have read it.  Per wave and K-tile 8 pieces in two L parts of 4:
//   L_0(t): B(t+1) parts 2, 3 and A quarters 2, 3 of t+1 into nxt (their previous
//           contents, K-tile t-1's B and second half, were read by both groups by
//           the barrier that opened this part);
//   L_1(t): B(t+2) parts 0, 1 and A quarters 0, 1 of t+2 into cur (read in L_0(t)).
// So every piece has ~1.5 K-tiles of lead instead of one.  RAW: a wave waits for its
// own pieces of a region at the end of the L part before the one that reads it:
// end of L_0(t) for A quarters 2, 3 of t (younger: L_1(t-1)'s 4 + L_0(t)'s 4 = 8);
// end of L_1(t) for K-tile t+1's B and quarters 0, 1 (younger than its last piece,
// B part 3 issued in L_0(t): quarters 2, 3 of t+1 + L_1(t)'s 4 = 6).  Near the end of
// the segment the counts shrink with the pieces not issued.  WAR: every L part
// retires its reads (lgkmcnt(0)) before its closing barrier.  Same MFMA order per
// accumulator as the other variants (bit-identical sums).
// DW != -1: a DIAGONAL tile.  Its B panel is its A panel, so no B pieces are staged
// and the B operands are read from the A quarters (the same bytes in the A layout);
// with 2 DMA pieces per L part instead of 4 the counted waits become 4 / 2, and the end
// of L_1 also waits for quarters 2, 3 of the next K-tile (phase 0 reads them as B).
// The same B-operand read point and restage points as before, so the WAR argument
// above holds unchanged.
// DW >= 0: a wave of a diagonal tile whose 128 x 64 block starts DW = 64 wj - 128 wi
// columns right of the diagonal (0, 64, or 128 for waves 2 and 3 alike, whose blocks lie
// wholly above it; waves 4 and 5 of the tile run DW = -2).
// store4 keeps only i >= j there, so the 16 x 16 MFMA blocks that lie wholly above the
// diagonal (dw_skip) are neither computed nor their operands read: all of waves 2 and
// 3 (DW = 128: they only stage their DMA pieces and pass the barriers), 22 of 32 blocks
// of waves 1 and 7, 6 of waves 0 and 6 - 120 of the tile's 256, MFMAs a power-held
// chip does not spend.  Every stored sum is the same MFMA chain as before
// (bit-identical); separate instantiations, so the other tiles' code is unchanged (a
// runtime test inside the loop measured slower, r06).
constexpr int kDwOff = -1, kDwDiag = -2;
constexpr bool dw_skip(int dw, int mb, int nb) { return dw >= 0 && 16 * mb + 15 < dw + 16 * nb; }
constexpr bool dw_row(int dw, int mb) { return !dw_skip(dw, mb, 0); }  // A block row mb is read
constexpr bool dw_col(int dw, int nb) { return !dw_skip(dw, 7, nb); }  // B block column nb is read
constexpr bool dw_idle(int dw) { return !dw_row(dw, 7); }

template <int PRIO, int DW>
__device__ __forceinline__ void segment_h(const SSched& s, unsigned char* lds, int tile, int64_t k0,
                                          int64_t k1, int slot, bool partial, const PaceSeq& pc) {
  constexpr bool idle = dw_idle(DW);
#ifndef DEIG_AB_SYRK_DIAG_B_DMA
  constexpr bool dgb = DW != kDwOff;  // B operands from the A quarters
#else
  constexpr bool dgb = false;
#endif
  constexpr int BUF_B = Geo<2>::BUF_B;
  constexpr int QB = 8 * 1024;  // one A quarter
  constexpr int BOFF = 4 * QB;  // the B panel
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wi = wave >> 2, wj = wave & 3;
  const bool lag = wave >= 4;
  const int tt = __builtin_amdgcn_readfirstlane(s.order[tile]);
  const int ti = tt & 0xffff, tj = tt >> 16;
  const int i0 = ti * BT, j0 = tj * BT;
  const bool diag = (ti == tj);
  Acc<16> acc;
  acc.zero();
  float* slab = partial ? s.part + (int64_t)slot * SLAB : s.accs + (int64_t)blockIdx.x * SLAB;
  bool flushed = false;
  const int64_t nkt = k1 - k0;
  auto bar = [&]() {  // raw barrier; nothing moves across it
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };
  const int a_off = ti * BLOCK_B + wave * SLICE_B + ((lane >> 5) * 128 + (lane & 31)) * 16;
  const int b_off = tj * BLOCK_B + wave * SLICE_B + lane * 16;
  const uint32_t nrec = (uint32_t)(s.nt * BLOCK_B);
  auto ring_rsrc = [&](int64_t kt) {
    return make_rsrc(s.XP + kt * (int64_t)s.nt * BLOCK_B, nrec);
  };
  auto issue_a = [&](int64_t kt, int q, unsigned char* buf) {
    const i32x4 r = ring_rsrc(kt);
    int o = a_off + q * 512;
    asm volatile("" : "+v"(o));
    dma16(r, o, buf + q * QB + wave * 1024);
  };
  auto issue_b = [&](int64_t kt, unsigned char* buf, int p0, int p1) {
    const i32x4 r = ring_rsrc(kt);
    int o = b_off;
    asm volatile("" : "+v"(o));
#pragma unroll
    for (int p = 0; p < 4; ++p)
      if (p >= p0 && p < p1) dma16(r, o + p * 1024, buf + BOFF + wave * SLICE_B + p * 1024);
  };
  if (nkt > 0) {
    wait_vm<0>();     // the previous segment's stores / flushes
    __syncthreads();  // ... and its last reads of the ring
    // K-tile k0 whole, then K-tile k0 + 1's B parts 0, 1 and quarters 0, 1 (as an
    // L_1 of K-tile k0 - 1 would have issued them)
    if constexpr (!dgb) issue_b(k0, lds, 0, 4);
#pragma unroll
    for (int q = 0; q < 4; ++q) issue_a(k0, q, lds);
    if (nkt > 1) {
      if constexpr (!dgb) issue_b(k0 + 1, lds + BUF_B, 0, 2);
      issue_a(k0 + 1, 0, lds + BUF_B);
      issue_a(k0 + 1, 1, lds + BUF_B);
      wait_vm<dgb ? 2 : 4>();  // K-tile k0 landed
    } else {
      wait_vm<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    if (lag) bar();  // the stagger
    const int c = lane & 15, g4 = lane >> 4;
    const int xcd = blockIdx.x & 7;
    // Flush stagger (r06): XCD x flushes x * flush_kt / 16 K-tiles earlier than XCD 0,
    // so the eight XCDs' slab bursts fall at different K-tiles instead of all at once
    // (each partial sum still spans flush_kt K-tiles, the first one of a segment fewer).
    int since = kFlushStaggerDiv > 0 ? xcd * (s.flush_kt / kFlushStaggerDiv) : 0;
    int since_pace = 0, pace_left = pc.n;
    unsigned pace_t = pc.base;
    int gcount = 0;
    unsigned gtarget = pc.gbase;
    bf16x8 bhi[4], blo[4];
    bf16x8 ahi[4], alo[4];
    for (int64_t t = 0; t < nkt; ++t) {
      unsigned char* cur = lds + (t & 1) * BUF_B;
      unsigned char* nxt = lds + ((t + 1) & 1) * BUF_B;
      const bool has1 = t + 1 < nkt, has2 = t + 2 < nkt;
      const unsigned char* pa = cur + ((g4 * 2) * 64 + 32 * wi + c) * 16;
      const unsigned char* pb = cur + BOFF + ((g4 * 2) * BT + 64 * wj + c) * 16;
      // B feature f = 64 wj + 16 nb + c of slice 2 g4 (+1: lo) in the A layout:
      // quarter (f % 128) / 32, lane 32 (f / 128) + f % 32
      const unsigned char* pbd = cur + (2 * (wj & 1)) * QB + (2 * g4) * 1024 + (32 * (wj >> 1) + c) * 16;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // ---------------- L part
        if (h == 0) {
          if (pace_left > 0 && ++since_pace == s.pace_kt) {
            since_pace = 0;
            --pace_left;
            pace_t += pc.mult;
            if (threadIdx.x == 0) xcd_pace(s.pace + 32 * xcd, pace_t);
            if (pc.g && ++gcount == kChipPaceEvery) {  // ... and every other one chip-wide
              gcount = 0;
              gtarget += pc.gmult;
              if (threadIdx.x == 0) xcd_pace(s.pace + 32 * 8, gtarget);
            }
          }
          if (since == s.flush_kt) {
            if constexpr (!idle) flush<16>(slab, !flushed, acc, wave, lane);
            wait_vm<0>();
            flushed = true;
            since = 0;
          }
          ++since;
          if (has1) {
            if constexpr (!dgb) issue_b(k0 + t + 1, nxt, 2, 4);
            issue_a(k0 + t + 1, 2, nxt);
            issue_a(k0 + t + 1, 3, nxt);
          }
#pragma unroll
          for (int nb = 0; nb < 4; ++nb) {
            if (dw_col(DW, nb)) {
              if constexpr (dgb) {
                const unsigned char* pq = pbd + (nb >> 1) * QB + (16 * (nb & 1)) * 16;
                bhi[nb] = *reinterpret_cast<const bf16x8*>(pq);
                blo[nb] = *reinterpret_cast<const bf16x8*>(pq + 1024);
              } else {
                bhi[nb] = *reinterpret_cast<const bf16x8*>(pb + (16 * nb) * 16);
                blo[nb] = *reinterpret_cast<const bf16x8*>(pb + (BT + 16 * nb) * 16);
              }
            }
          }
        } else if (has2) {
          if constexpr (!dgb) issue_b(k0 + t + 2, cur, 0, 2);
          issue_a(k0 + t + 2, 0, cur);
          issue_a(k0 + t + 2, 1, cur);
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int q = 2 * h + (m >> 1), mm = m & 1;
          if (dw_row(DW, 4 * h + m)) {
            ahi[m] = *reinterpret_cast<const bf16x8*>(pa + q * QB + (16 * mm) * 16);
            alo[m] = *reinterpret_cast<const bf16x8*>(pa + q * QB + (64 + 16 * mm) * 16);
          }
        }
        if constexpr (dgb) {  // 2 pieces per L part; phase 0 reads all four quarters
          if (h == 0) {
            if (has1) wait_vm<4>(); else wait_vm<0>();
          } else {
            if (has2) wait_vm<2>(); else wait_vm<0>();
          }
        } else if (h == 0) {
          if (has1) wait_vm<8>(); else wait_vm<0>();
        } else {
          if (has2) wait_vm<6>(); else if (has1) wait_vm<2>(); else wait_vm<0>();
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bar();
        // ---------------- M part
        if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int mb = 4 * h + m;
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
            if (!dw_skip(DW, mb, nb))
              acc.a[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi[m], bhi[nb], acc.a[mb][nb], 0, 0, 0);
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
            if (!dw_skip(DW, mb, nb))
              acc.a[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi[m], blo[nb], acc.a[mb][nb], 0, 0, 0);
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
            if (!dw_skip(DW, mb, nb))
              acc.a[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo[m], bhi[nb], acc.a[mb][nb], 0, 0, 0);
        }
        if (PRIO) __builtin_amdgcn_s_setprio(0);
        bar();
      }
    }
    if (!lag) bar();  // balance the stagger
  }
  if (flushed && !idle) unflush<16>(slab, acc, wave, lane);
  if (partial) {
#pragma unroll
    for (int q = 0; q < NQUAD; ++q)
      *slab_at(slab, wave, q, lane) = f32x4{acc.at(q, 0), acc.at(q, 1), acc.at(q, 2), acc.at(q, 3)};
    return;
  }
  if constexpr (idle) return;
#pragma unroll
  for (int q = 0; q < NQUAD; ++q) {
    const float a[4] = {acc.at(q, 0), acc.at(q, 1), acc.at(q, 2), acc.at(q, 3)};
    store4(s, i0 + 128 * wi + Acc<16>::qrow(q, lane), j0 + 64 * wj + Acc<16>::qcol(q, lane), diag, a);
  }
}

template <int PRIO>
__global__ __launch_bounds__(NTHR) void syrks_h_kernel(SSched s) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * Geo<2>::BUF_B];
  const int L = xcd_logical(blockIdx.x, s.G);
  const int nwork = s.q + rem_rounds(s, L);
  const int xcd = blockIdx.x & 7;
  const unsigned nx = (unsigned)((s.G >> 3) + (xcd < (s.G & 7) ? 1 : 0));
  // Full phases: every block runs P = NK / pace_kt points per tile.  Remainder rounds
  // (rpace): Pm points per item, Pm from the shortest segment, so every item of a
  // round runs the same count and the targets stay exact across rounds.
  const unsigned P = s.pace_kt > 0 ? (unsigned)(s.NK / s.pace_kt) : 0u;
  const int Pm = (s.pace_kt > 0 && s.rpace && s.nseg > 0) ? (int)(s.NK / s.nseg / s.pace_kt) : 0;
  unsigned rbase = (unsigned)s.q * P * nx;
  for (int w = 0; w < nwork; ++w) {
    int tile, slot = 0, sg = 0;
    int64_t k0 = 0, k1 = s.NK;
    const bool partial = w >= s.q;
    PaceSeq pc{0, 0u, 0u};
    if (!partial) {
      tile = w * s.G + L;
      pc = PaceSeq{(int)P, (unsigned)w * P * nx, nx};
      pc.g = true;
      pc.gbase = (unsigned)w * (P / kChipPaceEvery) * (unsigned)s.G;
      pc.gmult = (unsigned)s.G;
    } else {
      rem_item(s, L, w - s.q, tile, slot, sg);
      k0 = __builtin_amdgcn_readfirstlane((int)(s.NK * sg / s.nseg));
      k1 = __builtin_amdgcn_readfirstlane((int)(s.NK * (sg + 1) / s.nseg));
      if (Pm > 0) {
        unsigned before = 0;
        for (int u = 0; u < w - s.q; ++u) before += (unsigned)rem_active(s, L, u);
        pc = PaceSeq{Pm, rbase + before * (unsigned)Pm, (unsigned)rem_active(s, L, w - s.q)};
#ifndef DEIG_AB_SYRK_NO_REM_CHIP
        if (!s.xm) {  // global item numbering: round u runs min(G, items - u G) items
          const int items = s.R * s.nseg;
          unsigned gb = (unsigned)s.q * (P / kChipPaceEvery) * (unsigned)s.G;
          for (int u = 0; u < w - s.q; ++u)
            gb += (unsigned)min(s.G, items - u * s.G) * (unsigned)(Pm / kChipPaceEvery);
          pc.g = true;
          pc.gbase = gb;
          pc.gmult = (unsigned)min(s.G, items - (w - s.q) * s.G);
        }
#endif
      }
    }
    const int tt = __builtin_amdgcn_readfirstlane(s.order[tile]);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool dg = (tt & 0xffff) == (tt >> 16);
#ifndef DEIG_AB_SYRK_NO_DIAG_IDLE
    const int dw = 64 * (wv & 3) - 128 * (wv >> 2);
    if (dg && dw == 0)
      segment_h<PRIO, 0>(s, lds, tile, k0, k1, slot, partial, pc);
    else if (dg && dw == 64)
      segment_h<PRIO, 64>(s, lds, tile, k0, k1, slot, partial, pc);
    else if (dg && dw >= 128)  // waves 2 and 3: the whole block above the diagonal
      segment_h<PRIO, 128>(s, lds, tile, k0, k1, slot, partial, pc);
    else if (dg)
      segment_h<PRIO, kDwDiag>(s, lds, tile, k0, k1, slot, partial, pc);
    else
#endif
      segment_h<PRIO, kDwOff>(s, lds, tile, k0, k1, slot, partial, pc);
  }
}

template <int MF, int KT, int NST, bool FX>
__global__ __launch_bounds__(NTHR) void syrks_kernel(SSched s) {
  static_assert(NST * Geo<KT>::BUF_B <= 160 * 1024, "LDS ring exceeds 160 KiB");
  __shared__ __attribute__((aligned(16))) unsigned char lds[NST * Geo<KT>::BUF_B];
  const int b = blockIdx.x;
  const int L = xcd_logical(b, s.G);
  // Full phases (w < q): every block walks all K of one tile, in lock-step with
  // the rest.  Remainder: R tiles x nseg equal K segments, item i = seg * R + r,
  // taken by logical block i mod G in round i / G.  Segment-major numbering
  // keeps the items that run together (and, by the XCD-aware relabel, the ~G/8
  // on one XCD) on the same K rows of neighbouring tiles, so their panels are
  // shared in L2 rather than each item streaming its own K range from HBM.
  // One call site of segment(): its unrolled body is inlined once.
  const int items = s.R * s.nseg;
  const int nwork = s.q + (L < items ? (items - 1 - L) / s.G + 1 : 0);
  for (int w = 0; w < nwork; ++w) {
    int tile, slot = 0, cseg = 0;
    int64_t k0 = 0, k1 = s.NK;
    const bool partial = w >= s.q;
    if (!partial) {
      tile = w * s.G + L;
    } else {
      const int i = L + (w - s.q) * s.G;
      const int sg = i / s.R, r = i - sg * s.R;
      tile = s.q * s.G + r;
      slot = i;
      cseg = sg;
      // (64-bit divisions run on the VALU: pin the bounds to SGPRs, the DMA
      // descriptors built from them must be wave-uniform)
      k0 = __builtin_amdgcn_readfirstlane((int)(s.NK * sg / s.nseg));
      k1 = __builtin_amdgcn_readfirstlane((int)(s.NK * (sg + 1) / s.nseg));
    }
    // full phases pace (identical K work on every block); remainder items do not
    const int pace_j = (!partial && s.pace_kt > 0) ? (int)(w * (s.NK / s.pace_kt)) : -1;
    // fused: the lo^2 accumulation is compiled only into the copy that the
    // diagonal tiles' A-panel waves run
    if constexpr (FX) {
      const int tt = __builtin_amdgcn_readfirstlane(s.order[tile]);
      if ((tt & 0xffff) == (tt >> 16) && (threadIdx.x >> 6) < 4)
        segment<MF, KT, NST, true, true>(s, lds, tile, k0, k1, slot, partial, pace_j, cseg);
      else
        segment<MF, KT, NST, true, false>(s, lds, tile, k0, k1, slot, partial, pace_j, cseg);
    } else {
      segment<MF, KT, NST, false, false>(s, lds, tile, k0, k1, slot, partial, pace_j, cseg);
    }
  }
}

// grid (R, SLAB/4/256): one thread per float4 of a remainder tile's slab image.
template <int MF>
__global__ __launch_bounds__(256) void syrks_reduce_kernel(SSched s) {
  const int r = blockIdx.x;
  const int f = blockIdx.y * 256 + threadIdx.x;
  const int lane = f & 63, q = (f >> 6) & (NQUAD - 1), wave = f >> 11;
  const int wi = wave >> 2, wj = wave & 3;
  const int tt = s.order[s.q * s.G + r];
  const int ti = tt & 0xffff, tj = tt >> 16;
  const bool diag = (ti == tj);
  f32x4 sum = {0.f, 0.f, 0.f, 0.f};
  for (int sg = 0; sg < s.nseg; ++sg)  // fixed order: deterministic
    sum += *reinterpret_cast<const f32x4*>(s.part + (int64_t)(sg * s.R + r) * SLAB + (int64_t)f * 4);
  const float a[4] = {sum[0], sum[1], sum[2], sum[3]};
  store4(s, ti * BT + 128 * wi + Acc<MF>::qrow(q, lane), tj * BT + 64 * wj + Acc<MF>::qcol(q, lane),
         diag, a);
}

__device__ __forceinline__ uint32_t bf16_rne(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// (r04, measured and not kept: one 16-B load per lane and row, lane -> features
// 4 lane + j, so each hi / lo store covers 16 B at a 64-B stride: config 2 op 27.54 vs
// 25.74 ms, config-3 shard 315.3 vs 307.7, profiles/r04zb_syrk_*_ab.log - most likely
// the stores: below, each wave store instruction writes 1 KiB contiguous.)
// X rows [0, n) of the chunk -> XP (noct octets; rows >= n and features >= d
// are zeros) + per-block partial sums of lo^2 per feature (corr[blockIdx.y][f]).
// grid (dp / 256, YB), 256 threads; lane handles features fb + lane + 64 q.
__global__ __launch_bounds__(256) void split_kernel(const float* __restrict__ X, int64_t n,
                                                    int64_t ldx, int d, int64_t dp, int64_t noct,
                                                    unsigned char* __restrict__ XP,
                                                    float* __restrict__ corr) {
  __shared__ float red[4][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t fb = (int64_t)blockIdx.x * 256;
  float sq[4] = {0.f, 0.f, 0.f, 0.f};
  for (int64_t o = (int64_t)blockIdx.y * 4 + w; o < noct; o += (int64_t)gridDim.y * 4) {
    float v[4][8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int64_t row = o * 8 + r;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t f = fb + lane + 64 * q;
        v[q][r] = (row < n && f < d) ? __builtin_nontemporal_load(X + row * ldx + f) : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      u32x4 hv, lv;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const uint32_t h0 = bf16_rne(v[q][2 * p]), h1 = bf16_rne(v[q][2 * p + 1]);
        const float r0 = v[q][2 * p] - __uint_as_float(h0 << 16);
        const float r1 = v[q][2 * p + 1] - __uint_as_float(h1 << 16);
        const uint32_t l0 = bf16_rne(r0), l1 = bf16_rne(r1);
        const float lf0 = __uint_as_float(l0 << 16), lf1 = __uint_as_float(l1 << 16);
        sq[q] += lf0 * lf0 + lf1 * lf1;
        hv[p] = h0 | (h1 << 16);
        lv[p] = l0 | (l1 << 16);
      }
      const int64_t f = fb + lane + 64 * q;
      // [32-row block o/4][panel f/256][slice (o%4)*2 + hi|lo][f%256][16 B]
      unsigned char* dst = XP + ((o >> 2) * (dp / BT) + (f / BT)) * BLOCK_B +
                           ((o & 3) * 2) * SLICE_B + (f % BT) * 16;
      // non-temporal: the image is streamed back from HBM by the SYRK anyway (r04,
      // profiles/r04zv_split_nt_stores_ab.log: config-3 shard 298.7 -> 297.8 ms per op,
      // config 2 26.49 -> 26.33, bit-identical)
      __builtin_nontemporal_store(hv, reinterpret_cast<u32x4*>(dst));
      __builtin_nontemporal_store(lv, reinterpret_cast<u32x4*>(dst + SLICE_B));
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) red[w][lane + 64 * q] = sq[q];
  __syncthreads();
  const int t = threadIdx.x;
  corr[(int64_t)blockIdx.y * dp + fb + t] = red[0][t] + red[1][t] + red[2][t] + red[3][t];
}

// S[i][i] += alpha * sum_y corr[y][i]  (the dropped lo * lo term on the diagonal).
// grid (d / 64): 64 features x 4 row slices per block, the slices summed in order
// (r04: one thread per feature over all yb rows took 110 us at config 3 - 32 blocks,
// each thread a 256-long dependent chain of loads; profiles/r04fin_c3_kernel_stats.csv)
__global__ __launch_bounds__(256) void diag_corr_kernel(const float* __restrict__ corr, int yb,
                                                        int64_t dp, int d, float alpha, float* S,
                                                        int64_t lds) {
  __shared__ float part[4][64];
  const int t = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + t;
  float c = 0.f;
  if (i < d) {
#pragma unroll 8
    for (int y = sl; y < yb; y += 4) c += corr[(int64_t)y * dp + i];
  }
  part[sl][t] = c;
  __syncthreads();
  if (sl == 0 && i < d) S[(int64_t)i * lds + i] += alpha * (((part[0][t] + part[1][t]) + part[2][t]) + part[3][t]);
}

// Lower-triangle tiles in super-tile order (SUPER_H tile rows x SUPER_W tile cols).
// One thread per super-tile (r04: one thread for all took 110 us at d = 16384, 8 per
// config-5 step): a super-row starts after the R0 (R0 + 1) / 2 tiles of the rows above,
// a super-tile after its super-row's tiles left of it.
__global__ __launch_bounds__(256) void tile_order_kernel(int nt, int* order) {
  const int nsc = (nt + SUPER_W - 1) / SUPER_W;
  const int u = blockIdx.x * 256 + threadIdx.x;
  const int R0 = (u / nsc) * SUPER_H, C0 = (u % nsc) * SUPER_W;
  if (R0 >= nt) return;
  const int rmax = R0 + SUPER_H < nt ? R0 + SUPER_H : nt;
  if (C0 >= rmax) return;
  int idx = R0 * (R0 + 1) / 2;
  for (int c = 0; c < C0; c += SUPER_W)
    for (int ti = R0; ti < rmax; ++ti) {
      const int hi = c + SUPER_W < ti + 1 ? c + SUPER_W : ti + 1;
      idx += hi > c ? hi - c : 0;
    }
  for (int ti = R0; ti < rmax; ++ti)
    for (int tj = C0; tj < C0 + SUPER_W && tj <= ti; ++tj) order[idx++] = ti | (tj << 16);
}

// K segments per remainder tile: the smallest nseg (<= 64) whose critical path
// ceil(R nseg / G) / nseg (in full-tile passes) is within 2 % of the best.
int remainder_segments(int64_t R, int G) {
  if (R <= 0) return 0;
  double best = 1e30;
  for (int k = 1; k <= 64; ++k) best = fmin(best, (double)cdiv(R * k, G) / k);
  for (int k = 1; k <= 64; ++k)
    if ((double)cdiv(R * k, G) / k <= best * 1.02) return k;
  return 1;
}

// Compact XCD groups (r05; G = 256 blocks, nt % 8 == 0): the triangle of nt / 8 = m
// block rows of 8 tile rows is cut into m diagonal triangles (36 tiles: a group of 32
// on 8 panels plus 4 left over) and m (m - 1) / 2 off-diagonal 8 x 8 squares (two
// groups of 8 x 4 tiles on 12 panels each).  Group g holds order[32 g .. 32 g + 31]; in
// full phase w XCD x runs group 8 w + x (its G / 8 = 32 blocks, one tile each), so an
// XCD's concurrent tiles share 8-12 panels (the 8 x 4 super-tile order averaged 14.5
// at config 3: its 32-tile runs straddle super-tiles); the two halves of a square run in
// the same phase on neighbouring XCDs.  The 4 m leftover tiles end the order: they are
// the split-K remainder (T mod 256 = 4 m whenever m % 4 == 0).  Groups are listed by
// block row a: the triangle, then squares (a, 0 .. a - 1); block row a starts at group
// a^2.  One thread per group.
__global__ __launch_bounds__(256) void tile_order_compact_kernel(int nt, int* order) {
  const int m = nt / 8;
  const int u = blockIdx.x * 256 + threadIdx.x;
  if (u >= m * m) return;
  int a = (int)sqrtf((float)u);
  while (a * a > u) --a;
  while ((a + 1) * (a + 1) <= u) ++a;
  const int item = u - a * a;
  int* grp = order + 32 * u;
  if (item == 0) {
    int i = 0;
    for (int ti = 8 * a; ti < 8 * a + 8; ++ti)
      for (int tj = 8 * a; tj <= ti; ++tj) {
        const int v = ti | (tj << 16);
        if (i < 32) grp[i] = v;
        else order[32 * m * m + 4 * a + (i - 32)] = v;
        ++i;
      }
  } else {
    const int b = (item - 1) >> 1, h = (item - 1) & 1;
    int i = 0;
    for (int ti = 8 * a; ti < 8 * a + 8; ++ti)
      for (int tj = 8 * b + 4 * h; tj < 8 * b + 4 * h + 4; ++tj) grp[i++] = ti | (tj << 16);
  }
}

// Remainder schedule of the half-ring kernel: bit 0 paces remainder rounds, bit 1
// numbers remainder items XCD-major.  Default 1 since r04 (interleaved A/B in one
// process, profiles/r04za_syrk_*_ab.log, unpaced / paced / XCD-major / both): config 2
// (d = 3072, all 78 tiles remainder) 26.84 / 26.13 / 27.15 / 26.34 ms; d = 4096 22.78 /
// 22.45 / 23.37 / 22.58; d = 5120 71.8 / 66.7 / 72.6 / 66.1; config-3 shard 303.5 /
// 305.0 / 305.0 / 304.1 (its 16 remainder tiles are 1/33 of the work; the XCD-major
// build runs the same schedule there, so ~1.5 ms is the spread).  Unpaced, the blocks
// of a remainder round drift apart over their ~2500 K-tiles as the full phases' did
// (XCD pacing above); XCD-major numbering (each XCD's blocks on K ranges no other XCD
// reads) costs more in balance (nseg a multiple of 8) than it saves in L2 misses.
#ifdef DEIG_AB_SYRK_REM
constexpr int kSyrkRem = DEIG_AB_SYRK_REM;
#else
constexpr int kSyrkRem = 1;
#endif
int syrk_variant(int64_t d);

// XCD-major remainder: segments per XCD (<= 8) whose critical path
// ceil(R xm / gx) / (8 xm) is within 2 % of the best.
int xcd_segments(int64_t R, int gx) {
  double best = 1e30;
  for (int k = 1; k <= 8; ++k) best = fmin(best, (double)cdiv(R * k, gx) / (8 * k));
  for (int k = 1; k <= 8; ++k)
    if ((double)cdiv(R * k, gx) / (8 * k) <= best * 1.02) return k;
  return 1;
}

struct Layout {
  int64_t dp, nt, T, G, q, R, nseg, xm, yb_max, chunk_rows;
  size_t off_order, off_pace, off_accs, off_part, off_corr, off_xp, total;
};

// Workspace: [order][G flush slabs][R * nseg remainder slabs][corr YB x dp][XP chunk].
Layout make_layout(int64_t n, int64_t d, int G, int64_t chunk_rows) {
  Layout L;
  L.dp = cdiv(d, BT) * BT;
  L.nt = L.dp / BT;
  L.T = L.nt * (L.nt + 1) / 2;
  L.G = G;
  L.q = L.T / G;
  L.R = L.T % G;
  L.nseg = remainder_segments(L.R, G);
  L.xm = 0;
  if ((kSyrkRem & 2) && syrk_variant(d) % 100000 >= 30000 && G % 8 == 0 && L.R > 0) {
    L.xm = xcd_segments(L.R, G / 8);
    L.nseg = 8 * L.xm;
  }
  L.yb_max = SPLIT_YB;
  L.chunk_rows = chunk_rows;
  size_t off = 0;
  L.off_order = off;
  off = align_up(off + sizeof(int) * L.T, 256);
  L.off_pace = off;
  off += 16 * 128;  // 8 XCD counters and the chip-wide one, one per 128-B line
  L.off_accs = off;
  off += sizeof(float) * (size_t)G * SLAB;
  L.off_part = off;
  off += sizeof(float) * (size_t)(L.R * L.nseg) * SLAB;
  L.off_corr = off;
  off = align_up(off + sizeof(float) * (size_t)L.yb_max * L.dp, 256);
  L.off_xp = off;
  off += (size_t)chunk_rows * L.dp * 4;
  L.total = off;
  (void)n;
  return L;
}

int64_t default_chunk_rows(int64_t n, int64_t d) {
  const int64_t dp = cdiv(d, BT) * BT;
  const int64_t n32 = cdiv(n, ROWS_PAD) * ROWS_PAD;
  int64_t cap = (int64_t)(DEFAULT_CHUNK_BYTES / (size_t)(dp * 4)) / ROWS_PAD * ROWS_PAD;
  if (cap < ROWS_PAD) cap = ROWS_PAD;
  return n32 < cap ? n32 : cap;
}

// Kernel shape: 163 = fused split (X staged as fp32 and split in LDS), 162 = split
// pass + MFMA 16x16x32, 22 / 13 | 14 | 15 = split pass + 32x32x16 (2 k-steps per
// K-tile x 2 stages; 1 k-step x 3 | 4 | 5 stages).  Default by width: the fused
// split re-splits each panel once per tile that reads it (~d / 256 times), the
// split pass once (2 x 4nd bytes), so the split pass's share of the op falls as
// 1/d while the fused split's stays.  Measured (r02, interleaved A/B in one
// process, profiles/r02l_syrk_fused_ab.log): d = 3072 (config 2) fused 27.3 ms vs
// 29.0 ms; d = 8192 (config 3 shard) fused 370 ms vs 336 ms.
// A/B builds (tools/, never the shipped library) fix one with -DDEIG_AB_SYRK_VARIANT=N.
// Staggered-phase variants are 1PQR0: P phases per K-tile, the next K-tile's
// pieces over Q of them, R = 1: s_setprio(1) around the MFMA clusters; 20DR0: the
// quarter-refill ring (segment_q) with DMA schedule D; 30000: the two-phase half-
// refill ring (segment_h).  Default 30000 since r04 (config-3 shard, interleaved A/B in
// one process, bit-identical, two orders on one box: 310.6 / 312.6 ms against 316.2 /
// 319.3 for two staggered phases 12100 and 322.3 / 322.0 for the r03 default 20100,
// profiles/r04w_syrk_half_ring_ab*.log): two phases halve the barriers per K-tile and
// their 48-MFMA M parts cover the L parts' DMA issue (12100 alone: 311.0 vs 318.0 ms
// for 20100 on another box; four phases 14100 / 14300 350 / 331, eight 360-366 ms,
// s_setprio 12110 323.5, profiles/r04t_*, r04u_*), and the half ring gives every piece
// ~1.5 K-tiles of lead instead of one.  History: r03 20000 315.3 vs 14200 319.6 ms,
// profiles/r03f_syrk_qring_insplit_ab.log; 20100 318.5 vs 20000 323.7 ms,
// profiles/r03l_syrk_dma_schedule_ab.log.  + 100000 * KO adds the knock-outs
// (measurement builds only; the half ring has none).
// The fused split up to d = 2048 since r04 (was 4096): with the half-refill ring the
// split pass wins above (interleaved A/B, profiles/r04y_syrk_*_ab.log: config 2, d =
// 3072, 26.9 vs 28.8 ms; d = 4096 22.7 vs 25.3; d = 2048 26.10 vs 26.09 - a tie, and
// the fused path needs no image of the shard in the workspace).
constexpr int64_t kFusedMaxD = 2048;
#ifdef DEIG_AB_SYRK_VARIANT
constexpr int kSyrkLarge = DEIG_AB_SYRK_VARIANT;
#else
constexpr int kSyrkLarge = 30000;
#endif
int syrk_variant(int64_t d) {
#ifdef DEIG_AB_SYRK_VARIANT
  (void)d;
  return DEIG_AB_SYRK_VARIANT;
#else
  return d <= kFusedMaxD ? 163 : kSyrkLarge;
#endif
}

// The split-pass kernel of variant V (instantiated for kSyrkLarge only).
template <int V>
void launch_split_pass_kernel(int G, hipStream_t stream, const SSched& s) {
  if constexpr (V % 100000 >= 30000) {
    hipLaunchKernelGGL((syrks_h_kernel<(V / 10) % 10>), dim3(G), dim3(NTHR), 0, stream, s);
  }
#ifdef DEIG_AB_SYRK_VARIANT
  else if constexpr (V % 100000 >= 20000) {
    hipLaunchKernelGGL((syrks_q_kernel<(V / 10) % 10, V / 100000, (V / 100) % 10>), dim3(G), dim3(NTHR), 0,
                       stream, s);
  } else if constexpr (V >= 10000) {
    hipLaunchKernelGGL((syrks_st_kernel<(V / 1000) % 10, (V / 100) % 10, (V / 10) % 10, V / 100000>), dim3(G),
                       dim3(NTHR), 0, stream, s);
  } else if constexpr (V == 13 || V == 14 || V == 15) {
    hipLaunchKernelGGL((syrks_kernel<32, 1, V - 10, false>), dim3(G), dim3(NTHR), 0, stream, s);
  } else if constexpr (V == 22) {
    hipLaunchKernelGGL((syrks_kernel<32, 2, 2, false>), dim3(G), dim3(NTHR), 0, stream, s);
  } else {
    hipLaunchKernelGGL((syrks_kernel<16, 2, 2, false>), dim3(G), dim3(NTHR), 0, stream, s);
  }
#else
  else {
    static_assert(V % 100000 >= 30000, "the shipped library has only the half-refill ring");
  }
#endif
}

}  // namespace

// Persistent grid: one block per CU (measurement builds may set a smaller grid, for a
// stream whose CU mask leaves the rest of the chip to other work)
int syrk_cus() {
#ifdef DEIG_AB_SYRK_G
  return DEIG_AB_SYRK_G;
#else
  return num_cus();
#endif
}

size_t syrk_split_workspace_bytes(int64_t n, int64_t d) {
  if (n < 1 || d < 1) return 0;
  if (syrk_variant(d) == 163) return make_layout(n, d, syrk_cus(), 0).total;
  return make_layout(n, d, syrk_cus(), default_chunk_rows(n, d)).total;
}

int syrk_split_launch(const float* X, int64_t n, int64_t d, int64_t ldx, float alpha, float* S,
                      int64_t lds, void* ws, size_t ws_bytes, hipStream_t stream, bool accumulate) {
  DEIG_REQUIRE(n >= 1, "syrk: n must be >= 1 (got %lld)", (long long)n);
  DEIG_REQUIRE(d >= 1 && d % 4 == 0, "syrk: d must be a positive multiple of 4 (got %lld)",
               (long long)d);
  DEIG_REQUIRE(d <= (1 << 16) - BT, "syrk: d too large (%lld)", (long long)d);
  DEIG_REQUIRE(ldx >= d && ldx % 4 == 0, "syrk: ldx must be >= d and a multiple of 4");
  DEIG_REQUIRE(lds >= d && lds % 4 == 0, "syrk: lds must be >= d and a multiple of 4");
  DEIG_REQUIRE(X && S && aligned16(X) && aligned16(S), "syrk: X and S must be 16-byte aligned");
  const int G = syrk_cus();
  const int variant = syrk_variant(d);
  const bool fused = variant == 163;
  // Largest chunk (multiple of 32 rows, <= n rounded up) that fits the workspace.
  Layout L0 = make_layout(n, d, G, 0);
  const size_t ws_min = L0.total + (fused ? 0 : (size_t)ROWS_PAD * L0.dp * 4);
  if (!ws || ws_bytes < ws_min)
    return fail(DEIG_EWORKSPACE, "syrk: workspace %zu bytes < minimum %zu", ws_bytes, ws_min);
  int64_t chunk = (int64_t)((ws_bytes - L0.total) / (size_t)(L0.dp * 4)) / ROWS_PAD * ROWS_PAD;
  const int64_t n32 = cdiv(n, ROWS_PAD) * ROWS_PAD;
  if (chunk > n32) chunk = n32;
  const Layout L = make_layout(n, d, G, fused ? 0 : chunk);
  char* base = static_cast<char*>(ws);

  SSched s;
  s.S = S;
  s.lds = lds;
  s.dp = L.dp;
  s.d = (int)d;
  s.nt = (int)L.nt;
  s.T = (int)L.T;
  s.G = G;
  s.q = (int)L.q;
  s.R = (int)L.R;
  s.alpha = alpha;
  s.order = reinterpret_cast<const int*>(base + L.off_order);
  s.accs = reinterpret_cast<float*>(base + L.off_accs);
  s.part = reinterpret_cast<float*>(base + L.off_part);
  s.XP = reinterpret_cast<const unsigned char*>(base + L.off_xp);
  float* corr = reinterpret_cast<float*>(base + L.off_corr);
  unsigned char* xp = reinterpret_cast<unsigned char*>(base + L.off_xp);

  // Two-level fp32 summation: accumulators are added into a per-block slab every
  // flush_rows rows.  The error bound ~ (flush_rows / 32 + n / flush_rows) eps is
  // smallest at flush_rows ~ sqrt(32 n); each flush is a read-add-write of the block's
  // 256 KiB slab beside stalled MFMAs, and the measured error grows slowly above that
  // point, so the rule is 2^floor(log2 sqrt(128 n)) within [4096, 16384] (r05,
  // interleaved A/B with a float64 check of 64 sampled columns, tools/ab.py syrk,
  // profiles/r05z_syrk_flush_ab.log: config-3 shard 8192 -> 16384 rows 314.2 -> 308.6
  // ms, max error / max|S| 7.0e-7 -> 8.0e-7; config 2 4096 -> 8192 26.58 -> 25.78 ms,
  // 1.9e-7 -> 4.2e-7; 32768 rows at config 3: 305.8 ms but 1.4e-6, config 5's
  // n = 65536 at 16384: 2.0e-6 - not taken; r02: 4096 -> 8192 at config 3 337.6 ->
  // 331.1 ms, profiles/r02l_syrk_flush.log).
#ifdef DEIG_AB_SYRK_FLUSH_ROWS
  int64_t flush_rows = DEIG_AB_SYRK_FLUSH_ROWS;
#else
  int64_t flush_rows = 4096;
  while (flush_rows < 16384 && (flush_rows * 2) * (flush_rows * 2) <= 128 * n) flush_rows *= 2;
#endif
  s.prio = 0;  // s_setprio staggering measured slower (374 vs 342 ms, r02)
  s.pace = reinterpret_cast<unsigned*>(base + L.off_pace);
  // XCD pacing every 64 K-tiles (2048 rows): config 3 L2 hit rate 0.52 -> 0.75, fabric
  // read requests halved, 345 -> 334 ms (r02, interleaved A/B in one process;
  // 16 / 32 / 128 / 256 K-tiles measured 0.3-1.5 % slower).
#ifdef DEIG_AB_SYRK_PACE
  s.pace_kt = DEIG_AB_SYRK_PACE;
#else
  s.pace_kt = 64;
#endif
  s.xm = (int)L.xm;
  s.rpace = kSyrkRem & 1;
#ifndef DEIG_AB_SYRK_SUPER_ORDER
  if (G == 256 && s.nt % 8 == 0)
    hipLaunchKernelGGL(tile_order_compact_kernel, dim3((unsigned)cdiv((s.nt / 8) * (s.nt / 8), 256)), dim3(256), 0,
                       stream, s.nt, reinterpret_cast<int*>(base + L.off_order));
  else
#endif
    hipLaunchKernelGGL(tile_order_kernel,
                       dim3((unsigned)cdiv(cdiv(s.nt, SUPER_H) * cdiv(s.nt, SUPER_W), 256)), dim3(256), 0, stream,
                       s.nt, reinterpret_cast<int*>(base + L.off_order));
  DEIG_HIP_CHECK(hipGetLastError());
  s.X = X;
  s.ldx = ldx;
  s.nrows = n;
  s.corr = corr;
  if (fused) {
    DEIG_REQUIRE(ldx <= (int64_t(1) << 25), "syrk: ldx > 2^25 is not supported for d <= 2048");
    // One pass over all n rows (no XP image, no chunks).  lo^2 partials:
    // [segment < max(1, nseg)][octet wave < 4][dp], zero where no diagonal tile wrote.
    const int64_t yb = 4 * (L.nseg > 1 ? L.nseg : 1);
    DEIG_REQUIRE(yb <= L.yb_max, "syrk: %lld lo^2 partial rows exceed the workspace's %lld",
                 (long long)yb, (long long)L.yb_max);
    DEIG_HIP_CHECK(hipMemsetAsync(corr, 0, sizeof(float) * (size_t)(yb * L.dp), stream));
    s.NK = cdiv(n, ROWS_PAD);
    s.nseg = (int)L.nseg;
    s.beta = accumulate ? 1 : 0;
    s.flush_kt = (int)(flush_rows / ROWS_PAD);
    if (s.flush_kt < 1) s.flush_kt = 1;
    if (s.pace_kt > 0) DEIG_HIP_CHECK(hipMemsetAsync(s.pace, 0, 9 * 128, stream));
    hipLaunchKernelGGL((syrks_kernel<16, 2, 2, true>), dim3(G), dim3(NTHR), 0, stream, s);
    DEIG_HIP_CHECK(hipGetLastError());
    if (s.R > 0) {
      hipLaunchKernelGGL(syrks_reduce_kernel<16>, dim3(s.R, SLAB / 4 / 256), dim3(256), 0, stream, s);
      DEIG_HIP_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(diag_corr_kernel, dim3((unsigned)cdiv(d, 64)), dim3(256), 0, stream, corr,
                       (int)yb, L.dp, (int)d, alpha, S, lds);
    DEIG_HIP_CHECK(hipGetLastError());
    return DEIG_OK;
  }
  for (int64_t r0 = 0, c = 0; r0 < n; r0 += chunk, ++c) {
    const int64_t rows = (n - r0) < chunk ? (n - r0) : chunk;
    const int64_t nk32 = cdiv(rows, ROWS_PAD);  // 32-row blocks (zero-padded)
    const int64_t noct = nk32 * (ROWS_PAD / 8);
    const int kt_steps = (variant >= 13 && variant <= 15) ? 1 : 2;  // k-steps per K-tile
    const int64_t nk = nk32 * (ROWS_PAD / 16) / kt_steps;
    int64_t yb = cdiv(noct, 4);
    if (yb > L.yb_max) yb = L.yb_max;
    hipLaunchKernelGGL(split_kernel, dim3((unsigned)(L.dp / 256), (unsigned)yb), dim3(256), 0,
                       stream, X + r0 * ldx, rows, ldx, (int)d, L.dp, noct, xp, corr);
    DEIG_HIP_CHECK(hipGetLastError());
    s.NK = nk;
    s.nseg = (int)L.nseg;
    s.beta = (c > 0 || accumulate) ? 1 : 0;
    s.flush_kt = (int)(flush_rows / (16 * kt_steps));
    const bool mf16 = variant >= 100;  // 162, 163, 1PQR0, 2000R: 16x16x32 slabs
    if (s.pace_kt > 0) DEIG_HIP_CHECK(hipMemsetAsync(s.pace, 0, 9 * 128, stream));
    if (variant != 163) launch_split_pass_kernel<kSyrkLarge == 163 ? 162 : kSyrkLarge>(G, stream, s);
    DEIG_HIP_CHECK(hipGetLastError());
    if (s.R > 0) {
      if (mf16)
        hipLaunchKernelGGL(syrks_reduce_kernel<16>, dim3(s.R, SLAB / 4 / 256), dim3(256), 0, stream, s);
      else
        hipLaunchKernelGGL(syrks_reduce_kernel<32>, dim3(s.R, SLAB / 4 / 256), dim3(256), 0, stream, s);
      DEIG_HIP_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(diag_corr_kernel, dim3((unsigned)cdiv(d, 64)), dim3(256), 0, stream, corr,
                       (int)yb, L.dp, (int)d, alpha, S, lds);
    DEIG_HIP_CHECK(hipGetLastError());
  }
  return DEIG_OK;
}

}  // namespace deig
