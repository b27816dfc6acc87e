// Skinny GEMM on fp32 MFMA (v_mfma_f32_16x16x4_f32):
//   C[M x N] = alpha * op(A) * B + beta * C,   N <= 256, N % 16 == 0
//   trans_a: A is K x M row-major (op(A) = A^T)   -- S*Q (S symmetric), Z^T Z, W^T*Z
//   !trans_a: A is M x K row-major               -- Wt*Q (server), Xb*V (Oja)
//   B is K x N row-major.
//
// These are the block subspace-iteration products of the eigensolver that
// replaces LAPACK dsyevr in Node.top_k_eigenvectors (distributed.py:22-29) and
// the implicit projector-average operator that replaces the d x d
// sigma_tilde of distributed.py:126-130.  With N = p <= 128 the S*Q sweep
// streams S once: at p <= ~40 it is HBM-bound (4 d^2 bytes), above that it is
// MFMA-bound (2 d^2 p flops).
//
// Block = 4 waves; block tile 64 (M) x N, each wave 16 rows x N (N/16 MFMA
// accumulators).  K advances in chunks of 32 staged through LDS (register
// staging, double buffered, written after the compute of the previous chunk).
// LDS images are k-major ([k][m] and [k][n]) with row strides == 16 (mod 32)
// so the two 16-lane halves of a ds_read_b32 group hit disjoint banks.
// Split-K over gridDim.y writes fp32 partial slabs; skinny_reduce_kernel sums
// them in slice order (deterministic).
#include <stdlib.h>

#include <type_traits>

#include "deig_internal.hpp"

namespace deig {
namespace {

constexpr int SBM = 64;
constexpr int SBK = 32;
constexpr int ST = 256;
constexpr int AST = SBM + 16;  // 80 == 16 mod 32

__host__ __device__ constexpr int bstride(int N) { return (N % 32 == 0) ? N + 16 : N; }

template <int NB, bool TRANS>
__global__ __launch_bounds__(ST) void skinny_kernel(const float* __restrict__ A, int64_t lda,
                                                    const float* __restrict__ B, int64_t ldb,
                                                    float* __restrict__ C, int64_t ldc,
                                                    int64_t M, int64_t K, float alpha, float beta,
                                                    float* __restrict__ part, const ProbBatch pbt) {
  constexpr int N = NB * 16;
  if (const int prob = blockIdx.z) {  // batched: problem blockIdx.z's operands
    const int64_t o = pbt.off[prob];
    A = reinterpret_cast<const float*>(reinterpret_cast<const char*>(A) + o);
    B = reinterpret_cast<const float*>(reinterpret_cast<const char*>(B) + o);
    C = reinterpret_cast<float*>(reinterpret_cast<char*>(C) + o);
    part = reinterpret_cast<float*>(reinterpret_cast<char*>(part) + o);
  }
  constexpr int BST = bstride(N);
  constexpr int NB4 = SBK * N / 4;                 // float4s of a B chunk
  constexpr int BPT = (NB4 + ST - 1) / ST;         // per thread
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;                      // [2][SBK][AST]
  float* Bs = smem + 2 * SBK * AST;      // [2][SBK][BST]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t m0 = (int64_t)blockIdx.x * SBM;
  const int64_t nch = (K + SBK - 1) / SBK;
  const int ks = gridDim.y, sl = blockIdx.y;
  const int64_t c0 = nch * sl / ks, c1 = nch * (sl + 1) / ks;

  f32x4 acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  f32x4 ra[2];
  f32x4 rb[BPT];

  auto load = [&](int64_t ch) {
    const int64_t kb = ch * SBK;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int f = tid + ST * u;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (TRANS) {
        const int row = f >> 4, c4 = f & 15;
        const int64_t k = kb + row, m = m0 + 4 * c4;
        if (k < K && m < M) v = *reinterpret_cast<const f32x4*>(A + k * lda + m);
      } else {
        const int mm = f >> 3, kq = f & 7;
        const int64_t k = kb + 4 * kq, m = m0 + mm;
        if (k < K && m < M) v = *reinterpret_cast<const f32x4*>(A + m * lda + k);
      }
      ra[u] = v;
    }
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      const int f = tid + ST * u;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (f < NB4) {
        const int row = f / (N / 4), c4 = f % (N / 4);
        const int64_t k = kb + row;
        if (k < K) v = *reinterpret_cast<const f32x4*>(B + k * ldb + 4 * c4);
      }
      rb[u] = v;
    }
  };
  auto store = [&](int buf) {
    float* as = As + buf * SBK * AST;
    float* bs = Bs + buf * SBK * BST;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int f = tid + ST * u;
      if (TRANS) {
        const int row = f >> 4, c4 = f & 15;
        *reinterpret_cast<f32x4*>(as + row * AST + 4 * c4) = ra[u];
      } else {
        const int mm = f >> 3, kq = f & 7;
#pragma unroll
        for (int e = 0; e < 4; ++e) as[(4 * kq + e) * AST + mm] = ra[u][e];
      }
    }
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      const int f = tid + ST * u;
      if (f < NB4) {
        const int row = f / (N / 4), c4 = f % (N / 4);
        *reinterpret_cast<f32x4*>(bs + row * BST + 4 * c4) = rb[u];
      }
    }
  };

  const int r = lane & 15, kk = lane >> 4;
  if (c0 < c1) {
    load(c0);
    store(0);
    __syncthreads();
    int cur = 0;
    for (int64_t ch = c0; ch < c1; ++ch) {
      const bool more = ch + 1 < c1;
      if (more) load(ch + 1);
      const float* as = As + cur * SBK * AST + kk * AST + 16 * wave + r;
      const float* bs = Bs + cur * SBK * BST + kk * BST + r;
#pragma unroll
      for (int s = 0; s < SBK / 4; ++s) {
        const float a = as[4 * s * AST];
#pragma unroll
        for (int j = 0; j < NB; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bs[4 * s * BST + 16 * j], acc[j], 0, 0,
                                                       0);
      }
      if (more) store(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  }

  // C/D map of 16x16x4: col = lane & 15, row = 4 * (lane >> 4) + reg
  const int64_t mrow = m0 + 16 * wave + 4 * kk;
  if (ks == 1) {
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t m = mrow + e;
        if (m < M) {
          float* cp = C + m * ldc + 16 * j + r;
          const float v = alpha * acc[j][e];
          *cp = (beta != 0.0f) ? v + beta * *cp : v;
        }
      }
  } else {
    float* pp = part + (int64_t)sl * M * N;
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t m = mrow + e;
        if (m < M) pp[m * N + 16 * j + r] = acc[j][e];
      }
  }
}

// Slabs summed in slice order (deterministic); V = 4: four columns per thread
// (N % 16 == 0; C 16-byte aligned with ldc % 4 == 0), else one.
template <int V>
__global__ __launch_bounds__(256) void skinny_reduce_kernel(const float* __restrict__ part, int ks,
                                                            float* __restrict__ C, int64_t ldc,
                                                            int64_t M, int N, float alpha,
                                                            float beta, const ProbBatch pbt) {
  using fv = std::conditional_t<V == 1, float, f32x4>;
  if (const int prob = blockIdx.y) {
    part = reinterpret_cast<const float*>(reinterpret_cast<const char*>(part) + pbt.off[prob]);
    C = reinterpret_cast<float*>(reinterpret_cast<char*>(C) + pbt.off[prob]);
  }
  const int64_t idx = ((int64_t)blockIdx.x * 256 + threadIdx.x) * V;
  if (idx >= M * N) return;
  const int64_t m = idx / N;
  const int n = (int)(idx - m * N);
  fv s = *reinterpret_cast<const fv*>(part + idx);
#pragma unroll 8
  for (int k = 1; k < ks; ++k) s += *reinterpret_cast<const fv*>(part + (int64_t)k * M * N + idx);
  fv* cp = reinterpret_cast<fv*>(C + m * ldc + n);
  const fv v = alpha * s;
  *cp = (beta != 0.0f) ? v + beta * *cp : v;
}

template <int NB, bool TRANS>
int launch_nb(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
              int64_t M, int64_t K, float alpha, float beta, float* part, int ks,
              hipStream_t st, const ProbBatch& pbt) {
  constexpr int N = NB * 16;
  const size_t shm = (size_t)(2 * SBK * AST + 2 * SBK * bstride(N)) * sizeof(float);
  // once per instantiation (C++11 thread-safe static initialisation)
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)skinny_kernel<NB, TRANS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  DEIG_HIP_CHECK(attr);
  dim3 grid((unsigned)cdiv(M, SBM), (unsigned)ks, (unsigned)pbt.n);
  hipLaunchKernelGGL((skinny_kernel<NB, TRANS>), grid, dim3(ST), shm, st, A, lda, B, ldb, C, ldc,
                     M, K, alpha, beta, part, pbt);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

template <bool TRANS>
int launch_t(int NB, const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
             int64_t ldc, int64_t M, int64_t K, float alpha, float beta, float* part, int ks,
             hipStream_t st, const ProbBatch& pbt) {
  switch (NB) {
#define DEIG_NB(x) \
  case x:          \
    return launch_nb<x, TRANS>(A, lda, B, ldb, C, ldc, M, K, alpha, beta, part, ks, st, pbt);
    DEIG_NB(1) DEIG_NB(2) DEIG_NB(3) DEIG_NB(4) DEIG_NB(5) DEIG_NB(6) DEIG_NB(7) DEIG_NB(8)
    DEIG_NB(9) DEIG_NB(10) DEIG_NB(11) DEIG_NB(12) DEIG_NB(13) DEIG_NB(14) DEIG_NB(15)
    DEIG_NB(16)
#undef DEIG_NB
    default:
      return fail(DEIG_EINVAL, "skinny: unsupported N = %d", NB * 16);
  }
}

// Split-K factor: enough blocks for ~4 resident per CU (latency hiding: HBM
// latency under load is ~1-2 us, one chunk of MFMA work ~0.5 us), >= 8 chunks
// per slice.
constexpr int kBlocksPerCu = 4;

int choose_ks(int64_t M, int64_t K) {
  const int64_t mb = cdiv(M, SBM);
  const int64_t nch = cdiv(K, SBK);
  int64_t ks = cdiv((int64_t)kBlocksPerCu * num_cus(), mb);
  const int64_t cap = nch / 8 > 1 ? nch / 8 : 1;
  if (ks > cap) ks = cap;
  if (ks < 1) ks = 1;
  if (ks > 1024) ks = 1024;
  return (int)ks;
}

}  // namespace

size_t skinny_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  const int ks = choose_ks(M, K);
  return ks > 1 ? (size_t)ks * M * N * sizeof(float) : 0;
}

int skinny_launch(bool trans_a, const float* A, int64_t lda, const float* B, int64_t ldb,
                  float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, float alpha,
                  float beta, float* slab, size_t slab_bytes, hipStream_t stream,
                  const ProbBatch* batch) {
  DEIG_REQUIRE(N >= 16 && N <= 256 && N % 16 == 0, "skinny: N=%lld must be 16..256, %%16",
               (long long)N);
  const ProbBatch pbt = batch ? *batch : one_problem();
  DEIG_REQUIRE(pbt.n >= 1 && pbt.n <= kMaxProbBatch && pbt.off[0] == 0, "skinny: batch of %d", pbt.n);
  DEIG_REQUIRE(M >= 1 && K >= 1, "skinny: empty problem");
  DEIG_REQUIRE(lda % 4 == 0 && ldb % 4 == 0 && ldb >= N && ldc >= N, "skinny: bad leading dims");
  DEIG_REQUIRE(aligned16(A) && aligned16(B), "skinny: A, B must be 16-byte aligned");
  if (trans_a)
    DEIG_REQUIRE(M % 4 == 0 && lda >= M, "skinny(T): M %% 4 and lda >= M required");
  else
    DEIG_REQUIRE(K % 4 == 0 && lda >= K, "skinny(N): K %% 4 and lda >= K required");
  const int ks = choose_ks(M, K);
  const size_t need = ks > 1 ? (size_t)ks * M * N * sizeof(float) : 0;
  if (slab_bytes < need) return fail(DEIG_EWORKSPACE, "skinny: slab %zu < %zu", slab_bytes, need);
  const int NB = (int)(N / 16);
  int rc = trans_a ? launch_t<true>(NB, A, lda, B, ldb, C, ldc, M, K, alpha, beta, slab, ks, stream, pbt)
                   : launch_t<false>(NB, A, lda, B, ldb, C, ldc, M, K, alpha, beta, slab, ks,
                                     stream, pbt);
  if (rc) return rc;
  if (ks > 1) {
    const int64_t tot = M * N;
    if (ldc % 4 == 0 && aligned16(C))
      hipLaunchKernelGGL(skinny_reduce_kernel<4>, dim3((unsigned)cdiv(tot / 4, 256), (unsigned)pbt.n),
                         dim3(256), 0, stream, slab, ks, C, ldc, M, (int)N, alpha, beta, pbt);
    else
      hipLaunchKernelGGL(skinny_reduce_kernel<1>, dim3((unsigned)cdiv(tot, 256), (unsigned)pbt.n),
                         dim3(256), 0, stream, slab, ks, C, ldc, M, (int)N, alpha, beta, pbt);
    DEIG_HIP_CHECK(hipGetLastError());
  }
  return DEIG_OK;
}

}  // namespace deig
