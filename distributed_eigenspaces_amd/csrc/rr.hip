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

__global__ __launch_bounds__(256) void rr_init_kernel(float* __restrict__ Z, int64_t d, int p,
                                                      const float* __restrict__ Q0, int k0,
                                                      int64_t ldq0, uint64_t seed) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * p) return;
  const int64_t r = idx / p;
  const int j = (int)(idx - r * p);
  float v;
  if (j < k0) {
    v = Q0[r + (int64_t)j * ldq0];
  } else {
    const uint64_t h = mix64(seed ^ mix64((uint64_t)r * 0x100000001B3ull + (uint64_t)j));
    v = (float)((double)(h >> 11) * (1.0 / 9007199254740992.0)) * 2.0f - 1.0f;
  }
  Z[r * 2 * p + j] = v;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  // RT threads -> one value, broadcast.  red has >= RT/64 + 1 floats.
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < RT / 64; ++i) s += red[i];
    red[RT / 64] = s;
  }
  __syncthreads();
  return red[RT / 64];
}

__global__ __launch_bounds__(RT) void rr_small_kernel(const float* __restrict__ Cg, int p,
                                                      float* __restrict__ Linv_g,
                                                      float* __restrict__ Wtmp_g,
                                                      float* __restrict__ Wout,
                                                      float* __restrict__ lam_out,
                                                      float* __restrict__ cs_out,
                                                      int* __restrict__ info, int max_jsweeps) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int pp = p * p;
  float* X1 = sm;
  float* X2 = sm + pp;
  float* dsc = X2 + pp;   // p
  float* gam = dsc + p;   // p
  float* sig = gam + p;   // p
  float* lamv = sig + p;  // p
  float* gd = lamv + p;   // p
  int* part = reinterpret_cast<int*>(gd + p);  // p
  int* rank = part + p;                        // p
  float* red = reinterpret_cast<float*>(rank + p);  // RT/64 + 2
  const int tid = threadIdx.x;
  const int ldc = 2 * p;
  const float* Mg = Cg;
  const float* Hg = Cg + p;
  const float* Gg = Cg + (int64_t)p * ldc + p;

  // ---- 0. column scaling of Q
  for (int a = tid; a < p; a += RT) {
    const float m = Mg[a * ldc + a];
    dsc[a] = (m > 0.f && isfinite(m)) ? rsqrtf(m) : 1.0f;
  }
  if (tid == 0) info[0] = 0;
  __syncthreads();
  for (int idx = tid; idx < pp; idx += RT) {
    const int a = idx / p, b = idx - a * p;
    X1[idx] = Mg[a * ldc + b] * dsc[a] * dsc[b];
  }
  __syncthreads();

  // ---- 1. Cholesky  D M D = L L^T  (lower, in place in X1), pivots floored
  for (int j = 0; j < p; ++j) {
    if (tid == 0) {
      float v = X1[j * p + j];
      if (!(v > 1e-6f)) {
        v = 1e-6f;
        info[0] += 1;
      }
      X1[j * p + j] = sqrtf(v);
    }
    __syncthreads();
    const float inv = 1.0f / X1[j * p + j];
    for (int i = j + 1 + tid; i < p; i += RT) X1[i * p + j] *= inv;
    __syncthreads();
    const int n = p - j - 1;
    for (int idx = tid; idx < n * n; idx += RT) {
      const int i = j + 1 + idx / n, c = j + 1 + idx % n;
      if (c <= i) X1[i * p + c] -= X1[i * p + j] * X1[c * p + j];
    }
    __syncthreads();
  }

  // ---- 2. L^-1 (lower) into X2, row by row
  for (int idx = tid; idx < pp; idx += RT) X2[idx] = 0.f;
  __syncthreads();
  for (int i = 0; i < p; ++i) {
    const float inv = 1.0f / X1[i * p + i];
    for (int c = tid; c <= i; c += RT) {
      float s = (c == i) ? 1.0f : 0.0f;
      for (int t = c; t < i; ++t) s -= X1[i * p + t] * X2[t * p + c];
      X2[i * p + c] = s * inv;
    }
    __syncthreads();
  }
  for (int idx = tid; idx < pp; idx += RT) Linv_g[idx] = X2[idx];
  __syncthreads();

  // ---- 3. T1 = L^-1 (D H D) -> X1
  for (int idx = tid; idx < pp; idx += RT) {
    const int a = idx / p, b = idx - a * p;
    float s = 0.f;
    for (int t = 0; t <= a; ++t) s += X2[a * p + t] * (Hg[t * ldc + b] * dsc[t]);
    X1[idx] = s * dsc[b];
  }
  __syncthreads();
  // ---- 4. H~ = T1 L^-T -> X2   (L^-1 re-read from global; X2 is overwritten)
  for (int idx = tid; idx < pp; idx += RT) {
    const int a = idx / p, b = idx - a * p;
    float s = 0.f;
    for (int t = 0; t <= b; ++t) s += X1[a * p + t] * Linv_g[b * p + t];
    X2[idx] = s;
  }
  __syncthreads();
  for (int idx = tid; idx < pp; idx += RT) {
    const int a = idx / p, b = idx - a * p;
    if (a < b) {
      const float v = 0.5f * (X2[a * p + b] + X2[b * p + a]);
      X2[a * p + b] = v;
      X2[b * p + a] = v;
    }
  }
  for (int idx = tid; idx < pp; idx += RT) {
    const int a = idx / p, b = idx - a * p;
    X1[idx] = (a == b) ? 1.0f : 0.0f;
  }
  __syncthreads();

  // ---- 5. parallel cyclic Jacobi on X2; eigenvectors accumulate in X1 (columns)
  const int half = p >> 1;
  for (int sw = 0; sw < max_jsweeps; ++sw) {
    float off = 0.f, dg = 0.f;
    for (int idx = tid; idx < pp; idx += RT) {
      const int a = idx / p, b = idx - a * p;
      const float v = X2[idx];
      if (a == b) dg += v * v; else off += v * v;
    }
    off = block_sum(off, red);
    dg = block_sum(dg, red);
    if (off <= 1e-14f * dg) break;
    for (int st = 0; st < p - 1; ++st) {
      if (tid < half) {
        int a, b;
        if (tid == 0) {
          a = p - 1;
          b = st;
        } else {
          a = (st + tid) % (p - 1);
          b = (st - tid + (p - 1)) % (p - 1);
        }
        const float app = X2[a * p + a], aqq = X2[b * p + b], apq = X2[a * p + b];
        float c = 1.f, s = 0.f;
        if (fabsf(apq) > 1e-30f && fabsf(apq) > 1e-9f * sqrtf(fabsf(app * aqq))) {
          const float tau = (aqq - app) / (2.f * apq);
          const float t = (fabsf(tau) > 1e18f)
                              ? 0.5f / tau
                              : copysignf(1.f, tau) / (fabsf(tau) + sqrtf(1.f + tau * tau));
          c = rsqrtf(1.f + t * t);
          s = t * c;
        }
        gam[a] = c; sig[a] = -s; part[a] = b;
        gam[b] = c; sig[b] = s;  part[b] = a;
      }
      __syncthreads();
      float nv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int idx = tid + u * RT;
        nv[u] = 0.f;
        if (idx < pp) {
          const int r = idx / p, c = idx - r * p;
          const int r2 = part[r], c2 = part[c];
          const float gr = gam[r], sr = sig[r], gc = gam[c], sc = sig[c];
          nv[u] = gr * (gc * X2[r * p + c] + sc * X2[r * p + c2]) +
                  sr * (gc * X2[r2 * p + c] + sc * X2[r2 * p + c2]);
        }
      }
      // eigenvector columns: V[:, x] <- gam_x V[:, x] + sig_x V[:, partner(x)]
      for (int idx = tid; idx < p * half; idx += RT) {
        const int r = idx / half, t = idx - r * half;
        int a = (t == 0) ? p - 1 : (st + t) % (p - 1);
        const int b = part[a];
        const float va = X1[r * p + a], vb = X1[r * p + b];
        X1[r * p + a] = gam[a] * va + sig[a] * vb;
        X1[r * p + b] = gam[b] * vb + sig[b] * va;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int idx = tid + u * RT;
        if (idx < pp) X2[idx] = nv[u];
      }
      __syncthreads();
    }
  }

  // ---- 6. W = D L^-T U -> Wtmp_g ; eigenvalues -> lamv
  for (int a = tid; a < p; a += RT) lamv[a] = X2[a * p + a];
  for (int idx = tid; idx < pp; idx += RT) {
    const int a = idx / p, j = idx - a * p;
    float s = 0.f;
    for (int t = a; t < p; ++t) s += Linv_g[t * p + a] * X1[t * p + j];
    Wtmp_g[idx] = s * dsc[a];
  }
  __syncthreads();
  for (int idx = tid; idx < pp; idx += RT) X1[idx] = Wtmp_g[idx];
  __syncthreads();
  // ---- 7. g_j = w_j^T G w_j
  for (int idx = tid; idx < pp; idx += RT) {
    const int a = idx / p, j = idx - a * p;
    float s = 0.f;
    for (int b = 0; b < p; ++b) s += Gg[a * ldc + b] * X1[b * p + j];
    X2[idx] = s;
  }
  __syncthreads();
  for (int j = tid; j < p; j += RT) {
    float s = 0.f;
    for (int a = 0; a < p; ++a) s += X1[a * p + j] * X2[a * p + j];
    gd[j] = s;
    // rank for descending order (ties by index)
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
  for (int j = tid; j < p; j += RT) {
    const int rk = rank[j];
    lam_out[rk] = lamv[j];
    cs_out[rk] = (gd[j] > gthr && gd[j] > 0.f) ? rsqrtf(gd[j]) : 0.f;
  }
  for (int idx = tid; idx < pp; idx += RT) {
    const int a = idx / p, j = idx - a * p;
    Wout[a * p + rank[j]] = X1[idx];
  }
}

__global__ __launch_bounds__(256) void rr_update_kernel(float* __restrict__ Z, int64_t d, int p,
                                                        int k, const float* __restrict__ W,
                                                        const float* __restrict__ lam,
                                                        const float* __restrict__ cs,
                                                        float* __restrict__ V, int64_t ldv,
                                                        float* __restrict__ resid_part) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ws = sm;              // p x p
  float* Zs = sm + p * p;      // UR x 2p
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * UR;
  const int ld = 2 * p;
  for (int idx = tid; idx < p * p; idx += 256) Ws[idx] = W[idx];
  for (int idx = tid; idx < UR * ld; idx += 256) {
    const int rr = idx / ld, c = idx - rr * ld;
    const int64_t row = r0 + rr;
    Zs[idx] = (row < d) ? Z[row * ld + c] : 0.f;
  }
  __syncthreads();
  for (int j = tid; j < p; j += 256) {
    const float lj = lam[j], cj = cs[j];
    float racc = 0.f;
    for (int rr = 0; rr < UR; ++rr) {
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
      if (j < k) {
        const float e = yw - lj * qw;
        racc = fmaf(e, e, racc);
        V[row + (int64_t)(k - 1 - j) * ldv] = qw;
      }
      Z[row * ld + j] = (cj > 0.f) ? yw * cj : qw;
    }
    if (j < k) resid_part[(int64_t)blockIdx.x * k + j] = racc;
  }
}

__global__ __launch_bounds__(256) void rr_finish_kernel(const float* __restrict__ resid_part,
                                                        int nblk, int k,
                                                        const float* __restrict__ lam,
                                                        float* __restrict__ evals,
                                                        float* __restrict__ resid) {
  __shared__ float mx[256];
  const int tid = threadIdx.x;
  const float scale = fmaxf(fabsf(lam[0]), 1e-30f);
  float m = 0.f;
  for (int j = tid; j < k; j += 256) {
    float s = 0.f;
    for (int b = 0; b < nblk; ++b) s += resid_part[(int64_t)b * k + j];
    const float rel = sqrtf(s) / scale;
    resid[j] = rel;
    evals[k - 1 - j] = lam[j];
    m = fmaxf(m, rel);
  }
  mx[tid] = m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) mx[tid] = fmaxf(mx[tid], mx[tid + o]);
    __syncthreads();
  }
  if (tid == 0) resid[k] = mx[0];
}

size_t rr_small_shm(int p) {
  return (size_t)(2 * p * p + 7 * p + RT / 64 + 8) * sizeof(float);
}

}  // namespace

int rr_init_launch(float* Z, int64_t d, int p, const float* Q0, int k0, int64_t ldq0,
                   uint64_t seed, hipStream_t stream) {
  const int64_t tot = d * p;
  hipLaunchKernelGGL(rr_init_kernel, dim3((unsigned)cdiv(tot, 256)), dim3(256), 0, stream, Z, d,
                     p, Q0, k0, ldq0, seed);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

int rr_small_launch(const RRBuffers& b, int p, hipStream_t stream) {
  DEIG_REQUIRE(p >= 2 && p <= 128 && p % 2 == 0, "rr_small: p=%d out of range", p);
  const size_t shm = rr_small_shm(p);
  static bool attr = false;
  if (!attr) {
    DEIG_HIP_CHECK(hipFuncSetAttribute((const void*)rr_small_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)rr_small_shm(128)));
    attr = true;
  }
  hipLaunchKernelGGL(rr_small_kernel, dim3(1), dim3(RT), shm, stream, b.C, p, b.Linv, b.Wtmp, b.W,
                     b.lam, b.cs, b.info, 30);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

int rr_update_blocks(int64_t d) { return (int)cdiv(d, UR); }

int rr_update_launch(const RRBuffers& b, int64_t d, int p, int k, float* V, int64_t ldv,
                     float* evals, hipStream_t stream) {
  const int nblk = rr_update_blocks(d);
  const size_t shm = (size_t)(p * p + UR * 2 * p) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    DEIG_HIP_CHECK(hipFuncSetAttribute((const void*)rr_update_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)((128 * 128 + UR * 256) * sizeof(float))));
    attr = true;
  }
  hipLaunchKernelGGL(rr_update_kernel, dim3(nblk), dim3(256), shm, stream, b.Z, d, p, k, b.W,
                     b.lam, b.cs, V, ldv, b.resid_part);
  DEIG_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(rr_finish_kernel, dim3(1), dim3(256), 0, stream, b.resid_part, nblk, k, b.lam,
                     evals, b.resid);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

}  // namespace deig
