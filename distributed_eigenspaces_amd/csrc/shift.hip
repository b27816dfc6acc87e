// Mean-shifted covariance of float samples (the reference's float64 data flow).
//
// The reference hands float64 grey values (distributed.py:169-173: data.mean(axis=3),
// reshape) to compute_sigma_hat_ (:59-70), an UNCENTERED second moment: on byte
// images the mean direction's eigenvalue is ~10^4 x the k-th one, and an fp32-grade
// SYRK of the raw values carries its rounding relative to that dominant scale -
// numpy emulation (tools/emulate_f64flow.py, c1 / c1g shapes): 0.8-1.4e-4 in
// ||P - P_ref||_F and 1.7-1.9e-5 in the eigenvalues, over the bars.  Shifting first,
//   t_r = x_r - mu  (double),   c_r = fl32(t_r),   s = sum_r t_r  (double),
//   Sigma = alpha [ C^T C + s mu^T + mu s^T + n mu mu^T ]        (exact identity)
// puts the SYRK's error on the CENTRED scale (split3 of C: 1.1-1.9e-6 / 7e-8 in the
// same emulation); the rank-one terms are added in double and the result is kept
// in float64 (fp32 storage of the uncentered Sigma alone costs 2.6-4.4e-5).
//
// Pipeline: colsum (per row group, double) -> mu; center (C = fl32(X - mu) with row
// stride dp, zero padding columns, + per-group sums of t in double) -> s; the
// covariance SYRK of C (split3 / fp32 by n, syrk_split.hip / syrk.hip) into an fp32
// image Sc = alpha C^T C; shift_finalize: S64 = Sc + alpha (s mu^T + mu s^T + n mu mu^T)
// written from symmetric expressions (bit-exact symmetry), and optionally S = fl32(S64).
#include "deig_internal.hpp"

namespace deig {
namespace {

constexpr int CS_YB = 128;  // row groups of the column passes

template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* __restrict__ X, int64_t n,
                                                     int64_t ldx, int64_t d,
                                                     double* __restrict__ part) {
  const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (f >= d) return;
  const int64_t ys = gridDim.y;
  double s0 = 0.0, s1 = 0.0;
  int64_t r = blockIdx.y;
  for (; r + ys < n; r += 2 * ys) {  // two independent chains
    s0 += (double)X[r * ldx + f];
    s1 += (double)X[(r + ys) * ldx + f];
  }
  if (r < n) s0 += (double)X[r * ldx + f];
  part[(int64_t)blockIdx.y * d + f] = s0 + s1;
}

// out[f] = scale * sum_y part[y][f]  (fixed order: deterministic)
__global__ __launch_bounds__(256) void colreduce_kernel(const double* __restrict__ part, int yb,
                                                        int64_t d, double scale,
                                                        double* __restrict__ out) {
  const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (f >= d) return;
  double s = 0.0;
  for (int y = 0; y < yb; ++y) s += part[(int64_t)y * d + f];
  out[f] = scale * s;
}

template <typename T>
__global__ __launch_bounds__(256) void center_kernel(const T* __restrict__ X, int64_t n,
                                                     int64_t ldx, int64_t d, int64_t dp,
                                                     const double* __restrict__ mu,
                                                     float* __restrict__ C,
                                                     double* __restrict__ part) {
  const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (f >= dp) return;
  const bool live = f < d;
  const double m = live ? mu[f] : 0.0;
  double s = 0.0;
  for (int64_t r = blockIdx.y; r < n; r += gridDim.y) {
    const double t = live ? (double)X[r * ldx + f] - m : 0.0;
    C[r * dp + f] = (float)t;
    s += t;
  }
  part[(int64_t)blockIdx.y * dp + f] = s;
}

__global__ __launch_bounds__(256) void shift_finalize_kernel(const float* __restrict__ Sc,
                                                             int64_t ldc, int64_t d,
                                                             const double* __restrict__ mu,
                                                             const double* __restrict__ sv,
                                                             double n, double alpha,
                                                             double* __restrict__ S64,
                                                             int64_t lds64, float* __restrict__ S,
                                                             int64_t lds) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * d) return;
  const int64_t i = idx / d, j = idx - i * d;
  // every expression symmetric in (i, j): + and * commute, Sc is bit-symmetric.
  // No contraction: fused into fma(sv_i, mu_j, mu_i sv_j) the cross term would round
  // differently for (j, i) - r03's float64 Sigma was not bit-symmetric
  // (tests/test_gpu_integration_stub.py).
  const double mi = mu[i], mj = mu[j];
  double cross;
  {
#pragma clang fp contract(off)
    cross = sv[i] * mj + mi * sv[j];
  }
  const double v = (double)Sc[i * ldc + j] + alpha * (cross + n * (mi * mj));
  if (S64) S64[i * lds64 + j] = v;
  if (S) S[i * lds + j] = (float)v;
}

struct ShiftLayout {
  int64_t dp;
  int yb;
  int algo;
  size_t off_part, off_mu, off_s, off_c, off_sc, off_syrk, syrk_bytes, total;
};

ShiftLayout shift_layout(int64_t n, int64_t d) {
  ShiftLayout L;
  L.dp = cdiv(d, 4) * 4;
  L.yb = (int)(n < CS_YB ? (n > 0 ? n : 1) : CS_YB);
  L.algo = n >= DEIG_SYRK_SPLIT_MIN_ROWS ? DEIG_SYRK_SPLIT3 : DEIG_SYRK_FP32;
  L.syrk_bytes = L.algo == DEIG_SYRK_SPLIT3 ? syrk_split_workspace_bytes(n, L.dp)
                                            : syrk_workspace_bytes(n, L.dp);
  size_t off = 0;
  L.off_part = off;
  off = align_up(off + (size_t)L.yb * L.dp * sizeof(double), 256);
  L.off_mu = off;
  off = align_up(off + (size_t)L.dp * sizeof(double), 256);
  L.off_s = off;
  off = align_up(off + (size_t)L.dp * sizeof(double), 256);
  L.off_c = off;
  off = align_up(off + (size_t)n * L.dp * sizeof(float), 256);
  L.off_sc = off;
  off = align_up(off + (size_t)L.dp * L.dp * sizeof(float), 256);
  L.off_syrk = off;
  L.total = L.off_syrk + L.syrk_bytes;
  return L;
}

template <typename T>
int shift_run(const T* X, int64_t n, int64_t d, int64_t ldx, double alpha, double* S64,
              int64_t lds64, float* S, int64_t lds, char* base, const ShiftLayout& L,
              hipStream_t st) {
  double* part = reinterpret_cast<double*>(base + L.off_part);
  double* mu = reinterpret_cast<double*>(base + L.off_mu);
  double* sv = reinterpret_cast<double*>(base + L.off_s);
  float* C = reinterpret_cast<float*>(base + L.off_c);
  float* Sc = reinterpret_cast<float*>(base + L.off_sc);
  void* sws = base + L.off_syrk;
  const dim3 g1((unsigned)cdiv(d, 256), (unsigned)L.yb), gp((unsigned)cdiv(L.dp, 256), (unsigned)L.yb);
  hipLaunchKernelGGL(colsum_kernel<T>, g1, dim3(256), 0, st, X, n, ldx, d, part);
  DEIG_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(colreduce_kernel, dim3((unsigned)cdiv(d, 256)), dim3(256), 0, st, part, L.yb,
                     d, 1.0 / (double)n, mu);
  DEIG_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(center_kernel<T>, gp, dim3(256), 0, st, X, n, ldx, d, L.dp, mu, C, part);
  DEIG_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(colreduce_kernel, dim3((unsigned)cdiv(d, 256)), dim3(256), 0, st, part, L.yb,
                     L.dp, 1.0, sv);
  DEIG_HIP_CHECK(hipGetLastError());
  int rc = L.algo == DEIG_SYRK_SPLIT3
               ? syrk_split_launch(C, n, L.dp, L.dp, (float)alpha, Sc, L.dp, sws, L.syrk_bytes, st)
               : syrk_launch(C, n, L.dp, L.dp, (float)alpha, Sc, L.dp, sws, L.syrk_bytes, st);
  if (rc) return rc;
  hipLaunchKernelGGL(shift_finalize_kernel, dim3((unsigned)cdiv(d * d, 256)), dim3(256), 0, st, Sc,
                     L.dp, d, mu, sv, (double)n, alpha, S64, lds64, S, lds);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

}  // namespace

size_t syrk_shift_workspace_bytes(int64_t n, int64_t d, int xtype) {
  (void)xtype;
  if (n < 1 || d < 1) return 0;
  return shift_layout(n, d).total;
}

int syrk_shift_launch(const void* X, int xtype, int64_t n, int64_t d, int64_t ldx, double alpha,
                      double* S64, int64_t lds64, float* S, int64_t lds, void* ws, size_t ws_bytes,
                      hipStream_t st) {
  DEIG_REQUIRE(xtype == DEIG_F32 || xtype == DEIG_F64, "syrk_shift: unknown element type %d", xtype);
  DEIG_REQUIRE(n >= 1 && d >= 1, "syrk_shift: need n >= 1, d >= 1");
  DEIG_REQUIRE(ldx >= d, "syrk_shift: ldx must be >= d");
  DEIG_REQUIRE(X && (reinterpret_cast<uintptr_t>(X) % (xtype == DEIG_F64 ? 8 : 4)) == 0,
               "syrk_shift: X must be aligned to its element size");
  DEIG_REQUIRE(S64 || S, "syrk_shift: need S64 and/or S");
  DEIG_REQUIRE(!S64 || lds64 >= d, "syrk_shift: lds64 must be >= d");
  DEIG_REQUIRE(!S || lds >= d, "syrk_shift: lds must be >= d");
  const ShiftLayout L = shift_layout(n, d);
  if (!ws || ws_bytes < L.total)
    return fail(DEIG_EWORKSPACE, "syrk_shift: workspace %zu bytes < required %zu", ws_bytes, L.total);
  char* base = static_cast<char*>(ws);
  if (xtype == DEIG_F64)
    return shift_run(static_cast<const double*>(X), n, d, ldx, alpha, S64, lds64, S, lds, base, L, st);
  return shift_run(static_cast<const float*>(X), n, d, ldx, alpha, S64, lds64, S, lds, base, L, st);
}

}  // namespace deig
