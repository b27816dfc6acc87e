// Projection onto the estimated eigenspace:  Y = X W  (Online Distributed
// PCA.ipynb raw line 345: online_distributed_PCA = lambda X: X @ matrix_w).
// X: n x d row-major, W: d x k column-major (the solvers' output), Y: n x k
// row-major.  One skinny NN GEMM (HBM-bound: X is streamed once).
#include "deig_internal.hpp"

namespace deig {
namespace {

__global__ __launch_bounds__(256) void w_to_rowpad(const float* __restrict__ W, int64_t ldw,
                                                   int64_t d, int k, int kp,
                                                   float* __restrict__ Wr) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * kp) return;
  const int64_t r = idx / kp;
  const int j = (int)(idx - r * kp);
  Wr[idx] = (j < k) ? W[r + (int64_t)j * ldw] : 0.f;
}

__global__ __launch_bounds__(256) void crop_rows(const float* __restrict__ T, int64_t n, int k,
                                                 int kp, float* __restrict__ Y, int64_t ldy) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n * k) return;
  const int64_t r = idx / k;
  const int j = (int)(idx - r * k);
  Y[r * ldy + j] = T[r * kp + j];
}

struct ProjWs {
  float *Wr, *T, *slab;
  size_t slab_bytes;
};

ProjWs carve_proj(void* ws, size_t cap, int64_t n, int64_t d, int kp, bool direct, size_t* total) {
  Carve c(ws, cap);
  ProjWs o;
  o.Wr = c.take<float>((size_t)d * kp);
  o.T = direct ? nullptr : c.take<float>((size_t)n * kp);
  o.slab_bytes = skinny_workspace_bytes(n, kp, d);
  o.slab = c.take<float>(o.slab_bytes / sizeof(float) + 4);
  *total = c.off;
  return o;
}

}  // namespace

size_t project_workspace_bytes(int64_t n, int64_t d, int k) {
  const int kp = (int)cdiv(k, 16) * 16;
  size_t total = 0;
  carve_proj(nullptr, 0, n, d, kp, false, &total);
  return total;
}

int project_launch(const float* X, int64_t n, int64_t d, int64_t ldx, const float* W, int k,
                   int64_t ldw, float* Y, int64_t ldy, void* ws, size_t ws_bytes, hipStream_t st) {
  DEIG_REQUIRE(n >= 1 && d >= 4 && d % 4 == 0, "project: need n >= 1, d %% 4 == 0");
  DEIG_REQUIRE(k >= 1 && k <= 256 && ldw >= d && ldy >= k && ldx >= d && ldx % 4 == 0,
               "project: bad k or leading dims");
  DEIG_REQUIRE(X && W && Y && aligned16(X), "project: X must be 16-byte aligned");
  const int kp = (int)cdiv(k, 16) * 16;
  const bool direct = (k == kp) && ldy % 4 == 0 && aligned16(Y);
  size_t total = 0;
  ProjWs o = carve_proj(ws, ws_bytes, n, d, kp, direct, &total);
  if (!ws || total > ws_bytes)
    return fail(DEIG_EWORKSPACE, "project: workspace %zu < %zu", ws_bytes, total);
  hipLaunchKernelGGL(w_to_rowpad, dim3((unsigned)cdiv(d * kp, 256)), dim3(256), 0, st, W, ldw, d,
                     k, kp, o.Wr);
  DEIG_HIP_CHECK(hipGetLastError());
  int rc = skinny_launch(false, X, ldx, o.Wr, kp, direct ? Y : o.T, direct ? ldy : kp, n, kp, d,
                         1.f, 0.f, o.slab, o.slab_bytes, st);
  if (rc) return rc;
  if (!direct) {
    hipLaunchKernelGGL(crop_rows, dim3((unsigned)cdiv(n * k, 256)), dim3(256), 0, st, o.T, n, k,
                       kp, Y, ldy);
    DEIG_HIP_CHECK(hipGetLastError());
  }
  return DEIG_OK;
}

}  // namespace deig
