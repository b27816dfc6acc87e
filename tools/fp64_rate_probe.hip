// Throughput probe: fp64 VALU FMA vs fp64 MFMA vs fp32 VALU FMA on gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void valu64(double* out, int iters, double a) {
  double acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = threadIdx.x * 1e-3 + i;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = fma(acc[i], a, 1e-9);
  double s = 0;
  for (int i = 0; i < 16; ++i) s += acc[i];
  if (s == 12345.678) out[0] = s;
}
__global__ __launch_bounds__(256) void valu32(float* out, int iters, float a) {
  float acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = fmaf(acc[i], a, 1e-9f);
  float s = 0;
  for (int i = 0; i < 16; ++i) s += acc[i];
  if (s == 12345.678f) out[0] = s;
}
__global__ __launch_bounds__(256) void mfma64(double* out, int iters, double a) {
  f64x4 acc[4];
  for (int i = 0; i < 4; ++i) acc[i] = f64x4{0, 0, 0, (double)i};
  double x = threadIdx.x * 1e-3, y = a;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[i], 0, 0, 0);
  double s = 0;
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[0] = s;
}
int main() {
  double* o;
  hipMalloc(&o, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 8, iters = 4096;
  for (int rep = 0; rep < 2; ++rep) {
    float ms;
    hipEventRecord(e0);
    valu64<<<blocks, 256>>>(o, iters, 0.999);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("valu fp64 fma: %.1f TFLOP/s\n", 2.0 * blocks * 256 * iters * 16 / (ms * 1e9));
    hipEventRecord(e0);
    valu32<<<blocks, 256>>>((float*)o, iters, 0.999f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("valu fp32 fma: %.1f TFLOP/s\n", 2.0 * blocks * 256 * iters * 16 / (ms * 1e9));
    hipEventRecord(e0);
    mfma64<<<blocks, 256>>>(o, iters, 0.999);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("mfma fp64 16x16x4: %.1f TFLOP/s\n", 2.0 * 1024 * (blocks * 4) * iters * 4 / (ms * 1e9));
  }
  return 0;
}
