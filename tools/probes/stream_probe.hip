// Read-bandwidth probe: 256 MiB streamed by W waves per CU, each wave reading a
// contiguous run with R wave-wide 16-B loads in flight.  Tells the sweep kernel
// how many waves / bytes in flight the HBM stream needs.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int R>
__global__ __launch_bounds__(1024) void stream(const f32x4* __restrict__ a, long per_wave, float* out) {
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const f32x4* p = a + wave * per_wave + lane;
  f32x4 acc = {0, 0, 0, 0};
  f32x4 r[R];
#pragma unroll
  for (int i = 0; i < R; ++i) r[i] = p[i * 64];
  long n = per_wave / 64;
  for (long i = R; i < n; i += R) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      acc += r[j];
      r[j] = p[(i + j < n ? i + j : n - 1) * 64];
    }
  }
#pragma unroll
  for (int j = 0; j < R; ++j) acc += r[j];
  if (acc[0] == 12345.f) out[0] = acc[1];
}

int main() {
  f32x4* a;
  float* o;
  (void)hipMalloc(&a, 1l << 30);
  for (long bytes : {268435456l, 1l << 30}) {
  printf("buffer %ld MB\n", bytes >> 20);
  (void)hipMalloc(&o, 4);
  (void)hipMemset(a, 0, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int cus = 256;
  for (int wpc : {4, 8, 16}) {
    for (int R : {4, 8, 16, 24}) {
      const long waves = (long)cus * wpc;
      const long per_wave = bytes / 16 / waves;
      const int thr = 64 * wpc;
      auto run = [&]() {
        switch (R) {
          case 4: hipLaunchKernelGGL(stream<4>, dim3(cus), dim3(thr), 0, 0, a, per_wave, o); break;
          case 8: hipLaunchKernelGGL(stream<8>, dim3(cus), dim3(thr), 0, 0, a, per_wave, o); break;
          case 16: hipLaunchKernelGGL(stream<16>, dim3(cus), dim3(thr), 0, 0, a, per_wave, o); break;
          default: hipLaunchKernelGGL(stream<24>, dim3(cus), dim3(thr), 0, 0, a, per_wave, o); break;
        }
      };
      run();
      hipEventRecord(e0);
      for (int i = 0; i < 20; ++i) run();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / 20;
      printf("waves/CU=%2d loads in flight/wave=%2d (%3ld KiB/CU): %7.1f us  %6.2f TB/s\n", wpc, R,
             (long)wpc * R, us, bytes / us / 1e6);
    }
  }
  }
  return 0;
}
