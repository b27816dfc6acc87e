// Measurement tooling: which hardware CUs a launch on a CU-masked stream lands on.
// Each block spins ~spin_ns so that the dispatcher spreads the grid over every CU the
// stream may use, then lane 0 stores its XCC_ID and HW_ID registers (vector stores).
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/cu_mask_probe.hip -o tools/cu_mask_probe.so
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ __launch_bounds__(64) void cu_probe_kernel(unsigned* out, long long spin_cycles) {
  const long long t0 = wall_clock64();
  // wall_clock64 runs at 100 MHz: bounded spin, every wave exits
  while (wall_clock64() - t0 < spin_cycles) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0) {
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
}

extern "C" int cu_probe_launch(void* stream, int nblk, unsigned* out, long long spin_cycles) {
  if (nblk < 1 || nblk > (1 << 20) || spin_cycles < 0 || spin_cycles > 100000000LL) return 1;
  hipLaunchKernelGGL(cu_probe_kernel, dim3(nblk), dim3(64), 0, (hipStream_t)stream, out, spin_cycles);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// A stream limited to the CUs whose bits are set in mask[0..words).
extern "C" int cu_stream_create(const unsigned* mask, int words, void** stream) {
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask) != hipSuccess) return 1;
  *stream = s;
  return 0;
}

extern "C" int cu_stream_mask(void* stream, int words, unsigned* mask) {
  return hipExtStreamGetCUMask((hipStream_t)stream, (uint32_t)words, mask) == hipSuccess ? 0 : 1;
}

extern "C" int cu_stream_destroy(void* stream) {
  return hipStreamDestroy((hipStream_t)stream) == hipSuccess ? 0 : 1;
}
