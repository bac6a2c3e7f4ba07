// gfx950 experiment: does one-wave-workgroup dispatch keep 8 waves per SIMD busy?
// 32400 workgroups of 64 threads (the 4K frame's tile grid) each hold their slot for D us
// (s_memrealtime spin, no VALU), with a 2.2 KB kernel-argument block like k_trace_window_r<4>.
// Ideal time = ceil(32400 / slots) * D; prints measured vs ideal for several D and occupancies.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

struct Big { uint32_t w[560]; };  // 2240 B of kernel arguments

template <int W>
__global__ __launch_bounds__(64, W) void k_spin(Big b, uint32_t ticks, uint32_t* out) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0 && b.w[blockIdx.x % 560] == 12345u) out[0] = 1;  // keep b live
}

int main() {
  Big b = {};
  uint32_t* out;
  hipMalloc(&out, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = 32400;
  for (int rep = 0; rep < 2; rep++)
    for (double us : {5.0, 14.0, 28.0}) {
      const uint32_t ticks = (uint32_t)(us * 100.0);  // s_memrealtime runs at 100 MHz
      for (int w : {8, 4}) {
        // warm-up launch, then timed
        for (int it = 0; it < 2; it++) {
          hipEventRecord(e0);
          if (w == 8) hipLaunchKernelGGL(k_spin<8>, dim3(grid), dim3(64), 0, 0, b, ticks, out);
          else hipLaunchKernelGGL(k_spin<4>, dim3(grid), dim3(64), 0, 0, b, ticks, out);
          hipEventRecord(e1);
          hipEventSynchronize(e1);
        }
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double slots = (double)cus * 4 * 8;  // 8 waves per SIMD (launch_bounds W limits VGPRs only)
        const double ideal = (double)((grid + (long)slots - 1) / (long)slots) * us;
        printf("D %5.1f us, launch_bounds %d: %8.1f us  (ideal at %d slots: %.1f us; ratio %.3f)\n", us, w,
               ms * 1000.0, (int)slots, ideal, ms * 1000.0 / (grid * us / slots));
      }
    }
  return 0;
}
