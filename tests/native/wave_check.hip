// gfx950 check of the wave-wide helpers in sfrt_device.h against a plain
// lane loop: wave_min_u32 / wave_max_u32 (DPP row reduction + readlane) and
// uniform_u64 (lane 0's 64-bit value, no sign extension), for many random
// full waves (the kernels call them in wave-uniform control flow only).
// Built and run by tests/test_gpu_parity.py::test_wave_helpers:
//   hipcc --offload-arch=gfx950 -O3 wave_check.hip -o wave_check && ./wave_check
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../../sfml-software-raytracer_amd/csrc/sfrt_device.h"

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__global__ void k_check(int rounds, unsigned long long* bad) {
  __shared__ uint32_t vals[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned long long nbad = 0;
  for (int r = 0; r < rounds; r++) {
    const uint64_t seed = ((uint64_t)blockIdx.x * 4 + wave) * 1000003ull + (uint64_t)r;
    const uint64_t z = mix(seed * 64 + (uint64_t)lane);
    // small ranges make ties and equal lanes common; float-like patterns too
    uint32_t v = (r & 3) == 0 ? (uint32_t)(z & 15) : (r & 3) == 1 ? (uint32_t)z
                 : (uint32_t)(z & 0x7f7fffffu);
    vals[wave][lane] = v;
    __builtin_amdgcn_wave_barrier();
    uint32_t lo = 0xffffffffu, hi = 0u;
    for (int l = 0; l < 64; l++) {
      lo = vals[wave][l] < lo ? vals[wave][l] : lo;
      hi = vals[wave][l] > hi ? vals[wave][l] : hi;
    }
    if (sfrt::wave_min_u32(v) != lo) nbad++;
    if (sfrt::wave_max_u32(v) != hi) nbad++;
    // 64-bit uniform from lane 0, with bit 31 set in half the rounds
    const uint64_t m = mix(seed) | ((uint64_t)(r & 1) << 31);
    const uint64_t mine = lane == 0 ? m : mix(seed + 1 + (uint64_t)lane);
    if (sfrt::uniform_u64(mine) != m) nbad++;
    __builtin_amdgcn_wave_barrier();
  }
  if (nbad) atomicAdd(bad, nbad);
}

int main() {
  unsigned long long* d_bad = nullptr;
  if (hipMalloc(&d_bad, sizeof(*d_bad)) != hipSuccess) return 2;
  if (hipMemset(d_bad, 0, sizeof(*d_bad)) != hipSuccess) return 2;
  hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, 0, 64, d_bad);
  unsigned long long bad = 0;
  if (hipMemcpy(&bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  std::printf("waves=%d mismatches=%llu\n", 4096 * 4 * 64, bad);
  (void)hipFree(d_bad);
  return bad ? 1 : 0;
}
