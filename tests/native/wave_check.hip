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

// The march's pass body takes sqrt_cr_normal for every passing lane, also when
// the squared distance is below 2^-96 where sqrt_cr_normal is not the correctly
// rounded sqrt.  A pass needs rad - sqrtf(ss) > 0.01f, so rad > 0.01f; then
// rad - q == rad for any q < 2^-33, which both square roots of such ss are.
// Checked here for every binary32 ss in [0, 2^-96) and radii from 0.01f up.
__global__ void k_sqrt_tiny(unsigned long long* bad) {
  const float rads[] = {0.01f, 0.0100001f, 0.015625f, 0.0156250019f, 0.5f, 1.0f, 2.0f,
                        3.99999976f, 4.0f, 7.0f, 1.0e6f, 3.0e38f};
  unsigned long long nbad = 0;
  for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < 0x0F800000u;
       u += gridDim.x * blockDim.x) {
    const float x = __uint_as_float(u);
    const float q = sfrt::sqrt_cr_normal(x), ref = __builtin_sqrtf(x);
    if (!(q < 0x1.0p-40f)) nbad++;
    for (float rad : rads)
      if (__float_as_uint(rad - q) != __float_as_uint(rad - ref)) nbad++;
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
  hipLaunchKernelGGL(k_sqrt_tiny, dim3(8192), dim3(256), 0, 0, d_bad);
  unsigned long long bad_all = 0;
  if (hipMemcpy(&bad_all, d_bad, sizeof(bad_all), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  std::printf("sqrt_tiny: %llu mismatches over [0, 2^-96)\n", bad_all - bad);
  bad = bad_all;
  std::printf("waves=%d mismatches=%llu\n", 4096 * 4 * 64, bad);
  (void)hipFree(d_bad);
  return bad ? 1 : 0;
}
