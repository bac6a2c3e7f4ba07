// Exhaustive: raw v_sqrt_f32 vs the correctly rounded sqrtf, every non-negative binary32.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
__global__ void k(unsigned long long* lo, unsigned long long* hi) {
  const uint32_t base = (blockIdx.x * 256u + threadIdx.x) * 64u;
  for (uint32_t i = 0; i < 64; i++) {
    const uint32_t u = base + i;
    if (u > 0x7f800000u) return;
    const float x = __uint_as_float(u);
    const float a = __builtin_amdgcn_sqrtf(x);
    const float c = __builtin_sqrtf(x);
    if (__float_as_uint(a) != __float_as_uint(c)) {
      const int e = (int)(u >> 23);
      if (__float_as_uint(a) < __float_as_uint(c)) atomicAdd(&lo[e], 1ull);
      else atomicAdd(&hi[e], 1ull);
    }
  }
}
int main() {
  unsigned long long *lo, *hi;
  hipMalloc(&lo, 256 * 8); hipMalloc(&hi, 256 * 8);
  hipMemset(lo, 0, 256 * 8); hipMemset(hi, 0, 256 * 8);
  const uint32_t n = (0x7f800000u / 64u) / 256u + 1u;
  hipLaunchKernelGGL(k, dim3(n), dim3(256), 0, 0, lo, hi);
  unsigned long long L[256], H[256];
  hipMemcpy(L, lo, sizeof L, hipMemcpyDeviceToHost);
  hipMemcpy(H, hi, sizeof H, hipMemcpyDeviceToHost);
  unsigned long long tl = 0, th = 0;
  for (int e = 0; e < 256; e++) {
    tl += L[e]; th += H[e];
    if (L[e] || H[e]) printf("exp %3d (2^%d): raw below %llu, raw above %llu\n", e, e - 127, L[e], H[e]);
  }
  printf("total below %llu above %llu\n", tl, th);
  return 0;
}
