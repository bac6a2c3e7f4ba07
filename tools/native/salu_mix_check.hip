// gfx950 experiment: do scalar instructions take vector issue slots?  Eight waves per SIMD run a
// stream of independent v_add_f32 with 0, 8, 16 or 32 s_movk_i32 (independent, SCC untouched) per 32
// v_add_f32; if SALU issues beside VALU the VALU rate stays, if they share issue it drops.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <int NS>
__global__ __launch_bounds__(256) void k(float* out, int iters, float a) {
  float x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = (float)(threadIdx.x + i);
  uint32_t s0 = blockIdx.x, s1 = blockIdx.x + 1, s2 = 3, s3 = 4;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 16; i++) {
      float v = x[i];
      __asm__ volatile("v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0" : "+v"(v) : "v"(a));
      x[i] = v;
      if (NS >= 8 && (i & 1) == 0) __asm__ volatile("s_movk_i32 %0, 0x11" : "=s"(s0));
      if (NS >= 16 && (i & 1) == 1) __asm__ volatile("s_movk_i32 %0, 0x22" : "=s"(s1));
      if (NS >= 32) __asm__ volatile("s_movk_i32 %0, 0x33" : "=s"(s2));
      if (NS >= 32) __asm__ volatile("s_movk_i32 %0, 0x44" : "=s"(s3));
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s + (float)(s0 + s1 + s2 + s3);
}

int main() {
  float* out;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 8;
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 20000;
  for (int rep = 0; rep < 3; rep++)
    for (int ns : {0, 8, 16, 32}) {
      hipEventRecord(e0);
      if (ns == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f);
      if (ns == 8) hipLaunchKernelGGL(k<8>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f);
      if (ns == 16) hipLaunchKernelGGL(k<16>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f);
      if (ns == 32) hipLaunchKernelGGL(k<32>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double valu = (double)blocks * 4 * iters * 32;
      printf("%2d s_movk per 32 v_add: %.3f ms, %.3f T wave64 VALU/s\n", ns, ms, valu / ms / 1e9);
    }
  return 0;
}
