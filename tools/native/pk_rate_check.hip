// gfx950 experiment: the VALU issue rate a simple f32 stream reaches on the whole chip, and the
// shader clock while it runs (s_memtime against the 100 MHz s_memrealtime).  Eight waves per SIMD
// (the sphere kernel's occupancy), sixteen independent chains per wave:
//   mode 0: v_add_f32 + v_mul_f32 per chain; mode 1: the same element ops as v_pk_add_f32 +
//   v_pk_mul_f32 on pairs; mode 2: v_add_f32 only; mode 3: v_add_f32 with an SGPR operand (one
//   VGPR read per instruction instead of two).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float float2_t __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, unsigned long long* clk, int iters, float a) {
  float x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = (float)(threadIdx.x + i);
  const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; it++) {
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 16; i++) {
        float v = x[i];
        __asm__ volatile("v_add_f32 %0, %1, %0\n v_mul_f32 %0, %1, %0" : "+v"(v) : "v"(a));
        x[i] = v;
      }
    } else if (MODE == 1) {
      const float2_t a2 = {a, a};
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        float2_t v = {x[i], x[i + 1]};
        __asm__ volatile("v_pk_add_f32 %0, %1, %0\n v_pk_mul_f32 %0, %1, %0" : "+v"(v) : "v"(a2));
        x[i] = v.x; x[i + 1] = v.y;
      }
    } else if (MODE == 2) {
#pragma unroll
      for (int i = 0; i < 16; i++) {
        float v = x[i];
        __asm__ volatile("v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0" : "+v"(v) : "v"(a));
        x[i] = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; i++) {
        float v = x[i];
        __asm__ volatile("v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0" : "+v"(v) : "s"(a));
        x[i] = v;
      }
    }
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = c1 - c0; clk[1] = r1 - r0; }
}

int main() {
  float* out;
  unsigned long long* clk;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 8;  // 8 waves per SIMD: 4 waves per block, 8 blocks per CU
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipMalloc(&clk, 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 20000;
  for (int rep = 0; rep < 3; rep++)
    for (int mode = 0; mode < 4; mode++) {
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 1.0001f);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 1.0001f);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 1.0001f);
      if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 1.0001f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c[2];
      hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
      const double ghz = (double)c[0] / ((double)c[1] * 10.0);  // memrealtime: 100 MHz
      const double elem_ops = (double)blocks * 256 * iters * 32;
      const double waveinsts = (double)blocks * 4 * iters * (mode == 1 ? 16 : 32);
      const double rate = waveinsts / ms / 1e9;
      printf("%-26s %.3f ms, %.1f T element-ops/s, %.3f T wave64-insts/s, s_memtime clock %.2f GHz,"
             " %.3f wave64-insts per SIMD-clock\n",
             mode == 0 ? "v_add + v_mul" : mode == 1 ? "v_pk_add + v_pk_mul"
             : mode == 2 ? "v_add + v_add" : "v_add + v_add, SGPR operand", ms,
             elem_ops / ms / 1e9, rate, ghz, rate * 1e12 / (cus * 4.0 * ghz * 1e9));
    }
  return 0;
}
