// gfx950 experiment: VALU issue rate by operand kind.  Eight waves per SIMD, sixteen independent
// two-instruction chains per wave, each variant one inline-asm pair per chain:
//   vv: v_add_f32 v, v, v      sv: v_add_f32 v, s, v (VOP2, SGPR src0)    iv: v_add_f32 v, 1.0, v
//   lv: v_add_f32 v, literal, v   sv3: v_add_f32_e64 v, s, v (VOP3)      fma_vvs: v_fma_f32 v, v, v, s
//   mix: per chain one v_sub_f32 v, s, v then one v_mul_f32 v, v, v (the march's distance-test mix)
//   vmov: v_mov_b32 v, s once per chain then v_add_f32 v, v, v twice
//   cmp_s: v_cmp_gt_f32 vcc, s, v then v_add_f32 v, v, v
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define BODY(ASM, CONS) \
  _Pragma("unroll") for (int i = 0; i < 16; i++) { float v = x[i]; __asm__ volatile(ASM : "+v"(v) : CONS); x[i] = v; }

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, unsigned long long* clk, int iters, float a) {
  float x[16];
  float av = a + (float)threadIdx.x * 0.0f;
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = (float)(threadIdx.x + i);
  const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; it++) {
    if (MODE == 0) { BODY("v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0", "v"(av)) }
    if (MODE == 1) { BODY("v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0", "s"(a)) }
    if (MODE == 2) { BODY("v_add_f32 %0, 1.0, %0\n v_add_f32 %0, 1.0, %0", "v"(av)) }
    if (MODE == 3) { BODY("v_add_f32 %0, 0x3f8ccccd, %0\n v_add_f32 %0, 0x3f8ccccd, %0", "v"(av)) }
    if (MODE == 4) { BODY("v_add_f32_e64 %0, %1, %0\n v_add_f32_e64 %0, %1, %0", "s"(a)) }
    if (MODE == 5) { BODY("v_fma_f32 %0, %0, %0, %1\n v_fma_f32 %0, %0, %0, %1", "s"(a)) }
    if (MODE == 6) { BODY("v_fma_f32 %0, %0, %0, %1\n v_fma_f32 %0, %0, %0, %1", "v"(av)) }
    if (MODE == 7) { BODY("v_sub_f32 %0, %1, %0\n v_mul_f32 %0, %0, %0", "s"(a)) }
    if (MODE == 8) { BODY("v_sub_f32 %0, %1, %0\n v_mul_f32 %0, %0, %0", "v"(av)) }
    if (MODE == 9) {
      float t;
      __asm__ volatile("v_mov_b32 %0, %1" : "=v"(t) : "s"(a));
      BODY("v_add_f32 %0, %1, %0\n v_add_f32 %0, %1, %0", "v"(t))
    }
    if (MODE == 10) { BODY("v_cmp_gt_f32 vcc, %1, %0\n v_add_f32 %0, %0, %0", "s"(a)) }
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = c1 - c0; clk[1] = r1 - r0; }
}

typedef void (*kfn)(float*, unsigned long long*, int, float);

int main() {
  float* out;
  unsigned long long* clk;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 8;
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipMalloc(&clk, 16);
  const kfn fns[] = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>, k<9>, k<10>};
  const char* names[] = {"vv", "sv", "iv", "lv", "sv3", "fma_vvs", "fma_vvv", "mix_sub_s_mul", "mix_sub_v_mul",
                         "vmov_then_vv", "cmp_s"};
  const int per_iter[] = {32, 32, 32, 32, 32, 32, 32, 32, 32, 33, 32};
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 20000;
  for (int rep = 0; rep < 2; rep++)
    for (int m = 0; m < 11; m++) {
      hipLaunchKernelGGL(fns[m], dim3(blocks), dim3(256), 0, 0, out, clk, 200, 1.0001f);
      hipEventRecord(e0);
      hipLaunchKernelGGL(fns[m], dim3(blocks), dim3(256), 0, 0, out, clk, iters, 1.0001f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c[2];
      hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
      const double ghz = (double)c[0] / ((double)c[1] * 10.0);
      const double rate = (double)blocks * 4 * iters * per_iter[m] / (ms * 1e-3);
      printf("%-16s %7.3f ms  %.3f T wave64-VALU/s  clock %.2f GHz  %.3f per SIMD-clock\n", names[m], ms,
             rate / 1e12, ghz, rate / (cus * 4.0 * ghz * 1e9));
    }
  return 0;
}
