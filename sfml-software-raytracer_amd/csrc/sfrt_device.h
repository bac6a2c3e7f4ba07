// sfrt_device.h -- gfx950 device helpers shared by the trace kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "sfrt_math.h"

#pragma clang fp contract(off)

namespace sfrt {

// Wave-wide minimum through DPP row ops (no LDS): min within each 16-lane
// row, then the four row results via readlane.  Uniform result.
template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
      __builtin_bit_cast(int, x), __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}

// A 64-bit value made wave-uniform (SGPR pair) from lane 0's copy.  The
// builtin returns int: each half goes through uint32_t so the low word is
// zero-extended, not sign-extended into the high word.
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ __forceinline__ float wave_min(float v) {
  v = fminf(v, dpp<0xB1>(v));   // quad_perm [1,0,3,2]
  v = fminf(v, dpp<0x4E>(v));   // quad_perm [2,3,0,1]
  v = fminf(v, dpp<0x141>(v));  // row_half_mirror
  v = fminf(v, dpp<0x140>(v));  // row_mirror
  const int b = __builtin_bit_cast(int, v);
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48));
  return fminf(fminf(r0, r1), fminf(r2, r3));
}

// sqrtf(x) correctly rounded for x >= 2^-96 (not denormal/tiny): the raw
// v_sqrt_f32 (within 1 ulp) corrected by the two fma residual tests that the
// compiler's own correctly rounded lowering uses -- minus its tiny-input
// rescaling and special-value selects, which these inputs never need.
__device__ __forceinline__ float sqrt_cr_normal(float x) {
  const float r = __builtin_amdgcn_sqrtf(x);
  const float rm = sfrt_math::u2f(sfrt_math::f2u(r) - 1u);
  const float rp = sfrt_math::u2f(sfrt_math::f2u(r) + 1u);
  float q = __builtin_fmaf(-rm, r, x) <= 0.0f ? rm : r;
  q = __builtin_fmaf(-rp, r, x) > 0.0f ? rp : q;
  return q;
}

constexpr float kTinySqrtArg = 0x1.0p-96f;

// Correctly rounded sqrtf for any x: the short form unless some lane of the
// wave has a tiny argument (then the compiler's full lowering for all lanes).
__device__ __forceinline__ float sqrt_cr(float x) {
  if (__builtin_amdgcn_ballot_w64(x < kTinySqrtArg)) return __builtin_sqrtf(x);
  return sqrt_cr_normal(x);
}

}  // namespace sfrt
