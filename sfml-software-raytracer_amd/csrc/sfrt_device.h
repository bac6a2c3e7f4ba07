// sfrt_device.h -- gfx950 device helpers shared by the trace kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "sfrt_math.h"

#pragma clang fp contract(off)

namespace sfrt {

// A 64-bit value made wave-uniform (SGPR pair) from lane 0's copy.  The
// builtin returns int: each half goes through uint32_t so the low word is
// zero-extended, not sign-extended into the high word.
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Wave-wide min / max of unsigned words, all in DPP: the row reduction
// (quad_perm, half-mirror, mirror; each step one v_min_u32_dpp), then
// row_bcast:15 into rows 1 and 3 and row_bcast:31 into rows 2 and 3, so lane
// 63 holds the wave's result.  For binary32 values >= +0 (no NaN) the bit
// patterns order like the values, so these also reduce non-negative floats
// with no canonicalising VALU ops.  Call with the whole wave active (DPP
// reads inactive lanes' stale values).
// IDENTITY (the op's neutral value) fills lanes whose row is masked off, so
// the compiler folds each mov_dpp into the min / max itself.
template <int CTRL, int ROW_MASK, uint32_t IDENTITY>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)IDENTITY, (int)x, CTRL, ROW_MASK, 0xf, false);
}

template <bool MAX>
__device__ __forceinline__ uint32_t wave_reduce_u32(uint32_t v) {
  constexpr uint32_t I = MAX ? 0u : 0xffffffffu;
  auto op = [](uint32_t a, uint32_t b) {
    return MAX ? __builtin_elementwise_max(a, b) : __builtin_elementwise_min(a, b);
  };
  v = op(v, dpp_u32<0xB1, 0xf, I>(v));   // quad_perm [1,0,3,2]
  v = op(v, dpp_u32<0x4E, 0xf, I>(v));   // quad_perm [2,3,0,1]
  v = op(v, dpp_u32<0x141, 0xf, I>(v));  // row_half_mirror
  v = op(v, dpp_u32<0x140, 0xf, I>(v));  // row_mirror
  v = op(v, dpp_u32<0x142, 0xa, I>(v));  // row_bcast:15 -> rows 1, 3
  v = op(v, dpp_u32<0x143, 0xc, I>(v));  // row_bcast:31 -> rows 2, 3
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) { return wave_reduce_u32<false>(v); }
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) { return wave_reduce_u32<true>(v); }

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
