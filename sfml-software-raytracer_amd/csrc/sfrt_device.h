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

// atan2f(y, x), bit for bit sfrt_math::atan2f (= glibc's e_atan2f.c), with a
// cheaper path for the waves the renderers produce.  When every lane of the
// wave has finite non-zero x and y and |y/x| in [2^-29, 2^25), no special case
// of e_atan2f.c / s_atanf.c can fire: the |y|/x < -2^60 and |y/x| > 2^60
// overrides need an exponent gap above 60, the tiny and huge atanf branches an
// argument outside that range.  Then atanf runs on the positive |y/x| (no sign
// handling), and when all lanes also share the argument-reduction interval,
// only that interval's code runs (a uniform branch; one division, none for
// |y/x| < 7/16).  The quadrant fix-up uses (z + pi_lo) - pi == -(pi - (z + pi_lo))
// (round-to-nearest is symmetric).  Any other wave takes sfrt_math::atan2f.
__device__ __forceinline__ float atan2f_wave(float y, float x) {
  using sfrt_math::f2u;
  using sfrt_math::u2f;
  const uint32_t hx = f2u(x), hy = f2u(y);
  const uint32_t ix = hx & 0x7fffffffu, iy = hy & 0x7fffffffu;
  const float q = y / x;
  const uint32_t iq = f2u(q) & 0x7fffffffu;
  const bool general = (ix - 1u < 0x7f7fffffu) & (iy - 1u < 0x7f7fffffu) &
                       (iq - 0x31000000u < 0x4c000000u - 0x31000000u);
  if (__builtin_amdgcn_ballot_w64(!general)) return sfrt_math::atan2f(y, x);
  const float a = u2f(iq);
  const int id = iq < 0x3ee00000u ? -1
               : iq < 0x3f300000u ? 0
               : iq < 0x3f980000u ? 1
               : iq < 0x401c0000u ? 2
               : 3;
  // s_atanf.c tail for the reduced argument xr: (s1 + s2) * xr and the final sum
  auto poly = [](float xr) {
    const float z = xr * xr;
    const float w = z * z;
    float s1 = u2f(0x3c8569d7u) * w + u2f(0x3d4bda59u);
    s1 = s1 * w + u2f(0x3d886b35u);
    s1 = s1 * w + u2f(0x3dba2e6eu);
    s1 = s1 * w + u2f(0x3e124925u);
    s1 = s1 * w + u2f(0x3eaaaaabu);
    s1 = s1 * z;
    float s2 = u2f(0xbd15a221u) * w - u2f(0x3d6ef16bu);
    s2 = s2 * w - u2f(0x3d9d8795u);
    s2 = s2 * w - u2f(0x3de38e38u);
    s2 = s2 * w - u2f(0x3e4ccccdu);
    s2 = s2 * w;
    return (s1 + s2) * xr;
  };
  float zr;
  const int id0 = __builtin_amdgcn_readfirstlane(id);
  if (__builtin_amdgcn_ballot_w64(id != id0) == 0) {
    // one reduction interval for the whole wave (uniform branch)
    if (id0 < 0) {
      zr = a - poly(a);
    } else {
      float xr, hi, lo;
      if (id0 == 0) {
        xr = ((a + a) - 1.0f) / (a + 2.0f);
        hi = u2f(0x3eed6338u); lo = u2f(0x31ac3769u);
      } else if (id0 == 1) {
        xr = (a - 1.0f) / (a + 1.0f);
        hi = u2f(0x3f490fdau); lo = u2f(0x33222168u);
      } else if (id0 == 2) {
        xr = (a - 1.5f) / (a * 1.5f + 1.0f);
        hi = u2f(0x3f7b985eu); lo = u2f(0x33140fb4u);
      } else {
        xr = -1.0f / a;
        hi = u2f(0x3fc90fdau); lo = u2f(0x33a22168u);
      }
      zr = hi - ((poly(xr) - lo) - xr);
    }
  } else {
    float num = a, den = 1.0f;
    if (id == 0) { num = (a + a) - 1.0f; den = a + 2.0f; }
    if (id == 1) { num = a - 1.0f; den = a + 1.0f; }
    if (id == 2) { num = a - 1.5f; den = a * 1.5f + 1.0f; }
    if (id == 3) { num = -1.0f; den = a; }
    const float xr = num / den;
    const float xs = poly(xr);
    float hi = u2f(0x3fc90fdau), lo = u2f(0x33a22168u);
    if (id == 0) { hi = u2f(0x3eed6338u); lo = u2f(0x31ac3769u); }
    if (id == 1) { hi = u2f(0x3f490fdau); lo = u2f(0x33222168u); }
    if (id == 2) { hi = u2f(0x3f7b985eu); lo = u2f(0x33140fb4u); }
    zr = id < 0 ? xr - xs : hi - ((xs - lo) - xr);
  }
  // e_atan2f.c quadrants: m = 0: z, 1: -z, 2: pi - (z + pi_lo), 3: (z + pi_lo) - pi
  const float r = (int32_t)hx < 0 ? u2f(0x40490fdbu) - (zr + u2f(0x33bbbd2eu)) : zr;
  return u2f(f2u(r) ^ (hy & 0x80000000u));
}

constexpr float kTinySqrtArg = 0x1.0p-96f;

// Correctly rounded sqrtf for any x: the short form unless some lane of the
// wave has a tiny argument (then the compiler's full lowering for all lanes).
__device__ __forceinline__ float sqrt_cr(float x) {
  if (__builtin_amdgcn_ballot_w64(x < kTinySqrtArg)) return __builtin_sqrtf(x);
  return sqrt_cr_normal(x);
}

}  // namespace sfrt
