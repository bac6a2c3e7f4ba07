// sfrt_math.h -- bit-exact binary32 atanf / atan2f / asinf for host and device.
//
// The reference shades every pixel with std::atan2(float, float) and
// std::asinf (/root/reference/Raytracing/SphereWorld.cpp:326 via :373, and
// :374), i.e. the host libm's atan2f / asinf.  The device libm (OCML) uses
// different polynomials, so the kernel cannot call it and stay bit-exact.
// These functions restate the algorithm of glibc 2.35's float versions, which
// are the fdlibm-derived sysdeps/ieee754/flt-32/{s_atanf,e_atan2f,e_asinf}.c
// (no IFUNC variants on x86-64: `nm -D libm.so.6` shows plain W symbols).
// Constants are the exact binary32 values glibc uses (read from its .rodata;
// they equal fdlibm's published ones), and the operation order follows the
// compiled code, so the results are the same on any IEEE-754 binary32 target
// that evaluates without contraction.  tests/test_math_exhaustive.py checks
// them against the host libm over every binary32 input of atanf/asinf and
// ~10^8 atan2f pairs; tests/test_gpu_parity.py repeats that on gfx950.
//
// REQUIREMENTS: compile with -ffp-contract=off, no -ffast-math, and (device)
// correctly rounded fp32 division and sqrt (hipcc's default).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define SFRT_HD __host__ __device__ __forceinline__
#else
#define SFRT_HD static inline
#endif

#pragma clang fp contract(off)

namespace sfrt_math {

SFRT_HD uint32_t f2u(float x) { return __builtin_bit_cast(uint32_t, x); }
SFRT_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }

// s_atanf.c.  Written branch-free: every argument-reduction case keeps its
// own operands, and the one division they need is shared (a/b with the same
// a and b is the same correctly rounded value whichever case produced them),
// so a wave whose lanes fall into different cases pays for one division.
SFRT_HD float atanf(float x) {
  const uint32_t hx = f2u(x);
  const uint32_t ix = hx & 0x7fffffffu;
  const float ax = u2f(ix);  // fabsf
  // id: -1 for |x| < 0.4375, 0..3 for the fdlibm reduction intervals
  const int id = ix < 0x3ee00000u ? -1
               : ix < 0x3f300000u ? 0    // 7/16 <= |x| < 11/16
               : ix < 0x3f980000u ? 1    // 11/16 <= |x| < 19/16
               : ix < 0x401c0000u ? 2    // 19/16 <= |x| < 39/16
               : 3;                      // 39/16 <= |x| < 2^25
  float num = x, den = 1.0f;             // id -1: x / 1 == x exactly
  if (id == 0) { num = (ax + ax) - 1.0f; den = ax + 2.0f; }
  if (id == 1) { num = ax - 1.0f; den = ax + 1.0f; }
  if (id == 2) { num = ax - 1.5f; den = ax * 1.5f + 1.0f; }
  if (id == 3) { num = -1.0f; den = ax; }
  const float xr = num / den;
  const float z = xr * xr;
  const float w = z * z;
  // aT[0,2,..,10] (odd-power terms) and aT[1,3,..,9] (even-power terms)
  float s1 = u2f(0x3c8569d7u) * w + u2f(0x3d4bda59u);   // aT10*w + aT8
  s1 = s1 * w + u2f(0x3d886b35u);                      // aT6
  s1 = s1 * w + u2f(0x3dba2e6eu);                      // aT4
  s1 = s1 * w + u2f(0x3e124925u);                      // aT2
  s1 = s1 * w + u2f(0x3eaaaaabu);                      // aT0
  s1 = s1 * z;
  float s2 = u2f(0xbd15a221u) * w - u2f(0x3d6ef16bu);   // aT9*w + aT7
  s2 = s2 * w - u2f(0x3d9d8795u);                      // aT5
  s2 = s2 * w - u2f(0x3de38e38u);                      // aT3
  s2 = s2 * w - u2f(0x3e4ccccdu);                      // aT1
  s2 = s2 * w;
  const float xs = (s1 + s2) * xr;
  float hi = u2f(0x3fc90fdau), lo = u2f(0x33a22168u);  // atanhi[3], atanlo[3]
  if (id == 0) { hi = u2f(0x3eed6338u); lo = u2f(0x31ac3769u); }
  if (id == 1) { hi = u2f(0x3f490fdau); lo = u2f(0x33222168u); }
  if (id == 2) { hi = u2f(0x3f7b985eu); lo = u2f(0x33140fb4u); }
  float r = hi - ((xs - lo) - xr);
  r = (int32_t)hx < 0 ? -r : r;
  if (id < 0) r = xr - xs;                  // |x| < 0.4375: x - x*(s1+s2)
  if (ix < 0x31000000u) r = x;              // |x| < 2^-29: huge + x > one holds
  if (ix >= 0x4c000000u) {                  // |x| >= 2^25, inf, NaN
    r = (int32_t)hx > 0 ? u2f(0x33a22168u) + u2f(0x3fc90fdau)   // atanlo[3] + atanhi[3]
                        : u2f(0xbfc90fdau) - u2f(0x33a22168u);  // -atanhi[3] - atanlo[3]
    if (ix > 0x7f800000u) r = x + x;        // NaN
  }
  return r;
}

// e_atan2f.c, branch-free over the special cases.  The x == 1 shortcut of
// the source (return atanf(y)) is folded into the general path: atanf is odd
// and y/1 == y, so both give the same bits (checked exhaustively over y).
SFRT_HD float atan2f(float y, float x) {
  const float tiny = u2f(0x0da24260u);    // 1.0e-30
  const float pi_o_4 = u2f(0x3f490fdbu);
  const float pi_o_2 = u2f(0x3fc90fdbu);
  const float pi = u2f(0x40490fdbu);
  const float m_pi_lo = u2f(0x33bbbd2eu); // -pi_lo = 8.7422776573e-08
  const uint32_t hx = f2u(x), hy = f2u(y);
  const uint32_t ix = hx & 0x7fffffffu, iy = hy & 0x7fffffffu;
  const int m = (int)((hy >> 31) | ((hx >> 30) & 2u));     // 2*sign(x) + sign(y)
  const int32_t d = (int32_t)iy - (int32_t)ix;
  const int32_t k = d >> 23;
  float z = sfrt_math::atanf(u2f(f2u(y / x) & 0x7fffffffu));
  if ((int32_t)hx < 0 && k < -60) z = 0.0f;  // |y|/x < -2^60
  if (d > 0x1e7fffff) z = pi_o_2 - u2f(0x333bbd2eu);  // |y/x| > 2^60: pi_o_2 + 0.5*pi_lo
  float r = m == 0 ? z
          : m == 1 ? u2f(f2u(z) ^ 0x80000000u)
          : m == 2 ? pi - (z + m_pi_lo)
          : (z + m_pi_lo) - pi;
  const float pm_pi_o_2 = (int32_t)hy < 0 ? -pi_o_2 - tiny : tiny + pi_o_2;
  if (iy == 0x7f800000u) r = pm_pi_o_2;    // y = +-inf
  if (ix == 0x7f800000u) {                 // x = +-inf
    if (iy == 0x7f800000u) {
      r = m == 0 ? tiny + pi_o_4 : m == 1 ? -pi_o_4 - tiny
        : m == 2 ? 3.0f * pi_o_4 + tiny : -3.0f * pi_o_4 - tiny;
    } else {
      r = m == 0 ? 0.0f : m == 1 ? -0.0f : m == 2 ? tiny + pi : -pi - tiny;
    }
  }
  if (ix == 0) r = pm_pi_o_2;              // x = 0
  if (iy == 0) r = m <= 1 ? y : m == 2 ? tiny + pi : -pi - tiny;  // y = 0
  if (ix > 0x7f800000u || iy > 0x7f800000u) r = x + y;  // NaN
  return r;
}

// q / PI2 + 1.0f and q / PI + 0.5f (SphereWorld.cpp:373-374) without a
// general division: q*(1/b) corrected by one exact residual (fma).  For every
// FINITE binary32 q the final sums equal the reference's bits (exhaustive
// check in tests/native/math_check.cpp; below 2^-104 the quotient itself may
// differ but is absorbed by the + 1.0f / + 0.5f).
SFRT_HD float div_pi2_plus_1(float q) {
  const float b = 6.28318530718f, y = 1.0f / 6.28318530718f;
  const float t = q * y;
  return __builtin_fmaf(__builtin_fmaf(-t, b, q), y, t) + 1.0f;
}
SFRT_HD float div_pi_plus_half(float q) {
  const float b = 3.1415926535f, y = 1.0f / 3.1415926535f;
  const float t = q * y;
  return __builtin_fmaf(__builtin_fmaf(-t, b, q), y, t) + 0.5f;
}

// a / b from y = RN(1/b) (one correctly rounded division per b, reused for
// many a): q = RN(a*y), r = a - b*q (exact with fma), RN(q + r*y) is the
// correctly rounded quotient (Markstein's final correction; checked against
// the hardware's correctly rounded division for 10^10+ pairs per class in
// tests/native/div_check.hip).  Valid for normal b, y and quotients: callers
// take the plain division when b is not in [2^-60, 2^60].
SFRT_HD float div_recip(float a, float b, float y) {
  const float q = a * y;
  const float r = __builtin_fmaf(-b, q, a);
  return __builtin_fmaf(r, y, q);
}

// (t - df*df) / (s + df) of e_asinf.c's |x| in [0.5, 0.975) branch.  There t is in
// (0.0125, 0.25], so the numerator is +0 or a non-zero multiple of 2^-30 and the
// denominator lies in (0.2, 1]: on the device the division runs as the compiler's
// own correctly rounded sequence without its range scaling, which is the identity
// for such operands (sfrt_device.h div_inrange has the argument); same bits as `/`.
SFRT_HD float asinf_tail_div(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float y0 = __builtin_amdgcn_rcpf(b);
  const float y = __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
  float q = a * y;
  q = __builtin_fmaf(__builtin_fmaf(-b, q, a), y, q);
  return __builtin_fmaf(__builtin_fmaf(-b, q, a), y, q);
#else
  return a / b;
#endif
}

// sqrtf(t) for e_asinf.c's t = (1 - |x|) / 2 in [2^-25, 0.25]: on the device the raw
// v_sqrt_f32 corrected by the compiler's own two fma residual tests, without its rescaling
// for arguments below 2^-96 and its special-value selects, which such t never need (the
// same sequence as sfrt_device.h sqrt_cr_normal); `sqrtf` elsewhere.  Same bits.
SFRT_HD float asinf_sqrt(float t) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float r = __builtin_amdgcn_sqrtf(t);
  const float rm = u2f(f2u(r) - 1u), rp = u2f(f2u(r) + 1u);
  float q = __builtin_fmaf(-rm, r, t) <= 0.0f ? rm : r;
  q = __builtin_fmaf(-rp, r, t) > 0.0f ? rp : q;
  return q;
#else
  return __builtin_sqrtf(t);
#endif
}

// e_asinf.c
SFRT_HD float asinf(float x) {
  const float pio2_hi = u2f(0x3fc90fdbu);
  const float pio2_lo = u2f(0xb33bbd2eu);     // -4.3711388287e-08
  const float pio4_hi = u2f(0x3f490fdbu);
  const float p0 = u2f(0x3e2aaae4u), p1 = u2f(0x3d9980f2u), p2 = u2f(0x3d3a3f25u),
              p3 = u2f(0x3cc6141eu), p4 = u2f(0x3d2cb694u);
  const uint32_t hx = f2u(x);
  const uint32_t ix = hx & 0x7fffffffu;
  if (ix == 0x3f800000u) return x * pio2_lo + x * pio2_hi;  // |x| == 1
  if (ix > 0x3f800000u) return (x - x) / (x - x);          // |x| > 1: NaN
  if (ix < 0x3f000000u) {                                 // |x| < 0.5
    if (ix < 0x32000000u) return x;                       // |x| < 2^-27
    const float t = x * x;
    const float w = ((((p4 * t + p3) * t + p2) * t + p1) * t + p0) * t;
    return x + x * w;
  }
  const float w = 1.0f - u2f(ix);
  const float t = w * 0.5f;
  const float p = ((((p4 * t + p3) * t + p2) * t + p1) * t + p0) * t;
  const float s = asinf_sqrt(t);
  float r;
  if (ix >= 0x3f79999au) {                                // |x| > 0.975
    const float q = s * p + s;
    r = pio2_hi - ((q + q) - pio2_lo);
  } else {
    const float df = u2f(f2u(s) & 0xfffff000u);
    const float c = asinf_tail_div(t - df * df, s + df);
    const float pp = (s + s) * p - (pio2_lo - (c + c));
    const float q = pio4_hi - (df + df);
    r = pio4_hi - (pp - q);
  }
  return (int32_t)hx > 0 ? r : -r;
}

// e_acosf.c (glibc's __ieee754_acosf, the `acos` of the GLSL restatement,
// rayShader.frag:142).
SFRT_HD float acosf(float x) {
  const float pi = u2f(0x40490fdau);
  const float pio2_hi = u2f(0x3fc90fdau);
  const float pio2_lo = u2f(0x33a22168u);
  const float pS0 = u2f(0x3e2aaaabu), pS1 = u2f(0xbea6b090u), pS2 = u2f(0x3e4e0aa8u),
              pS3 = u2f(0xbd241146u), pS4 = u2f(0x3a4f7f04u), pS5 = u2f(0x3811ef08u);
  const float qS1 = u2f(0xc019d139u), qS2 = u2f(0x4001572du), qS3 = u2f(0xbf303361u),
              qS4 = u2f(0x3d9dc62eu);
  const uint32_t hx = f2u(x);
  const uint32_t ix = hx & 0x7fffffffu;
  if (ix == 0x3f800000u)                                   // |x| == 1
    return (int32_t)hx > 0 ? 0.0f : pi + u2f(0x34222168u);  // pi + 2*pio2_lo
  if (ix > 0x3f800000u) return (x - x) / (x - x);          // |x| > 1: NaN
  if (ix < 0x3f000000u) {                                  // |x| < 0.5
    if (ix <= 0x32800000u) return pio2_hi + pio2_lo;       // |x| <= 2^-26
    const float z = x * x;
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  }
  if ((int32_t)hx < 0) {                                   // x < -0.5
    const float z = (1.0f + x) * 0.5f;
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float s = __builtin_sqrtf(z);
    const float r = p / q;
    const float w = r * s - pio2_lo;
    return pi - 2.0f * (s + w);
  }
  const float z = (1.0f - x) * 0.5f;                       // x > 0.5
  const float s = __builtin_sqrtf(z);
  const float df = u2f(f2u(s) & 0xfffff000u);
  const float c = (z - df * df) / (s + df);
  const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  const float r = p / q;
  const float w = r * s + c;
  return 2.0f * (df + w);
}

}  // namespace sfrt_math
