// sphere_trace.hip -- gfx950 kernels for the sphere-cave trace-and-shade path.
//
// Replaces the per-pixel body of SphereWorld::UpdateImage / Raycast
// (/root/reference/Raytracing/SphereWorld.cpp:83-112, 355-382): one wave64 per
// (8R)x8 pixel tile, R = 1..4 pixels per lane (records in the kernel arguments for
// n <= 64 spheres, a per-wave culled list above that), RGBA8 written straight to HBM.
//
// Bit-exactness rules (see DESIGN.md "Exactness"):
//  * built with -ffp-contract=off; every float expression keeps the
//    reference's operand order; division and sqrt are the correctly rounded
//    gfx950 sequences (hipcc default), or the same sequences without their
//    range scaling where the operands provably need none (div_inrange,
//    sqrt_cr_normal: sfrt_device.h);
//  * atan2f / asinf are sfrt_math:: restatements of the host libm;
//  * the sphere test `r - sqrtf(s) > 0.01f` is replaced by `s < s_pass`, where
//    s_pass is the exact binary32 threshold found on the host (the test is
//    monotone in s), so sqrtf runs only for spheres that pass;
//  * a sphere is skipped for a whole wave only when it provably cannot pass
//    for any ray of the tile (cone test with margins, below); the surviving
//    spheres are visited in their original order, so "last passing index"
//    (drawSphere, :368) and the max (:367) are unchanged.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "sfrt_device.h"
#include "sfrt_math.h"
#include "sfrt_probe.h"
#include "sfrt_trace.h"

#pragma clang fp contract(off)

// Diagnostic builds (-DSFRT_EXP=<bits>: timing and counter probes that write wrong bytes) go
// through the probe type P of trace_tile_window_r (sfrt_probe.h); the shipped library's
// NoProbe hooks are empty.
#ifndef SFRT_BUILD_FLAVOUR
#define SFRT_BUILD_FLAVOUR "release"
#endif

namespace sfrt {
namespace {

constexpr float kPI = 3.1415926535f;     // SphereWorld.h:6
constexpr float kPI2 = 6.28318530718f;   // SphereWorld.h:7

// Primary direction of pixel (i, j), normalised (SphereWorld.cpp:95-106, :358).
__device__ __forceinline__ void primary_dir(const FrameRec& f, int i, int j, float& dx,
                                            float& dy, float& dz) {
  const float h = f.h_start + f.h_inc * (float)i;
  const float v = f.v_start + (float)j * f.v_inc;
  float x = (f.fwd[0] + f.right[0] * h) + f.up[0] * v;
  float y = (f.fwd[1] + f.right[1] * h) + f.up[1] * v;
  float z = (f.fwd[2] + f.right[2] * h) + f.up[2] * v;
  // |(x,y,z)|^2 >= 1 - tiny: forward is a unit vector orthogonal to right and up
  const float len = sqrt_cr_normal((x * x + y * y) + z * z);
  // components in [2^-40, 2^40) put len there too: one shared reciprocal seed
  // (div_inrange, the same bits as `/`); a wave with a zero component takes `/`
  if ((ballot_bad_operand(x) | ballot_bad_operand(y) | ballot_bad_operand(z)) == 0) {
    const float s = div_seed(len);
    dx = div_inrange(x, len, s);
    dy = div_inrange(y, len, s);
    dz = div_inrange(z, len, s);
  } else {
    const float l = keep_branch(len);
    dx = x / l;
    dy = y / l;
    dz = z / l;
  }
}

// Shading tail, SphereWorld.cpp:373-381, in two parts so that a lane's R pixels
// can issue their texel loads together: shade_texel computes the texel index --
// `tex` indexes f.tex (the sphere's first texel when the index falls outside the
// texture: the reference would read outside the image there; `outside` reports
// it) -- and the brightness; shade_rgba applies the brightness (RGBA8 packed, r
// in byte 0).
struct Shading {
  uint32_t tex;
  float brightness;
  bool outside;
};

template <class P>
__device__ __forceinline__ Shading shade_texel(const FrameRec& f, const SphereRec& d, float px,
                                               float py, float pz, PixelDump* dump) {
  float ang = d.atan_c - P::hit_atan2(pz, px);  // atan2f_wave == sfrt_math::atan2f (sfrt_device.h)
  ang = ang > kPI ? ang - kPI2 : (ang < -kPI ? ang + kPI2 : ang);
  const float xcoord = sfrt_math::div_pi2_plus_1(ang);  // == ang / PI2 + 1.0f
  const float ex = px - d.cx, ey = py - d.cy, ez = pz - d.cz;
  const float el = sqrt_cr((ex * ex + ey * ey) + ez * ez);
  const float bx = px - f.cam[0], by = py - f.cam[1], bz = pz - f.cam[2];
  const float bl = sqrt_cr((bx * bx + by * by) + bz * bz);
  const float bd = bl < 3.0f ? 3.0f : bl;
  // ey / el and 3 / bd through div_inrange (same bits) unless some lane's operands
  // leave [2^-40, 2^40) (bd >= 3 needs only the upper bound)
  float ny, brightness;
  if ((ballot_bad_operand(ey) | ballot_bad_operand(el) | __builtin_amdgcn_ballot_w64(!(bd < 0x1.0p40f))) == 0) {
    ny = div_inrange(ey, el);
    brightness = div_inrange(3.0f, bd);
  } else {
    ny = ey / keep_branch(el);
    brightness = 3.0f / keep_branch(bd);
  }
  const float ycoord = sfrt_math::div_pi_plus_half(P::hit_asin(ny));  // == asinf / PI + 0.5f
  // fmodf(v, 1.0f) == v - truncf(v) exactly for every binary32 v (NaN/inf -> NaN).
  // texsize of textures[0] (or of the sphere's extension slot), (float)(unsigned) as :376
  const uint32_t tw = d.tex_wh & 0xffffu, th = d.tex_wh >> 16;
  float u = xcoord * 4.0f * d.r;
  u = (u - __builtin_truncf(u)) * (float)tw;
  float w = ycoord * 2.0f * d.r;
  w = (w - __builtin_truncf(w)) * (float)th;
  // float -> unsigned: v_cvt_u32_f32 (NaN -> 0), as x86's cvttss2si for [0, 2^31).
  const uint32_t tx = __float2uint_rz(u), ty = __float2uint_rz(w);
  // ty < th <= 0xffff (a fraction in [0, 1) times th, or 0 from NaN; radii are > 0, so no
  // negative fraction reaches -1 / th): the 24-bit multiply is the exact product
  const uint32_t idx = tx + __umul24(ty, tw);
  Shading sh;
  sh.outside = !(idx < tw * th);
  sh.tex = d.tex_off + (sh.outside ? 0u : idx);
  sh.brightness = brightness;
  if (dump) {
    dump->xcoord = xcoord;
    dump->ycoord = ycoord;
    dump->brightness = brightness;
    dump->texel[0] = tx;
    dump->texel[1] = ty;
  }
  return sh;
}

// (Uint8)(component * brightness) for r, g, b; alpha kept (:377-379, :109).
[[maybe_unused]] __device__ __forceinline__ uint32_t shade_rgba(uint32_t texel, float brightness) {
  const uint32_t r = __float2uint_rz((float)(texel & 0xffu) * brightness);
  const uint32_t g = __float2uint_rz((float)((texel >> 8) & 0xffu) * brightness);
  const uint32_t b = __float2uint_rz((float)((texel >> 16) & 0xffu) * brightness);
  return (r & 0xffu) | ((g & 0xffu) << 8) | ((b & 0xffu) << 16) | (texel & 0xff000000u);
}

// Cone of the wave's rays: unit axis through the tile centre, and the sine
// and cosine of a half-angle that contains every lane's unit ray.  The sine
// is taken from |d x a| (accurate for the small angles of a tile, unlike a
// cosine near 1), maximised over the wave, plus slack for binary32 rounding.
// A tile whose rays spread past ~60 degrees (strided subsets) gets wide = true
// and is not culled.
// Square roots of the culling geometry (cone, window): the raw v_sqrt_f32, within 1 ulp of
// the correctly rounded root for normal arguments (the compiler's sqrtf adds a rescaling for
// arguments below 2^-96 and a correction step).  Every use is covered by a slack far above
// 1 ulp: 4e-6 |w| on the cone distances, 1e-5 on the half-angle's sine and relative on the
// window half-width, plus the absolute cull margin; below 2^-96 the root's absolute error is
// below 2^-48 either way.
__device__ __forceinline__ float sqrt_cull(float x) { return __builtin_amdgcn_sqrtf(x); }

struct Cone {
  float ax, ay, az, cos_t, sin_t;
  bool wide;
};

// Wave-level cull ("wavefront ballot") plus march window.  Lane l tests sphere
// base + l against the cone; bit l of the result is set when the sphere may
// pass the march test for some ray of the wave's tile.  A sphere is dropped
// only when its distance to the cone exceeds its radius inflated by
// f.cull_margin, which bounds how far the binary32 march positions can drift
// from their rays (sfrt_world.cpp) -- there r - |p - c| > 0.01f cannot hold.
// The distance from a centre at axial coordinate t and radial distance perp to
// the cone's side line is perp * cos_t - t * sin_t; it is the distance to the
// cone where the centre projects onto the side, and a lower bound of it
// everywhere (behind the apex the distance is |w|).  Evaluating it in binary32
// errs by < 1e-6 |w|, covered by the 4e-6 |w| slack.  Spheres whose pass
// threshold is 0 never pass and are dropped.  In addition lane l returns, for
// sphere base + l, an interval (lo, hi) of along-ray distance outside which
// the sphere cannot pass for any ray of the cone.  A ray's march position p
// at along-ray distance tau lies within the drift bound of the ray's point
// cam + u*tau (cull_margin), so a pass needs |cam + u*tau - c| < rr, i.e.
// |tau - dot(w, u)| < sqrt(rr^2 - d^2) with d the distance of the centre from
// the ray's line (the half-width h below bounds it over the cone).  Over the
// cone's rays dot(w, u) = |w| cos(angle(w, u)) with the angle in
// [max(0, alpha - theta), min(pi, alpha + theta)] (alpha = angle(w, axis),
// theta = half-angle): |w| cos(alpha -+ theta) = t cos_t +- perp sin_t,
// clamped to +-|w| where alpha - theta < 0 or alpha + theta > pi.  The
// interval is widened by h + cull_margin: the binary32 error of the lanes'
// accumulated distance (<= 1.3e-4 R over kCullSafeIterations steps) and of
// these expressions fit in the second margin.
__device__ __forceinline__ uint64_t cull_window(const FrameRec& f, const SphereRec* __restrict__ sph,
                                                int base, const Cone& c, float& lo, float& hi) {
  const int k = base + (int)(threadIdx.x & 63);
  bool inc = false;
  lo = __builtin_inff();
  hi = -__builtin_inff();
  if (k < f.n) {
    const SphereRec s = sph[k];
    if (s.s_pass > 0.0f) {
      const float wx = s.cx - f.cam[0], wy = s.cy - f.cam[1], wz = s.cz - f.cam[2];
      const float wl = sqrt_cull((wx * wx + wy * wy) + wz * wz);
      const float rr = s.r + f.cull_margin + 4e-6f * wl;
      const float t = (wx * c.ax + wy * c.ay) + wz * c.az;
      const float px = wx - t * c.ax, py = wy - t * c.ay, pz = wz - t * c.az;
      const float perp = sqrt_cull((px * px + py * py) + pz * pz);
      const bool side = t * c.cos_t + perp * c.sin_t >= -rr;
      const float sa = perp * c.cos_t - t * c.sin_t;  // |w| sin(alpha - theta)
      inc = c.wide || wl <= rr || (side && sa <= rr);
      if (inc) {
        if (c.wide) {
          hi = __builtin_inff();
          lo = -__builtin_inff();
        } else {
          const float sb = perp * c.cos_t + t * c.sin_t;  // |w| sin(alpha + theta)
          const float up = sa >= 0.0f ? t * c.cos_t + perp * c.sin_t : wl;
          const float dn = sb >= 0.0f ? t * c.cos_t - perp * c.sin_t : -wl;
          // Half-width: a ray whose line passes the centre at distance d has |q - c|^2 =
          // (tau - dot(w, u))^2 + d^2 at its exact point q(tau), so a pass (|q - c| < rr)
          // needs |tau - dot(w, u)| < sqrt(rr^2 - d^2).  Over the cone d >= |w| *
          // min(sin(alpha - theta), sin(alpha + theta)) = min(sa, sb) when both are >= 0
          // (else the cone's angles reach 0 or pi and d can be 0), taken 4e-6 |w| lower
          // for the binary32 error of sa and sb; the product form keeps the root's
          // relative error at a few ulps, and the 1e-5 relative slack covers it.
          const float dmin = fmaxf(0.0f, fminf(sa, sb) - 4e-6f * wl);
          const float h = sqrt_cull((rr - dmin) * (rr + dmin)) * 1.00001f;
          const float ext = h + f.cull_margin;
          lo = dn - ext;
          hi = up + ext;
        }
      }
    }
  }
  return __builtin_amdgcn_ballot_w64(inc);
}

// Record k read through the constant address space: the records are never written
// while a launch runs (kernel arguments, or a device ring slot reused only after the
// event of the launch that read it), and wave-uniform loads from that space are scalar
// loads -- through the generic pointer the compiler must assume the frame's stores may
// alias them and emits vector loads into VGPRs (the n > 64 kernel's records).
// k is unsigned and < 2^27, so k * 32 is a 32-bit byte offset the scalar load takes as its
// SGPR offset (a signed index costs a 64-bit shift and add per record).
__device__ __forceinline__ SphereRec rec_at(const SphereRec* p, uint32_t k) {
  const __attribute__((address_space(4))) uint32_t* q =
      (const __attribute__((address_space(4))) uint32_t*)(
          (const __attribute__((address_space(4))) char*)p + k * (uint32_t)sizeof(SphereRec));
  uint32_t w[sizeof(SphereRec) / 4];
#pragma unroll
  for (int i = 0; i < (int)(sizeof(SphereRec) / 4); i++) w[i] = q[i];
  SphereRec r;
  __builtin_memcpy(&r, w, sizeof r);
  return r;
}

// std::max(largestDist, t) (SphereWorld.cpp:367) for L >= +0 and t > 0.01f
// (the pass test), both finite: their bit patterns order like the values, so
// one v_max_u32 gives the compare-select's bits (v_max_f32 would first
// canonicalise the loop-carried L).
__device__ __forceinline__ float max_nonneg(float L, float t) {
  return __uint_as_float(__builtin_elementwise_max(__float_as_uint(L), __float_as_uint(t)));
}

// One sphere test of the march (SphereWorld.cpp:365-369), exact: the pass
// test is s < s_pass (see sfrt_world.cpp, pass_threshold) and sqrtf runs only
// for a sphere that passes.
__device__ __forceinline__ float dist2(float px, float py, float pz, float cx, float cy,
                                       float cz) {
  const float ex = px - cx, ey = py - cy, ez = pz - cz;
  return (ex * ex + ey * ey) + ez * ez;
}

// Cone of an (8R)x8 tile whose lanes hold R rays each (columns c, c + 8, ...).
template <int R>
__device__ __forceinline__ Cone tile_cone_r(const FrameRec& f, int tile_x, int tile_y,
                                            const float (&dx)[R], const float (&dy)[R],
                                            const float (&dz)[R]) {
  const float ic = (float)f.xstart +
                   ((float)(tile_x * R * kTile) + (0.5f * (float)(R * kTile) - 0.5f)) * (float)f.xadd;
  const float jc = (float)f.ystart +
                   ((float)(f.sub_row0 + tile_y * kTile) + 3.5f) * (float)f.yadd;
  const float h = f.h_start + f.h_inc * ic;
  const float v = f.v_start + jc * f.v_inc;
  float ax = (f.fwd[0] + f.right[0] * h) + f.up[0] * v;
  float ay = (f.fwd[1] + f.right[1] * h) + f.up[1] * v;
  float az = (f.fwd[2] + f.right[2] * h) + f.up[2] * v;
  const float inv = __builtin_amdgcn_rsqf((ax * ax + ay * ay) + az * az);
  ax *= inv; ay *= inv; az *= inv;
  float sin_l = 0.0f;
  bool wide = false;
#pragma unroll
  for (int r = 0; r < R; r++) {
    const float cx = dy[r] * az - dz[r] * ay, cy = dz[r] * ax - dx[r] * az,
                cz = dx[r] * ay - dy[r] * ax;
    sin_l = fmaxf(sin_l, sqrt_cull((cx * cx + cy * cy) + cz * cz));
    wide = wide || ((dx[r] * ax + dy[r] * ay) + dz[r] * az) < 0.5f;
  }
  Cone c;
  c.ax = ax; c.ay = ay; c.az = az;
  c.sin_t = fminf(1.0f, __uint_as_float(wave_max_u32(__float_as_uint(sin_l))) + 1e-5f);
  c.cos_t = sqrt_cull(fmaxf(0.0f, 1.0f - c.sin_t * c.sin_t));
  c.wide = __builtin_amdgcn_ballot_w64(wide) != 0;
  return c;
}


// The same cone from the tile's four corner rays only.  Restricted to the image plane
// {fwd + right h + up v}, the angle to the axis has convex sublevel sets below 90 degrees (a
// convex circular cone cut by a plane), so over the tile's rectangle of (h, v) it is largest
// at a corner; every ray of the tile, edge duplicates included, lies in that rectangle (h and
// v are monotone in the pixel indices, also after rounding).  So if every corner ray is
// within 60 degrees of the axis, so is every ray, and the largest corner sine plus the same
// 1e-5 slack bounds every ray's (the slack covers the binary32 error of the corners' and of
// the rays' directions, a few 1e-8); otherwise the tile is wide.  Lane l computes corner l % 4.
template <int R>
__device__ __forceinline__ Cone tile_cone_corners(const FrameRec& f, int tile_x, int tile_y, int lane) {
  const float ic = (float)f.xstart +
                   ((float)(tile_x * R * kTile) + (0.5f * (float)(R * kTile) - 0.5f)) * (float)f.xadd;
  const float jc = (float)f.ystart +
                   ((float)(f.sub_row0 + tile_y * kTile) + 3.5f) * (float)f.yadd;
  const float hc = f.h_start + f.h_inc * ic;
  const float vc = f.v_start + jc * f.v_inc;
  float ax = (f.fwd[0] + f.right[0] * hc) + f.up[0] * vc;
  float ay = (f.fwd[1] + f.right[1] * hc) + f.up[1] * vc;
  float az = (f.fwd[2] + f.right[2] * hc) + f.up[2] * vc;
  const float inv = __builtin_amdgcn_rsqf((ax * ax + ay * ay) + az * az);
  ax *= inv; ay *= inv; az *= inv;
  // corner lane % 4: column 0 or 8R - 1, row 0 or 7 of the tile, clamped like the rays
  const int a0 = tile_x * R * kTile + ((lane & 1) ? R * kTile - 1 : 0);
  const int b0 = f.sub_row0 + tile_y * kTile + ((lane & 2) ? kTile - 1 : 0);
  const int a = a0 < f.sub_w ? a0 : f.sub_w - 1;
  const int b = b0 < f.sub_row0 + f.sub_rows ? b0 : f.sub_row0 + f.sub_rows - 1;
  const float h = f.h_start + f.h_inc * (float)(f.xstart + a * f.xadd);
  const float v = f.v_start + (float)(f.ystart + b * f.yadd) * f.v_inc;
  float x = (f.fwd[0] + f.right[0] * h) + f.up[0] * v;
  float y = (f.fwd[1] + f.right[1] * h) + f.up[1] * v;
  float z = (f.fwd[2] + f.right[2] * h) + f.up[2] * v;
  const float il = __builtin_amdgcn_rsqf((x * x + y * y) + z * z);
  x *= il; y *= il; z *= il;
  const float cx = y * az - z * ay, cy = z * ax - x * az, cz = x * ay - y * ax;
  const float sin_l = sqrt_cull((cx * cx + cy * cy) + cz * cz);
  Cone c;
  c.ax = ax; c.ay = ay; c.az = az;
  c.sin_t = fminf(1.0f, __uint_as_float(wave_max_u32(__float_as_uint(sin_l))) + 1e-5f);
  c.cos_t = sqrt_cull(fmaxf(0.0f, 1.0f - c.sin_t * c.sin_t));
  c.wide = __builtin_amdgcn_ballot_w64(!(((x * ax + y * ay) + z * az) >= 0.5f)) != 0;
  return c;
}

// L = +0 for a lane's R rays at the start of a march step, two registers per
// v_mov_b64 (left to itself the compiler copies one zero register into three
// others and then pairs them: five moves a step for R = 4, not two).
template <int R>
__device__ __forceinline__ void zero_steps(float (&L)[R]) {
#pragma unroll
  for (int r = 0; r + 1 < R; r += 2) {
    uint64_t z;
    __asm__ volatile("v_mov_b64 %0, 0" : "=v"(z));
    L[r] = __uint_as_float((uint32_t)z);
    L[r + 1] = __uint_as_float((uint32_t)(z >> 32));
  }
  if (R & 1) L[R - 1] = 0.0f;
}

// Pass bodies of one sphere for the lane's R rays under one scalar branch.
// (Lane-masked selects through inline asm instead of these exec-masked
// updates were measured slower: 1% at R = 2, 15% at R = 1.)
// sqrt_cr_normal serves every passing lane, also ss < 2^-96, where it is not
// the correctly rounded sqrt: a pass needs rad - sqrtf(ss) > 0.01f, so
// rad > 2^-7, and rad - q == rad for any q < 2^-33, which both roots of such
// ss are (tests/native/wave_check.hip, every ss).
template <int R>
__device__ __forceinline__ bool pass_body_r(const float (&ss)[R], float s_pass, float rad, int k,
                                            float (&L)[R], int (&draw)[R]) {
  uint64_t any = 0;
#pragma unroll
  for (int r = 0; r < R; r++) any |= __builtin_amdgcn_ballot_w64(ss[r] < s_pass);
  if (any) {
    __asm__ volatile("; sphere passes for some ray of the wave");  // keeps the branch
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (ss[r] < s_pass) {
        const float t = rad - sqrt_cr_normal(ss[r]);
        L[r] = max_nonneg(L[r], t);
        draw[r] = k;
      }
    }
  }
  return any != 0;
}

// The march (SphereWorld.cpp:359-372), one wave per (8R)x8 tile.  Lane l holds
// R rays (columns c, c + 8, ...), so the wave-uniform half of a sphere visit --
// record load, window bits, branch -- is shared by R rays and each lane carries
// R independent dependency chains.  Per wave: cull the spheres against the tile
// cone (cull_window).  With n <= 64 (LIST = false, records in the kernel
// arguments) lane l holds sphere l's march window and bit l of the culling mask
// is sphere l; with n > 64 (LIST, records in device memory) the culled spheres
// of every 64-sphere word are compacted, in index order, into lanes 0.. of a
// culled list (cidx = the sphere index) -- a wave that culls more than 64
// visits every sphere every step instead (exact; rare at the tile sizes used).
// A wave with <= kSlots culled spheres holds them in SGPRs and tests each every
// step; otherwise each step visits, in index order, the culled spheres whose
// march window meets the along-ray distances [min over marching rays, max over
// the wave] (the low end refreshed every second step: it only rises).  Then
// shade and store.
//
// A stopped ray advances unmasked: it had no passing sphere at its position
// (its last step visited every sphere that could pass for it) and never moves
// again, so each later step again has none: L = +0, draw unchanged, tacc + 0 =
// tacc, and p + d * (+0) = p -- also for p = -0, which a marching wave's ray
// only reaches through -0 + d * l0 with d of negative sign, so d * (+0) = -0.
// Edge lanes trace a clamped duplicate pixel (never stored) as the duplicate
// it is, which keeps the tile cone tight.
// DUMP (sfrt_world_trace_points only): the same march and shading, plus a per-ray
// iteration count and an epilogue writing the float intermediates of listed pixels.
// P: the probe hooks (sfrt_probe.h; NoProbe in the shipped library, all empty).
template <int R, bool LIST, bool DUMP, class P>
__device__ __forceinline__ void trace_tile_window_r(const FrameRec& f,
                                                    const SphereRec* __restrict__ sph,
                                                    DumpArgs dmp) {
  const int lane = threadIdx.x & 63;
  P probe;
  probe.wave_entry();
  // Adaptive tile order (sfrt_trace.h FrameRec): workgroup 0 may be the sorter.
  const int ntiles = f.tiles_x * ((f.sub_rows + kTile - 1) / kTile);
  int slot = (int)blockIdx.x;
  if (f.prev_cost) {
    if (blockIdx.x == 0) {
      sort_tiles(f.prev_cost, ntiles, f.next_order, f.order_dilate != 0);
      return;
    }
    slot -= 1;
  }
  uint32_t cls;  // the tile's class in the order (sfrt_device.h slot_tile)
  const int tile = slot_tile(f.tile_order, slot, ntiles, cls);
  const int tile_y = tile / f.tiles_x;  // f.tiles_x = ceil(sub_w / (8 R)) for this kernel
  const int tile_x = tile - tile_y * f.tiles_x;
  if (tile_y * kTile >= f.sub_rows) return;  // grid rounding; uniform per wave
  probe.tile_begin();
  const int b = f.sub_row0 + tile_y * kTile + (lane >> 3);
  const int b_end = f.sub_row0 + f.sub_rows;
  const int bc = b < b_end ? b : b_end - 1;
  const int j = f.ystart + bc * f.yadd;
  const float l0 = f.first_l;
  int draw[R];
  int iters[R];  // DUMP only: loop trips of :362 per ray, the host's first one included
  float dx[R], dy[R], dz[R], px[R], py[R], pz[R], mv[R], tacc[R];
  // mv: the ray's last step length (> 0 while it marches, +0 once it stopped);
  // `mv > 0` is one compare per step, where a loop-carried bool would be
  // rematerialised through VGPRs.
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int a = tile_x * R * kTile + r * kTile + (lane & 7);
    const int ac = a < f.sub_w ? a : f.sub_w - 1;
    primary_dir(f, f.xstart + ac * f.xadd, j, dx[r], dy[r], dz[r]);
    px[r] = f.cam[0] + dx[r] * l0;
    py[r] = f.cam[1] + dy[r] * l0;
    pz[r] = f.cam[2] + dz[r] * l0;
    draw[r] = f.first_draw;
    iters[r] = 1;
    mv[r] = l0 > 0.0f ? 1.0f : 0.0f;
    tacc[r] = l0;  // along-ray distance marched (binary32 sum of the steps)
  }
  auto any_marching = [&]() {
    uint64_t q = 0;
#pragma unroll
    for (int r = 0; r < R; r++) q |= __builtin_amdgcn_ballot_w64(mv[r] > 0.0f);
    return q != 0;
  };
  const bool windowed = f.cull && l0 > 0.0f;
  bool full = !windowed;  // visit every sphere every step
  uint64_t m = 0;         // culled spheres (LIST: culled-list entries)
  float lo = -__builtin_inff(), hi = __builtin_inff();
  int cidx = lane;        // sphere of culled-list entry `lane`
  if (windowed) {
    // R >= 3: four corner rays per wave are cheaper than R rays per lane (profiles/ab/r3_ab9)
    const Cone cone = R >= 3 ? tile_cone_corners<R>(f, tile_x, tile_y, lane)
                             : tile_cone_r<R>(f, tile_x, tile_y, dx, dy, dz);
    if (!LIST) {
      m = cull_window(f, sph, 0, cone, lo, hi);
    } else {
      __shared__ float s_list[3][64];  // compaction scratch: lo, hi, index
      int count = 0;
      const int nwords = (f.n + 63) >> 6;
      for (int w = 0; w < nwords; w++) {
        float wlo, whi;
        const uint64_t mw = cull_window(f, sph, w * 64, cone, wlo, whi);
        const int cw = __builtin_popcountll(mw);
        if (count + cw > 64) {
          full = true;
          break;
        }
        if ((mw >> lane) & 1ull) {
          const int dst = count + (int)__builtin_amdgcn_mbcnt_hi(
                                      (uint32_t)(mw >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mw, 0u));
          s_list[0][dst] = wlo;
          s_list[1][dst] = whi;
          s_list[2][dst] = __int_as_float(w * 64 + lane);
        }
        count += cw;
      }
      __syncthreads();  // one wave: orders its own LDS writes before the reads
      if (!full) {
        m = count >= 64 ? ~0ull : ((1ull << count) - 1ull);
        if (lane < count) {
          lo = s_list[0][lane];
          hi = s_list[1][lane];
          cidx = __float_as_int(s_list[2][lane]);
        }
      }
    }
  }
  // sphere of culled entry e (wave-uniform)
  auto entry = [&](uint32_t e) { return LIST ? (uint32_t)__builtin_amdgcn_readlane(cidx, (int)e) : e; };
  // First set bit of a 64-bit culling mask, 63 for an empty mask (s_ff1 gives -1): entry 63 is
  // always readable -- a record of the n <= 64 kernel's argument block, or lane 63 of the list
  // (its sphere, or sphere 63 < n) -- so a lookahead past the last entry loads a record it never uses.
  static_assert(kInlineSpheres == 64,
                "entry 63 must be readable: record 63 of the 64-entry argument block, or lane 63 "
                "of the list kernel's culled list (that kernel runs only for n > kInlineSpheres, "
                "so lane 63's default sphere 63 exists; launch_trace checks n >= 64)");
  auto first_entry = [](uint64_t x) -> uint32_t {
    uint32_t e;
    __asm__("s_ff1_i32_b64 %0, %1" : "=s"(e) : "s"(x));
    return e & 63u;
  };
  auto clear_entry = [](uint64_t x, uint32_t e) -> uint64_t { return x & ~(1ull << e); };  // s_bitset0

  // pos += dir * L (SphereWorld.cpp:371) on every lane (see above)
  auto advance = [&](const float (&L)[R]) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      px[r] = px[r] + dx[r] * L[r];
      py[r] = py[r] + dy[r] * L[r];
      pz[r] = pz[r] + dz[r] * L[r];
      if constexpr (DUMP) iters[r] += mv[r] > 0.0f ? 1 : 0;  // a step of a marching ray
      mv[r] = L[r];
      tacc[r] = tacc[r] + L[r];
    }
  };
  auto visit = [&](float cx, float cy, float cz, float rad, float s_pass, int k, float (&L)[R]) {
    float ss[R];
#pragma unroll
    for (int r = 0; r < R; r++) ss[r] = dist2(px[r], py[r], pz[r], cx, cy, cz);
    probe.visit(pass_body_r<R>(ss, s_pass, rad, k, L, draw));
  };
  // Every sphere in index order (no culling: cull off, or past kCullSafeIterations steps).
  auto visit_all = [&](float (&L)[R]) {
    for (int k = 0; k < f.n; k++) {
      const SphereRec s = rec_at(sph, k);
      visit(s.cx, s.cy, s.cz, s.r, s.s_pass, k, L);
    }
  };
  int trips = 1;
  // Culled steps run while trips < kCullSafeIterations (the margins' bound, sec. 4 of
  // DESIGN.md); a wave still marching then continues in the full-list loop below.  Each
  // loop is single-exit (the guard is its condition) with one body shape: a second exit,
  // or a full/culled branch inside the step, makes the compiler copy every loop-carried
  // register (draw, L) between register sets each step.
  const int cull_end = full ? 1 : kCullSafeIterations;
  constexpr int kSlotsR = kSlots;
  if (kSlotsR > 0 && !full && __builtin_popcountll(m) <= kSlotsR) {
    constexpr int NS = kSlotsR > 0 ? kSlotsR : 1;
    // Few culled spheres: hold them in SGPR slots and test every one each step
    // (cheaper than maintaining the window).  Empty slots never pass.
    float scx[NS], scy[NS], scz[NS], sr[NS], ssp[NS];
    int sk[NS];
    uint64_t mm = m;
#pragma unroll
    for (int q = 0; q < kSlotsR; q++) {
      scx[q] = scy[q] = scz[q] = sr[q] = ssp[q] = 0.0f;
      sk[q] = 0;
      if (mm) {
        const int k = entry(__builtin_ctzll(mm));
        mm &= mm - 1;
        const SphereRec s = rec_at(sph, k);
        scx[q] = s.cx; scy[q] = s.cy; scz[q] = s.cz;
        sr[q] = s.r; ssp[q] = s.s_pass;
        sk[q] = k;
      }
    }
    for (; any_marching() && trips < cull_end; ++trips) {
      float L[R];
      zero_steps<R>(L);
#pragma unroll
      for (int q = 0; q < kSlotsR; q++) visit(scx[q], scy[q], scz[q], sr[q], ssp[q], sk[q], L);
      advance(L);
    }
  } else {
    probe.window_mode();
    float tlo = 0.0f;
    for (; any_marching() && trips < cull_end; ++trips) {
      float L[R];
      zero_steps<R>(L);
      // tacc >= +0: reduce the bit patterns (wave_min_u32 / wave_max_u32)
      uint32_t th = 0u;  // +0
#pragma unroll
      for (int r = 0; r < R; r++) {
        const uint32_t u = __float_as_uint(tacc[r]);
        th = u > th ? u : th;
      }
      if (trips % 2 == 1) {  // the low end, every second step (every 3rd/4th: slower)
        uint32_t tl = 0x7f800000u;  // +inf
#pragma unroll
        for (int r = 0; r < R; r++) {
          const uint32_t u = __float_as_uint(tacc[r]);
          const uint32_t ua = mv[r] > 0.0f ? u : 0x7f800000u;
          tl = ua < tl ? ua : tl;
        }
        tlo = __uint_as_float(wave_min_u32(tl));
      }
      const float thi = __uint_as_float(wave_max_u32(th));
      const uint64_t win =
          m & __builtin_amdgcn_ballot_w64(lo < thi) & __builtin_amdgcn_ballot_w64(hi > tlo);
      // The visits, in index order, each issuing the next record's scalar loads
      // before its own arithmetic (the loads' latency hides under the R rays'
      // distance tests; past the last entry the lookahead loads entry 63's record,
      // unused).  Scalar work per visit is kept short: the scalar unit is shared by
      // the CU's four SIMDs (profiles/r3y_salu_mix_check.txt).
      if (win) {
        uint32_t e = first_entry(win);
        uint64_t mm = clear_entry(win, e);
        uint32_t k = entry(e);
        const SphereRec s0 = rec_at(sph, k);
        float cx = s0.cx, cy = s0.cy, cz = s0.cz, rad = s0.r, sp = s0.s_pass;
        bool more;
        do {  // the exit test at the bottom: a mid-loop exit made the back edge ~18 scalar ops
          const uint32_t en = first_entry(mm);
          const uint32_t kn = entry(en);
          const SphereRec sn = rec_at(sph, kn);
          const float ncx = sn.cx, ncy = sn.cy, ncz = sn.cz, nr = sn.r, nsp = sn.s_pass;
          visit(cx, cy, cz, rad, sp, (int)k, L);
          more = mm != 0;
          mm = clear_entry(mm, en);
          k = kn; cx = ncx; cy = ncy; cz = ncz; rad = nr; sp = nsp;
        } while (more);
      }
      advance(L);
    }
  }
  // Every sphere in index order, every step: culling off, or past kCullSafeIterations.
  for (; any_marching() && trips < kMaxIterations; ++trips) {
    float L[R];
    zero_steps<R>(L);
    visit_all(L);
    advance(L);
  }
  if (trips >= kMaxIterations && any_marching() && lane == 0) atomicOr(f.status, 1);
  if (f.tile_cost && lane == 0) store_cost(f.tile_cost, tile, tile_bucket((uint32_t)trips), cls, f.cost_diff);
  // Pixel (a, b) of ray r, recomputed here from a fresh lane id (mbcnt, so that the
  // compiler does not reuse the kernel entry's values): kept from there, the columns sat
  // in registers through the whole march, and at R = 4 one of them was spilled.
  const int lane_s = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int b_s = f.sub_row0 + tile_y * kTile + (lane_s >> 3);
  auto col = [&](int r) { return tile_x * R * kTile + r * kTile + (lane_s & 7); };
  auto valid = [&](int r) { return col(r) < f.sub_w && b_s < b_end; };
  // the row's first pixel, once per lane (inside each slot's store branch the compiler
  // recomputed the 64-bit row offset, three quarter-rate multiplies per slot)
  uint32_t* const row_out = f.out + (long long)(b_s - f.sub_row0) * f.out_pitch;
  auto px_out = [&](int r) { return row_out + col(r); };
  if constexpr (!P::kShade) {  // timing probe (sfrt_probe.h): the march without the shading tail
#pragma unroll
    for (int r = 0; r < R; r++)
      if (valid(r))
        probe.march_only(px_out(r), __float_as_uint(px[r]) ^ __float_as_uint(py[r]) ^
                                        __float_as_uint(pz[r]) ^ (uint32_t)draw[r]);
  } else {
    // Shading: the R records gathered first, then the R texel indices, the R texel
    // loads back to back, and the stores.  Edge lanes shade their duplicates too
    // (same values as the real pixel) and store nothing.
    SphereRec d[R];
#pragma unroll
    for (int r = 0; r < R; r++)  // draw < n <= 1024: a 32-bit byte offset from the records' base
      d[r] = *(const SphereRec*)((const char*)sph + (uint32_t)draw[r] * (uint32_t)sizeof(SphereRec));
    Shading sh[R];
    PixelDump dl[DUMP ? R : 1];
#pragma unroll
    for (int r = 0; r < R; r++)
      sh[r] = shade_texel<P>(f, d[r], px[r], py[r], pz[r], DUMP ? &dl[DUMP ? r : 0] : nullptr);
    uint32_t texel[R];
#pragma unroll
    for (int r = 0; r < R; r++) texel[r] = f.tex[sh[r].tex];
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (valid(r)) {
        if (sh[r].outside) atomicOr(f.status, 2);  // the reference would read outside the image
        const uint32_t rgba = shade_rgba(sh[r].outside ? 0u : texel[r], sh[r].brightness);
        if constexpr (!DUMP) {
          *px_out(r) = rgba;
        } else {  // the listed pixel's record, if it is listed (no frame store)
          const long long pid = (long long)(b_s - f.sub_row0) * f.sub_w + col(r);
          int q = 0, qe = dmp.npix;  // first entry >= pid
          while (q < qe) {
            const int mid = (q + qe) >> 1;
            if (dmp.pix[mid] < pid) q = mid + 1;
            else qe = mid;
          }
          if (q < dmp.npix && dmp.pix[q] == pid) {
            PixelDump& o = dl[r];
            o.pos[0] = px[r]; o.pos[1] = py[r]; o.pos[2] = pz[r];
            o.draw = draw[r];
            o.iters = iters[r];
            o.rgba = rgba;
            dmp.out[q] = o;
          }
        }
      }
    }
  }
  probe.tile_end(px_out(0), lane_s, valid(0), trips, slot, m);
}

// n <= 64: the records travel in the kernel-argument segment.  8 waves/SIMD: <= 64
// VGPRs (R = 4 needs 60; measured equal to 7 waves when it spilled one, ab/r2_ab10).
template <int R>
__global__ __launch_bounds__(64, 8) void k_trace_window_r(InlineArgs args) {
  trace_tile_window_r<R, false, false, ActiveProbe>(args.f, args.s, DumpArgs{});
}

// n > 64: the records in device memory (f.spheres, read with scalar loads: rec_at), the
// culled list per wave.  57 VGPRs at R = 4 (8 waves/SIMD).
template <int R>
__global__ __launch_bounds__(64) void k_trace_window_list(FrameRec f) {
  trace_tile_window_r<R, true, false, ActiveProbe>(f, f.spheres, DumpArgs{});
}

// The DUMP instantiations of both (sfrt_world_trace_points): the shipped march and
// shading, with the float intermediates of listed pixels written out (never probed).
template <int R>
__global__ __launch_bounds__(64) void k_trace_window_r_dump(InlineArgs args, DumpArgs d) {
  trace_tile_window_r<R, false, true, NoProbe>(args.f, args.s, d);
}
template <int R>
__global__ __launch_bounds__(64) void k_trace_window_list_dump(FrameRec f, DumpArgs d) {
  trace_tile_window_r<R, true, true, NoProbe>(f, f.spheres, d);
}


}  // namespace

// Pixels per lane R of an ordered launch (adaptive tile order): the widest
// tile -- four pixels per lane (32x8), else three (24x8) -- whose grid still
// has >= 30000 tiles, about four waves per wave slot of the chip, enough for
// longest-first to balance; else two (16x8).  Measured: 4K 64 spheres 177
// (16x8) -> 173.5 (24x8) -> 172.9 us (32x8), 8K 645.6 -> 636.7 us (24x8 ->
// 32x8); 1080p 10 spheres 37.3 us at 16x8 against 39.4 / 41.0 wider.
static int ordered_rays(const FrameRec& f) {
  const long long rows = (f.sub_rows + kTile - 1) / kTile;
  const long long t4 = (long long)((f.sub_w + 4 * kTile - 1) / (4 * kTile)) * rows;
  const long long t3 = (long long)((f.sub_w + 3 * kTile - 1) / (3 * kTile)) * rows;
  return t4 >= 30000 ? 4 : t3 >= 30000 ? 3 : 2;
}

// The one kernel table, shared by launch_trace and trace_tile_key: pixels per
// lane R (k_trace_window_r for n <= 64, k_trace_window_list above).  Row-major launches
// use 16x8 tiles above kPairMinSpheres spheres and 8x8 tiles otherwise (their
// tighter cones win there); ordered launches ordered_rays for any scene (1080p,
// 10 spheres: 16x8 37.4 us against 42.0 with 8x8, which win only in row-major
// order: 45.7 vs 48.5).  f.rays (SFRT_OPT_RAYS_PER_LANE) overrides the choice.
static int trace_rays(const FrameRec& f, bool ordered) {
  if (f.rays >= 1 && f.rays <= 4) return f.rays;
  if (ordered) return ordered_rays(f);
  return f.n > kPairMinSpheres ? 2 : 1;
}

const char* trace_build_flavour() {
  return kDiagnosticBuild ? "diagnostic" : kSlots != 2 ? "ab" : SFRT_BUILD_FLAVOUR;
}

long long trace_tile_key(const FrameRec& f, long long* tiles) {
  *tiles = 0;
  const int rays = trace_rays(f, true);
  const long long tiles_x = (f.sub_w + rays * kTile - 1) / (rays * kTile);
  const long long tiles_y = (f.sub_rows + kTile - 1) / kTile;
  if (tiles_x <= 0 || tiles_y <= 0) return 0;
  *tiles = tiles_x * tiles_y;
  return (1ll << 62) | ((long long)rays << 56) | (tiles_x << 28) | tiles_y;
}

int launch_trace(const FrameRec& f, const SphereRec* host_spheres, void* stream,
                 const DumpArgs* dump, void* done_event) {
  const long long tiles_y = (f.sub_rows + kTile - 1) / kTile;
  if (tiles_y <= 0 || f.sub_w <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const bool ordered = f.tile_cost != nullptr;  // linked into the tile-order chain
  const int rays = trace_rays(f, ordered);
  FrameRec g = f;
  g.tiles_x = (f.sub_w + rays * kTile - 1) / (rays * kTile);
  const long long tiles = tiles_y * g.tiles_x;
  long long key_tiles = 0;
  if (!ordered || trace_tile_key(f, &key_tiles) == 0 || key_tiles != tiles) {
    g.tile_order = nullptr; g.tile_cost = nullptr; g.prev_cost = nullptr;
  }
  // one wave per workgroup (a finished wave's slot refills at once), plus the
  // tile-order sorter (sfrt_trace.h FrameRec)
  const long long blocks = tiles + (g.prev_cost ? 1 : 0);
  if (blocks > 0x7fffffffLL) return -1;
  const dim3 gr((unsigned)blocks), b(64);
  if (f.n <= kInlineSpheres) {
    InlineArgs args;
    args.f = g;
    for (int k = 0; k < f.n; k++) args.s[k] = host_spheres[k];
    if (dump) {
      switch (rays) {
        case 1: hipLaunchKernelGGL(k_trace_window_r_dump<1>, gr, b, 0, s, args, *dump); break;
        case 2: hipLaunchKernelGGL(k_trace_window_r_dump<2>, gr, b, 0, s, args, *dump); break;
        case 3: hipLaunchKernelGGL(k_trace_window_r_dump<3>, gr, b, 0, s, args, *dump); break;
        default: hipLaunchKernelGGL(k_trace_window_r_dump<4>, gr, b, 0, s, args, *dump); break;
      }
    } else {
      switch (rays) {
        case 1: hipLaunchKernelGGL(k_trace_window_r<1>, gr, b, 0, s, args); break;
        case 2: hipLaunchKernelGGL(k_trace_window_r<2>, gr, b, 0, s, args); break;
        case 3: hipLaunchKernelGGL(k_trace_window_r<3>, gr, b, 0, s, args); break;
        default: hipLaunchKernelGGL(k_trace_window_r<4>, gr, b, 0, s, args); break;
      }
    }
  } else if (f.n < 64) {
    return -1;  // the list kernel's lookahead reads culled-list lane 63 (a sphere index < n)
  } else if (dump) {
    switch (rays) {
      case 1: hipLaunchKernelGGL(k_trace_window_list_dump<1>, gr, b, 0, s, g, *dump); break;
      case 2: hipLaunchKernelGGL(k_trace_window_list_dump<2>, gr, b, 0, s, g, *dump); break;
      case 3: hipLaunchKernelGGL(k_trace_window_list_dump<3>, gr, b, 0, s, g, *dump); break;
      default: hipLaunchKernelGGL(k_trace_window_list_dump<4>, gr, b, 0, s, g, *dump); break;
    }
  } else {
    const hipEvent_t ev = (hipEvent_t)done_event;  // the record ring's slot (sfrt_world.cpp)
    switch (rays) {
      case 1: hipExtLaunchKernelGGL(k_trace_window_list<1>, gr, b, 0, s, nullptr, ev, 0, g); break;
      case 2: hipExtLaunchKernelGGL(k_trace_window_list<2>, gr, b, 0, s, nullptr, ev, 0, g); break;
      case 3: hipExtLaunchKernelGGL(k_trace_window_list<3>, gr, b, 0, s, nullptr, ev, 0, g); break;
      default: hipExtLaunchKernelGGL(k_trace_window_list<4>, gr, b, 0, s, nullptr, ev, 0, g); break;
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace sfrt
