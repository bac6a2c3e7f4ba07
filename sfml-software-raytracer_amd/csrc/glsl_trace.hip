// glsl_trace.hip -- gfx950 kernel for the GLSL renderer:
// one lane per fragment of rayShader.frag (/root/reference/Raytracing/
// rayShader.frag:63-179), one wave64 per 8x8 tile, RGBA8 straight to HBM.
//
// The semantics the shader leaves to the OpenGL driver are fixed in DESIGN.md
// section 4b (IEEE binary32 without contraction, correctly rounded / and
// sqrt, glibc acosf, GLSL-spec min/max/mod/step/smoothstep, GL_NEAREST /
// GL_NEAREST_MIPMAP_LINEAR sampling of the mipmapped REPEAT `ground`, unorm8
// framebuffer rounding) and this kernel is held to the CPU restatement
// (oracle/glsl_oracle.c) bit for bit.  Every expression keeps the shader's
// operand order.  Sphere data are wave-uniform (scalar loads); only the
// per-fragment lookups by drawSphere (:123-125, :154) are vector loads.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "glsl_trace.h"
#include "sfrt_device.h"
#include "sfrt_math.h"

#pragma clang fp contract(off)

namespace sfrt {
namespace {

// GLSL spec built-ins (min(x, y) = y < x ? y : x, ...), NaN behaviour included.
__device__ __forceinline__ float gmin(float x, float y) { return y < x ? y : x; }
__device__ __forceinline__ float gmax(float x, float y) { return x < y ? y : x; }
__device__ __forceinline__ float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }
// mod(x, y) = x - y * floor(x / y) (GLSL spec) is written out at its one use, :124-125.

__device__ __forceinline__ float len3(float x, float y, float z) {
  return sqrt_cr((x * x + y * y) + z * z);
}

// Nearest texel of one level with REPEAT wrap, channels / 255.
__device__ __forceinline__ void texel(const GlslFrame& f, int level, float s, float t, float& r,
                                      float& g, float& b) {
  const int w = f.mip_w[level], h = f.mip_h[level];
  const float fu = floorf(s * (float)w), fv = floorf(t * (float)h);
  const int i = fabsf(fu) < 16777216.0f ? ((int)fu & (w - 1)) : 0;  // w, h powers of two
  const int j = fabsf(fv) < 16777216.0f ? ((int)fv & (h - 1)) : 0;
  const uint32_t p = f.mip[f.mip_off[level] + j * w + i];
  r = div255((float)(p & 255u));  // == / 255.0f (sfrt_device.h)
  g = div255((float)((p >> 8) & 255u));
  b = div255((float)((p >> 16) & 255u));
}

__device__ __forceinline__ uint32_t unorm8(float v) {
  if (!(v > 0.0f)) return 0u;  // NaN too
  if (!(v < 1.0f)) return 255u;
  return (uint32_t)(int)floorf(v * 255.0f + 0.5f);
}

// The wall / ball / pair tables through the constant address space (the kernel never
// writes them): wave-uniform loads from it are scalar loads.
template <typename T>
using const_ptr = const __attribute__((address_space(4))) T*;
template <typename T>
__device__ __forceinline__ const_ptr<T> as_const(const T* p) {
  return (const_ptr<T>)p;
}
template <typename T>
__device__ __forceinline__ T ld(const_ptr<T> p, int i) {
  static_assert(sizeof(T) % 4 == 0, "dword records");
  const __attribute__((address_space(4))) uint32_t* q =
      (const __attribute__((address_space(4))) uint32_t*)(p + i);
  uint32_t w[sizeof(T) / 4];
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); k++) w[k] = q[k];
  T v;
  __builtin_memcpy(&v, w, sizeof(T));
  return v;
}

// The march's dominance-test bounds: RU(1.00001f * (1 + 6e-6)) and RU(1e-4f * (1 + 6e-6)); the
// host inflates r_skip by the same (1 + 6e-6), rounding up (sfrt_glsl.cpp).
constexpr float kThrMul = 0x1.00010ep+0f, kThrAdd = 0x1.a36ed4p-14f;

// The walls the wave's rays can meet (bit k: wall k; sc <= 64, all 64 lanes active).  Every
// position of the wall pass lies on its lane's ray campos + d t (t >= 0) up to the binary32 drift
// of its few moves, and a lane can be inside wall k only within r_k of its centre; so when the
// centre is farther than r_k + margin from every ray of the wave, `inside` is false for every
// lane at every visit of wall k, whose body the loop skips anyway, and leaving the wall out of the
// passes changes nothing.  The rays lie in a cone around the axis through the
// tile's first and last lanes' rays: its half-angle's sine is the wave's largest |d x a| plus
// slack.  The centre's distance from the cone's rays is |w| sin(alpha - theta) for alpha > theta
// (alpha the angle of w = c - campos from the axis), |w| when alpha - theta >= 90 degrees (the
// apex is nearest), 0 inside the cone.  A wave whose rays spread past 60 degrees keeps all walls.
// margin = f.wall_cull_margin (host: 1e-3 of the largest coordinate the pass can reach, + 1e-4),
// far above the positions' drift (at most 3 sc moves, each an add and a multiply rounding within
// 2^-24 of it: 2 * 3 * sc * 2^-24 < 2.3e-5 of it for sc <= 64) and this test's own rounding.
__device__ __forceinline__ uint64_t wall_mask(const GlslFrame& f, float dx, float dy, float dz) {
  const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  float ax = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dx), 0)) +
             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dx), 63));
  float ay = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dy), 0)) +
             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dy), 63));
  float az = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dz), 0)) +
             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dz), 63));
  const float al = __builtin_amdgcn_sqrtf((ax * ax + ay * ay) + az * az);
  if (!(al > 0.5f)) return ~0ull;  // the corner rays more than 120 degrees apart: no cull
  const float ia = __builtin_amdgcn_rcpf(al);  // (1 ulp: the margin dwarfs it)
  ax *= ia; ay *= ia; az *= ia;
  // the largest |d x a| over the wave (bit patterns of non-negative floats), and every ray within
  // 60 degrees of the axis (d . a >= 0.5)
  const float cx = dy * az - dz * ay, cy = dz * ax - dx * az, cz = dx * ay - dy * ax;
  const float s2 = (cx * cx + cy * cy) + cz * cz;
  const bool wide = (dx * ax + dy * ay) + dz * az < 0.5f;
  if (__builtin_amdgcn_ballot_w64(wide)) return ~0ull;
  const float sin_t = __builtin_amdgcn_sqrtf(__uint_as_float(wave_max_u32(__float_as_uint(s2)))) + 1e-5f;
  if (!(sin_t < 0.87f)) return ~0ull;
  const float cos_t = __builtin_amdgcn_sqrtf(1.0f - sin_t * sin_t);
  bool keep = true;
  if (lane < f.sc) {
    const GlslWall w = f.walls[lane];
    const float wx = w.x - f.campos[0], wy = w.y - f.campos[1], wz = w.z - f.campos[2];
    const float wl = __builtin_amdgcn_sqrtf((wx * wx + wy * wy) + wz * wz);
    const float reach = w.r + f.wall_cull_margin;
    if (wl >= reach) {  // else the camera is within reach of the wall: kept
      const float iw = __builtin_amdgcn_rcpf(wl);
      const float ca = ((wx * ax + wy * ay) + wz * az) * iw;                  // cos alpha
      const float qx = wy * az - wz * ay, qy = wz * ax - wx * az, qz = wx * ay - wy * ax;
      const float sa = __builtin_amdgcn_sqrtf((qx * qx + qy * qy) + qz * qz) * iw;  // sin alpha
      const float s_at = sa * cos_t - ca * sin_t;   // sin(alpha - theta)
      const float c_at = ca * cos_t + sa * sin_t;   // cos(alpha - theta)
      const float dist = s_at <= 0.0f ? 0.0f : (c_at <= 0.0f ? wl : wl * s_at);
      keep = dist < reach;
    }
  }
  return __builtin_amdgcn_ballot_w64(keep);
}

template <bool CULL>
__device__ __forceinline__ void fragment(const GlslFrame& f, const_ptr<GlslWall> walls,
                                         const_ptr<GlslBall> balls, int i, int row,
                                         uint32_t& work, bool store = true) {
  const float fx = (float)i + 0.5f;
  const float fy = (float)(f.height - 1 - row) + 0.5f;
  const float ax = -f.fov_x + f.hk * fx;                                   // :172-173
  const float ay = -f.fov_y + f.vk * fy;
  float dx = (f.fwd[0] + f.right[0] * ax) + f.up[0] * ay;                 // :175
  float dy = (f.fwd[1] + f.right[1] * ax) + f.up[1] * ay;
  float dz = (f.fwd[2] + f.right[2] * ax) + f.up[2] * ay;
  {
    const float l = len3(dx, dy, dz);                                     // :65
    const float a[3] = {dx, dy, dz};
    float q[3];
    div_shared(a, l, q);  // == dx / l, ... (one seed; sfrt_device.h)
    dx = q[0]; dy = q[1]; dz = q[2];
  }
  const float cx = f.campos[0], cy = f.campos[1], cz = f.campos[2];

  // ---- furthest wall: 3 passes over the walls (:71-85) ----
  float px = cx, py = cy, pz = cz;
  int draw = 0;
  float total = 0.0f;
  // Iterations before wall_start leave every lane at campos outside the wall
  // (host-checked with the same test), so they change nothing; a whole pass
  // in which no lane of the wave is inside a wall leaves the state at a fixed
  // point, so the remaining passes would repeat it and are skipped.
  // The passes as an outer loop and the walls as a counted inner loop (the record address
  // stepped, not recomputed): the single loop with its wrap-around index kept ~20 scalar
  // instructions per wall visit (tools/isa_block_profile.py).
  auto wall_visit = [&](int k, uint64_t& moved) {
    const GlslWall w = ld(walls, k);
    const float rx = px - w.x, ry = py - w.y, rz = pz - w.z;
    const float s = (rx * rx + ry * ry) + rz * rz;
    const bool inside = s <= w.s_in;                   // step(length(rpos), r) == 1
    const uint64_t inside_mask = __builtin_amdgcn_ballot_w64(inside);  // scalar tests only
    if ((inside_mask | (uint64_t)(uint32_t)f.cam_negzero) != 0) {
      moved |= inside_mask;
      const float cs = inside ? 1.0f : 0.0f;
      const float b = cs * 2.0f * ((rx * dx + ry * dy) + rz * dz);
      const float c = cs * s - w.rr;
      const float tosurf = cs * (-b + fabsf(sqrt_cr(b * b - 4.0f * c))) * 0.5f;
      px = px + dx * tosurf;
      py = py + dy * tosurf;
      pz = pz + dz * tosurf;
      total = total + tosurf;
    }
    draw = inside ? k : draw;
  };
  if (CULL && f.sc > 0 && f.sc <= 64 && f.wall_cull_margin > 0.0f) {
    // only the walls the wave's rays can meet, in index order (wall_mask above): at 4K each
    // 8x8 tile's rays meet 2.4 of the default scene's 10 walls
    const uint64_t wm = wall_mask(f, dx, dy, dz) & (f.sc == 64 ? ~0ull : ((1ull << f.sc) - 1ull));
    int k0 = f.wall_start % f.sc;
    for (int pass = f.wall_start / f.sc; pass < 3; pass++) {
      uint64_t moved = 0;
      uint64_t todo = wm & (~0ull << k0);
      while (todo) {
        const int k = (int)__builtin_ctzll(todo);
        todo &= todo - 1ull;
        wall_visit(k, moved);
      }
      k0 = 0;
      if (!moved) break;  // uniform: a pass in which no lane moved is a fixed point
    }
  } else if (f.sc > 0) {
    int k = f.wall_start % f.sc;
    for (int pass = f.wall_start / f.sc; pass < 3; pass++) {
      uint64_t moved = 0;
      for (; k < f.sc; k++) wall_visit(k, moved);
      k = 0;
      if (!moved) break;  // uniform: a pass in which no lane moved is a fixed point
    }
  }

  // ---- metaball march over lights + ospheres (:87-112) ----
  const int nballs = f.all - f.sc;
  float ball_dist = 0.0f;
  float smooth = 999999999.0f;
  int closest = 0;
  float snx = 0.0f, sny = 0.0f, snz = 0.0f;
  int steps = 0;
  // One way out of the march: the shader's loop test and our step cap as one condition at the
  // bottom (the cap's status after the loop): two divergent exits cost a lane mask merge each.
  // With the wall passes' loop split (above): 4K 455.8 -> 435.3 us (profiles/ab/r5_ab3).  The
  // ball records loaded one ball ahead (two register sets, an empty asm statement placing each
  // wait before the next issue) measured slower: 464.7 us (same A/B).
  if (ball_dist < total && smooth > 0.01f) {
    for (;;) {
      ++steps;
      const float tx = cx + dx * ball_dist, ty = cy + dy * ball_dist, tz = cz + dz * ball_dist;
      float shortest, thr;
      // The step's first ball runs its body for every lane (its dominance test compares with
      // (r_skip + 1e30)^2 = inf), from the step's start values, where polsmin's h is +0 once
      // |999999999 - other| >= 0.5: for a wave whose every lane has other <= 999999936 (the float
      // below 1e9) the body reduces to these assignments, the same bits: no test,
      // no start values, no polsmin for it (4K 399.2 -> 385.9 us, profiles/ab/r5_ab6).
      auto body = [&](const GlslBall& b, int k, float ox, float oy, float oz) {
        const float ss = (ox * ox + oy * oy) + oz * oz;  // the shader's length(), :100
        const float other = sqrt_cr(ss) - b.r;
        const float h = gmax(0.5f - fabsf(smooth - other), 0.0f) / 0.5f;  // polsmin(:57-61)
        smooth = gmin(smooth, other) - h * h * 0.5f * (1.0f / 4.0f);
        closest = other < shortest ? f.sc + k : closest;                  // :105
        shortest = gmin(shortest, other);
        const float nf = gclamp(other, 0.0f, 0.5f) * 2.0f;
        snx = nf * snx - (1.0f - nf) * ox;
        sny = nf * sny - (1.0f - nf) * oy;
        snz = nf * snz - (1.0f - nf) * oz;
        thr = fmaxf(fmaxf(smooth + 0.5f, shortest), 0.5f) * kThrMul + kThrAdd;
      };
      if (nballs > 0) {
        const GlslBall b = ld(balls, 0);
        const float ox = b.x - tx, oy = b.y - ty, oz = b.z - tz;
        const float ss = (ox * ox + oy * oy) + oz * oz;
        const float other = sqrt_cr(ss) - b.r;
        if (__builtin_amdgcn_ballot_w64(!(other <= 999999936.0f))) {
          smooth = 999999999.0f;  // the literal body from the start values
          closest = 0;
          shortest = 9999999.0f;
          snx = sny = snz = 0.0f;
          body(b, 0, ox, oy, oz);
        } else {
          smooth = other;  // gmin(999999999, other) - (+0)
          closest = other < 9999999.0f ? f.sc : 0;
          shortest = gmin(9999999.0f, other);
          const float nf = gclamp(other, 0.0f, 0.5f) * 2.0f;
          snx = 0.0f - (1.0f - nf) * ox;  // nf * (+0) - ...
          sny = 0.0f - (1.0f - nf) * oy;
          snz = 0.0f - (1.0f - nf) * oz;
          thr = fmaxf(fmaxf(smooth + 0.5f, shortest), 0.5f) * kThrMul + kThrAdd;
        }
      } else {
        smooth = 999999999.0f;
        closest = 0;
        shortest = 9999999.0f;
        snx = sny = snz = 0.0f;
        thr = 1e30f;
      }
      for (int k = 1; k < nballs; k++) {
        const GlslBall b = ld(balls, k);
        const float ox = b.x - tx, oy = b.y - ty, oz = b.z - tz;
        // Dominated ball: if otherDist >= max(smooth + 0.5, shortest, 0.5) (with
        // margin), polsmin returns smooth, closest/shortest keep their values and
        // normalFactor == 1, so the body changes nothing (smoothNormal at most
        // flips the sign of a zero component, which no output depends on).
        // The test is ours, not the shader's: the squared length by two fmas and both bounds
        // inflated by (1+6e-6) (r_skip on the host, thr here), which implies the round-3 test
        // ss >= (r + t*(1+1e-5) + 1e-4)^2 * (1+1e-5) on the shader's own ss.
        const float ssf = __builtin_fmaf(ox, ox, __builtin_fmaf(oy, oy, oz * oz));
        const float bnd = b.r_skip + thr;
        const bool dominated = ssf >= bnd * bnd;
        if (!__builtin_amdgcn_ballot_w64(!dominated)) continue;
        body(b, k, ox, oy, oz);
      }
      ball_dist += smooth + 0.01f;
      if (!((ball_dist < total) & (smooth > 0.01f) & (steps < kGlslMarchCap))) break;
    }
    if (steps == kGlslMarchCap && ball_dist < total && smooth > 0.01f) atomicOr(f.status, 1);
  }
  work = (uint32_t)steps;

  // ---- wall or ball (:114-120) ----
  const int wall = smooth < 0.01f ? 0 : 1;
  const float cw = (float)wall, cb = (float)(1 - wall);
  total = cw * total + cb * ball_dist;
  draw = wall ? draw : closest;
  px = cw * px + cb * (cx + dx * ball_dist);
  py = cw * py + cb * (cy + dy * ball_dist);
  pz = cw * pz + cb * (cz + dz * ball_dist);
  const float nsign = cw * -1.0f + cb;

  // ---- texture (:123-126) ----
  const GlslMat& m = f.mats[draw];
  const float rpx = snx * (1.0f - cw) + cw * (px - m.cx);
  const float rpy = sny * (1.0f - cw) + cw * (py - m.cy);
  const float rpz = snz * (1.0f - cw) + cw * (pz - m.cz);
  const float uv0 = m.uv[0];
  // mod(v, uv0) = v - uv0 * floor(v / uv0) for both coordinates: the two divisions by uv0
  // share a seed (div_shared), as do the lighting's divisions by tll and vl below
  float yq;
  {
    const float a[1] = {rpy};
    float q[1];
    div_shared(a, 0.8f + 0.2f * (fabsf(rpx) + fabsf(rpz)), q);
    yq = q[0];
  }
  const float xv = gmin(fabsf(rpz), fabsf(rpx));
  float mq[2];
  {
    const float a[2] = {yq, xv};
    div_shared(a, uv0, mq);
  }
  const float ycoord = (yq - uv0 * floorf(mq[0])) + m.uv[3];  // mod(yq, uv0) + uv.w
  const float xcoord = (xv - uv0 * floorf(mq[1])) + m.uv[2];
  const float lod = total * 0.05f;
  float cr, cg, cbl;
  const int q = f.mip_levels - 1;
  if (!(lod > 0.0f)) {
    texel(f, 0, xcoord, ycoord, cr, cg, cbl);
  } else if (lod >= (float)q) {
    texel(f, q, xcoord, ycoord, cr, cg, cbl);
  } else {
    const float fl = floorf(lod);
    const int d1 = (int)fl;
    const float fr = lod - fl;
    float r1, g1, b1, r2, g2, b2;
    texel(f, d1, xcoord, ycoord, r1, g1, b1);
    texel(f, d1 + 1, xcoord, ycoord, r2, g2, b2);
    cr = (1.0f - fr) * r1 + fr * r2;
    cg = (1.0f - fr) * g1 + fr * g2;
    cbl = (1.0f - fr) * b1 + fr * b2;
  }

  // ---- lighting (:128-151) ----
  float bright;
  {
    const float a[1] = {1.0f};
    float q[1];
    div_shared(a, gmax(total, 1.0f), q);
    bright = q[0];
  }
  const float lightc = ((float)draw < (float)f.sc ? 0.0f : 1.0f) *
                       ((float)(f.sc + f.lc - 1) < (float)draw ? 0.0f : 1.0f);
  const int nshadow = f.all - f.sc - f.lc;
  for (int li = 0; li < f.lc; li++) {
    const GlslBall L = ld(balls, li);
    const float tlx = L.x - px, tly = L.y - py, tlz = L.z - pz;
    const float tll = len3(tlx, tly, tlz);
    // tl / tll (:133) and 10 / tll / tll (:150): four divisions by tll on one seed
    float tq[4];
    {
      const float a[4] = {tlx, tly, tlz, 10.0f};
      div_shared(a, tll, tq);
    }
    const float tnx = tq[0], tny = tq[1], tnz = tq[2];
    const float vx = rpx * nsign, vy = rpy * nsign, vz = rpz * nsign;
    const float vl = len3(vx, vy, vz);
    float vq[3];
    {
      const float a[3] = {vx, vy, vz};
      div_shared(a, vl, vq);
    }
    const float nm = len3(vq[0] + tnx, vq[1] + tny, vq[2] + tnz) - 1.0f;
    float shadow = 1.0f;
    if (draw < f.sc + f.lc) {             // `drawSphere < j` holds for every j >= sc + lc
      const float t = gclamp((nm - 0.0f) / (0.5f - 0.0f), 0.0f, 1.0f);
      const float smooth_nm = t * t * (3.0f - 2.0f * t);                 // smoothstep(0, .5, nm)
      const bool near = total < 1000.0f;
      for (int k = 0; k < nshadow; k++) {
        const GlslPair P = ld(as_const(f.pairs), li * nshadow + k);
        const float cosang = (-tnx * P.ux + -tny * P.uy) + -tnz * P.uz;
        // Ball outside the light cone seen from pos: acos(cosang) >= sanglet
        // (with margin) makes the clamp's argument >= 1, factor 1 exactly.  Not below -1:
        // a rounded cosang of -1.0000001 (a ball straight behind pos from the light) makes
        // acos NaN and the shader's clamp passes NaN on (its brightness, then the pixel, 0).
        if (!__builtin_amdgcn_ballot_w64(!(near && cosang <= P.cos_lit && cosang >= -1.0f))) continue;
        float sangle = sfrt_math::acosf(cosang);
        const float psd = 1.5f / (0.8f + 0.2f * len3(px - P.bx, py - P.by, pz - P.bz));
        sangle = sangle * psd - (psd - 1.0f) * P.sanglet;
        const float st = tll < P.dist ? 0.0f : 1.0f;                      // step(dist, tll)
        shadow *= gclamp(sangle / P.sanglet + 1.0f - st * smooth_nm, 0.0f, 1.0f);
      }
    }
    float t2[1];  // (10 / tll) / tll
    {
      const float a[1] = {tq[3]};
      div_shared(a, tll, t2);
    }
    bright += t2[0] * gmax(0.5f + 0.5f * nm, 0.0f) * shadow;
  }

  // ---- colour (:153-158) ----
  bright = lightc * 2.0f + (1.0f - lightc) * bright;
  const float la = m.light[3];
  cr = la * m.light[0] * 0.5f + (1.0f - la) * cr;
  cg = la * m.light[1] * 0.5f + (1.0f - la) * cg;
  cbl = la * m.light[2] * 0.5f + (1.0f - la) * cbl;
  const float viewDist = 50.0f;
  const float fog = gclamp(bright, 0.0f, 3.0f) + gmin(-total + viewDist * 0.66f, 0.0f);
  cr *= fog;
  cg *= fog;
  cbl *= fog;
  if (store)
    f.out[(long long)(row - f.row0) * f.out_pitch + i] =
        unorm8(cr) | (unorm8(cg) << 8) | (unorm8(cbl) << 16) | (255u << 24);
}

// Wall and ball records are read once per visit by every wave with scalar loads
// (constant address space, above); staging them in LDS measured 5-10% slower
// (profiles/r1_glsl_variants.json), a next-record prefetch 7-8% slower (profiles/ab/r2_ab18).  Four 8x8 tiles (one per
// wave) per 256-thread workgroup, row-major.
__global__ __launch_bounds__(256) void k_glsl(GlslFrame f) {
  const int lane = threadIdx.x & 63;
  const int tile = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  const int tx = tile % f.tiles_x, ty = tile / f.tiles_x;
  const int i = tx * 8 + (lane & 7);
  const int r = ty * 8 + (lane >> 3);
  if (i >= f.width || r >= f.rows) return;
  uint32_t work = 0;
  fragment<false>(f, as_const(f.walls), as_const(f.balls), i, f.row0 + r, work);
}

// One 8x8 tile per one-wave workgroup in the adaptive tile order (sfrt_device.h
// sort_tiles; workgroup 0 is the sorter when prev_cost is set).  Edge lanes run
// no fragment but stay for the wave's reduction.
__global__ __launch_bounds__(64) void k_glsl_ordered(GlslFrame f, int ntiles) {
  const int lane = threadIdx.x & 63;
  int slot = (int)blockIdx.x;
  if (f.prev_cost) {
    if (slot == 0) {
      sort_tiles(f.prev_cost, ntiles, f.next_order);
      return;
    }
    slot -= 1;
  }
  uint32_t cls;  // the tile's class in the order (sfrt_device.h slot_tile)
  const int tile = slot_tile(f.tile_order, slot, ntiles, cls);
  const int tx = tile % f.tiles_x, ty = tile / f.tiles_x;
  const int i = tx * 8 + (lane & 7);
  const int r = ty * 8 + (lane >> 3);
  // Edge lanes shade a clamped duplicate pixel and store nothing: a divergent
  // branch around fragment() would cost its wave-uniform skips their uniformity.
  const bool in = i < f.width && r < f.rows;
  uint32_t work = 0;
  fragment<true>(f, as_const(f.walls), as_const(f.balls), i < f.width ? i : f.width - 1,
                  f.row0 + (r < f.rows ? r : f.rows - 1), work, in);
  if (f.tile_cost) {
    const uint32_t w = wave_max_u32(work);  // the tile's longest march
    if (lane == 0) store_cost(f.tile_cost, tile, tile_bucket(w), cls, f.cost_diff);
  }
}

}  // namespace

long long glsl_tile_key(const GlslFrame& f, long long* tiles) {
  *tiles = 0;
  if (f.tiles_x <= 0 || f.rows <= 0) return 0;
  const long long ty = (f.rows + 7) / 8;
  *tiles = (long long)f.tiles_x * ty;
  return (1ll << 62) | ((long long)f.tiles_x << 28) | ty;
}

int launch_glsl(const GlslFrame& f, void* stream, void* done_event) {
  const int tiles_y = (f.rows + 7) / 8;
  const long long tiles = (long long)f.tiles_x * tiles_y;
  if (tiles == 0) return 0;
  if (f.tile_cost) {  // adaptive tile order (the host linked this launch into its chain)
    if (tiles > 0x7ffffffeLL) return -1;
    hipExtLaunchKernelGGL(k_glsl_ordered, dim3((unsigned)(tiles + (f.prev_cost ? 1 : 0))), dim3(64), 0,
                          (hipStream_t)stream, nullptr, (hipEvent_t)done_event, 0, f, (int)tiles);
    return hipGetLastError() != hipSuccess;
  }
  hipExtLaunchKernelGGL(k_glsl, dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                        nullptr, (hipEvent_t)done_event, 0, f);
  return hipGetLastError() != hipSuccess;
}

}  // namespace sfrt
