// sphere_trace.hip -- gfx950 kernels for the sphere-cave trace-and-shade path.
//
// Replaces the per-pixel body of SphereWorld::UpdateImage / Raycast
// (/root/reference/Raytracing/SphereWorld.cpp:83-112, 355-382): one lane per
// pixel, one wave64 per 8x8 tile, RGBA8 written straight to HBM.
//
// Bit-exactness rules (see DESIGN.md "Exactness"):
//  * built with -ffp-contract=off; every float expression keeps the
//    reference's operand order; division and sqrt are the correctly rounded
//    gfx950 sequences (hipcc default);
//  * atan2f / asinf are sfrt_math:: restatements of the host libm;
//  * the sphere test `r - sqrtf(s) > 0.01f` is replaced by `s < s_pass`, where
//    s_pass is the exact binary32 threshold found on the host (the test is
//    monotone in s), so sqrtf runs only for spheres that pass;
//  * a sphere is skipped for a whole wave only when it provably cannot pass
//    for any ray of the tile (cone test with margins, below); the surviving
//    spheres are visited in their original order, so "last passing index"
//    (drawSphere, :368) and the max (:367) are unchanged.
#include <hip/hip_runtime.h>


#include "sfrt_device.h"
#include "sfrt_math.h"
#include "sfrt_trace.h"

#pragma clang fp contract(off)

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
  dx = x / len;
  dy = y / len;
  dz = z / len;
}

// Shading tail, SphereWorld.cpp:373-381.  Returns RGBA8 packed (r in byte 0).
__device__ __forceinline__ uint32_t shade(const FrameRec& f, const SphereRec& d, float px,
                                         float py, float pz, PixelDump* dump) {
  float ang = d.atan_c - atan2f_wave(pz, px);  // == sfrt_math::atan2f (sfrt_device.h)
  ang = ang > kPI ? ang - kPI2 : (ang < -kPI ? ang + kPI2 : ang);
  const float xcoord = sfrt_math::div_pi2_plus_1(ang);  // == ang / PI2 + 1.0f
  const float ex = px - d.cx, ey = py - d.cy, ez = pz - d.cz;
  const float ny = ey / sqrt_cr((ex * ex + ey * ey) + ez * ez);
  const float ycoord = sfrt_math::div_pi_plus_half(sfrt_math::asinf(ny));  // == asinf / PI + 0.5f
  const float bx = px - f.cam[0], by = py - f.cam[1], bz = pz - f.cam[2];
  const float bl = sqrt_cr((bx * bx + by * by) + bz * bz);
  const float brightness = 3.0f / (bl < 3.0f ? 3.0f : bl);
  // fmodf(v, 1.0f) == v - truncf(v) exactly for every binary32 v (NaN/inf -> NaN).
  // texsize of textures[0] (or of the sphere's extension slot), (float)(unsigned) as :376
  const uint32_t tw = d.tex_wh & 0xffffu, th = d.tex_wh >> 16;
  float u = xcoord * 4.0f * d.r;
  u = (u - __builtin_truncf(u)) * (float)tw;
  float w = ycoord * 2.0f * d.r;
  w = (w - __builtin_truncf(w)) * (float)th;
  // float -> unsigned: v_cvt_u32_f32 (NaN -> 0), as x86's cvttss2si for [0, 2^31).
  const uint32_t tx = __float2uint_rz(u), ty = __float2uint_rz(w);
  const uint32_t idx = tx + ty * tw;
  uint32_t texel = 0;
  if (idx < tw * th) {
    texel = f.tex[d.tex_off + idx];
  } else {
    atomicOr(f.status, 2);  // the reference would read outside the image here
  }
  const uint32_t r = __float2uint_rz((float)(texel & 0xffu) * brightness);
  const uint32_t g = __float2uint_rz((float)((texel >> 8) & 0xffu) * brightness);
  const uint32_t b = __float2uint_rz((float)((texel >> 16) & 0xffu) * brightness);
  const uint32_t rgba = (r & 0xffu) | ((g & 0xffu) << 8) | ((b & 0xffu) << 16) | (texel & 0xff000000u);
  if (dump) {
    dump->xcoord = xcoord;
    dump->ycoord = ycoord;
    dump->brightness = brightness;
    dump->texel[0] = tx;
    dump->texel[1] = ty;
    dump->rgba = rgba;
  }
  return rgba;
}

// Cone of the wave's rays: unit axis through the tile centre, and the sine
// and cosine of a half-angle that contains every lane's unit ray.  The sine
// is taken from |d x a| (accurate for the small angles of a tile, unlike a
// cosine near 1), maximised over the wave, plus slack for binary32 rounding.
// A tile whose rays spread past ~60 degrees (strided subsets) gets wide = true
// and is not culled.
struct Cone {
  float ax, ay, az, cos_t, sin_t;
  bool wide;
};

__device__ __forceinline__ Cone tile_cone(const FrameRec& f, int tile_x, int tile_y, float dx,
                                          float dy, float dz) {
  const float ic = (float)f.xstart + ((float)(tile_x * kTile) + 3.5f) * (float)f.xadd;
  const float jc = (float)f.ystart +
                   ((float)(f.sub_row0 + tile_y * kTile) + 3.5f) * (float)f.yadd;
  const float h = f.h_start + f.h_inc * ic;
  const float v = f.v_start + jc * f.v_inc;
  float ax = (f.fwd[0] + f.right[0] * h) + f.up[0] * v;
  float ay = (f.fwd[1] + f.right[1] * h) + f.up[1] * v;
  float az = (f.fwd[2] + f.right[2] * h) + f.up[2] * v;
  const float inv = __builtin_amdgcn_rsqf((ax * ax + ay * ay) + az * az);
  ax *= inv; ay *= inv; az *= inv;
  const float cx = dy * az - dz * ay, cy = dz * ax - dx * az, cz = dx * ay - dy * ax;
  const float sin_l = __builtin_sqrtf((cx * cx + cy * cy) + cz * cz);
  const float cos_l = (dx * ax + dy * ay) + dz * az;
  Cone c;
  c.ax = ax; c.ay = ay; c.az = az;
  // sin_l >= +0 (inputs finite, sfrt_world.cpp): max over the bit patterns
  c.sin_t = fminf(1.0f, __uint_as_float(wave_max_u32(__float_as_uint(sin_l))) + 1e-5f);
  c.cos_t = __builtin_sqrtf(fmaxf(0.0f, 1.0f - c.sin_t * c.sin_t));
  c.wide = __builtin_amdgcn_ballot_w64(cos_l < 0.5f) != 0;  // min over lanes < 0.5
  return c;
}

// Wave-level cull ("wavefront ballot"): bit (k - base) of the result is set
// when sphere k may pass the march test for some ray of this wave's tile.
// Lane l tests sphere base + l against the cone.  A sphere is dropped only
// when its distance to the cone exceeds its radius inflated by
// f.cull_margin, which bounds how far the binary32 march positions can drift
// from their rays (sfrt_world.cpp) -- there r - |p - c| > 0.01f cannot hold.
// The distance from a centre at axial coordinate t and radial distance perp
// to the cone's side line is perp * cos_t - t * sin_t; it is the distance to
// the cone where the centre projects onto the side, and a lower bound of it
// everywhere (behind the apex the distance is |w|).  Evaluating it in
// binary32 errs by < 1e-6 |w|, covered by the 4e-6 |w| slack.  Spheres whose pass threshold is 0 never
// pass and are dropped.
__device__ __forceinline__ uint64_t cull_mask(const FrameRec& f, const SphereRec* __restrict__ sph,
                                              int base, const Cone& c) {
  const int k = base + (int)(threadIdx.x & 63);
  bool inc = false;
  if (k < f.n) {
    const SphereRec s = sph[k];
    if (s.s_pass > 0.0f) {
      const float wx = s.cx - f.cam[0], wy = s.cy - f.cam[1], wz = s.cz - f.cam[2];
      const float wl = __builtin_sqrtf((wx * wx + wy * wy) + wz * wz);
      const float rr = s.r + f.cull_margin + 4e-6f * wl;
      const float t = (wx * c.ax + wy * c.ay) + wz * c.az;
      const float px = wx - t * c.ax, py = wy - t * c.ay, pz = wz - t * c.az;
      const float perp = __builtin_sqrtf((px * px + py * py) + pz * pz);
      // side distance, used where the centre projects onto the side (or
      // within rr of that region: there it is still a lower bound)
      const bool side = t * c.cos_t + perp * c.sin_t >= -rr;
      inc = c.wide || wl <= rr || (side && perp * c.cos_t - t * c.sin_t <= rr);
    }
  }
  return __builtin_amdgcn_ballot_w64(inc);
}

// Cull plus march window.  As cull_mask; in addition lane l returns, for
// sphere base + l, an interval (lo, hi) of along-ray distance outside which
// the sphere cannot pass for any ray of the cone.  A ray's march position p
// at along-ray distance tau lies within the drift bound of the ray's point
// cam + u*tau (cull_margin), and |cam + u*tau - c| >= |tau - dot(c - cam, u)|,
// so a pass needs |tau - dot(w, u)| < r + drift.  Over the cone's rays
// dot(w, u) = |w| cos(angle(w, u)) with the angle in
// [max(0, alpha - theta), min(pi, alpha + theta)] (alpha = angle(w, axis),
// theta = half-angle): |w| cos(alpha -+ theta) = t cos_t +- perp sin_t,
// clamped to +-|w| where alpha - theta < 0 or alpha + theta > pi.  The
// interval is widened by r + 2 * cull_margin: the drift, the binary32 error
// of the lanes' accumulated distance (<= 1.3e-4 R over kCullSafeIterations
// steps) and of these expressions all fit in the second margin.
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
      const float wl = __builtin_sqrtf((wx * wx + wy * wy) + wz * wz);
      const float rr = s.r + f.cull_margin + 4e-6f * wl;
      const float t = (wx * c.ax + wy * c.ay) + wz * c.az;
      const float px = wx - t * c.ax, py = wy - t * c.ay, pz = wz - t * c.az;
      const float perp = __builtin_sqrtf((px * px + py * py) + pz * pz);
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
          const float ext = rr + f.cull_margin;
          lo = dn - ext;
          hi = up + ext;
        }
      }
    }
  }
  return __builtin_amdgcn_ballot_w64(inc);
}

// std::max(largestDist, t) (SphereWorld.cpp:367) for L >= +0 and t > 0.01f
// (the pass test), both finite: their bit patterns order like the values, so
// one v_max_u32 gives the compare-select's bits (v_max_f32 would first
// canonicalise the loop-carried L).
__device__ __forceinline__ float max_nonneg(float L, float t) {
  return __uint_as_float(__builtin_elementwise_max(__float_as_uint(L), __float_as_uint(t)));
}

// Pass body of a sphere test (SphereWorld.cpp:366-368) for the lanes in
// `pass`: t = r - sqrtf(ss) exactly; largestDist = max; drawSphere = k.
__device__ __forceinline__ void pass_body(bool pass, float ss, float r, int k, float& L,
                                          int& dnew) {
  // Scalar branch around the sqrt: most culled spheres pass for no lane of
  // the wave in a given step, and then the whole body is skipped (the
  // compiler would otherwise if-convert it and run the sqrt every time).
  // sqrt_cr_normal also serves ss < 2^-96: see pass_body_r (NOTINY).
  if (__builtin_amdgcn_ballot_w64(pass)) {
    __asm__ volatile("; sphere passes for some lane");  // keeps the branch (no if-conversion)
    if (pass) {
      const float t = r - sqrt_cr_normal(ss);
      L = max_nonneg(L, t);
      dnew = k;
    }
  }
}

// One sphere test of the march (SphereWorld.cpp:365-369), exact: the pass
// test is s < s_pass (see sfrt_world.cpp, pass_threshold) and sqrtf runs only
// for a sphere that passes.
__device__ __forceinline__ float dist2(float px, float py, float pz, float cx, float cy,
                                       float cz) {
  const float ex = px - cx, ey = py - cy, ez = pz - cz;
  return (ex * ex + ey * ey) + ez * ez;
}

__device__ __forceinline__ void sphere_step(float px, float py, float pz, float cx, float cy,
                                            float cz, float r, float s_pass, int k, float& L,
                                            int& dnew) {
  const float ss = dist2(px, py, pz, cx, cy, cz);
  pass_body(ss < s_pass, ss, r, k, L, dnew);
}

template <bool INLINE, int SLOTS>
__device__ __forceinline__ void trace_tile(const FrameRec& f, const SphereRec* __restrict__ sph,
                                           const SphereRec* __restrict__ rest_sph) {
  __shared__ uint64_t s_mask[kWavesPerBlock][kMaskWords];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tile = blockIdx.x * kWavesPerBlock + wave;
  const int tile_y = tile / f.tiles_x;
  const int tile_x = tile - tile_y * f.tiles_x;
  if (tile_y * kTile >= f.sub_rows) return;  // grid rounding; uniform per wave
  const int a = tile_x * kTile + (lane & 7);
  const int b = f.sub_row0 + tile_y * kTile + (lane >> 3);
  const int b_end = f.sub_row0 + f.sub_rows;
  const bool valid = a < f.sub_w && b < b_end;
  // Lanes past the frame edge trace a clamped duplicate pixel (never stored)
  // so that the tile cone stays tight.
  const int ac = a < f.sub_w ? a : f.sub_w - 1;
  const int bc = b < b_end ? b : b_end - 1;
  const int i = f.xstart + ac * f.xadd;
  const int j = f.ystart + bc * f.yadd;

  float dx, dy, dz;
  primary_dir(f, i, j, dx, dy, dz);

  const float l0 = f.first_l;
  float px = f.cam[0] + dx * l0;
  float py = f.cam[1] + dy * l0;
  float pz = f.cam[2] + dz * l0;
  int draw = f.first_draw;
  // March state as a float: the lane's last step length (> 0 while it marches;
  // 0 once it stopped or for lanes that never march).  `mv > 0` is one compare
  // per step, where a loop-carried bool is rematerialised through VGPRs.
  float mv = (valid && l0 > 0.0f) ? 1.0f : 0.0f;

  // ---- per-wave sphere cull (the "wavefront ballot") ----
  const int nwords = (f.n + 63) >> 6;
  const bool any_march = __builtin_amdgcn_ballot_w64(mv > 0.0f) != 0;
  Cone cone{};
  if (f.cull && any_march) cone = tile_cone(f, tile_x, tile_y, dx, dy, dz);
  auto word_mask = [&](int w) -> uint64_t {
    if (f.cull && any_march) return cull_mask(f, sph, w * 64, cone);
    const int rem = f.n - w * 64;
    return rem >= 64 ? ~0ull : ((1ull << rem) - 1ull);
  };

  if (INLINE) {
    // ---- march with the culled spheres in SGPR slots ----
    uint64_t m = any_march ? word_mask(0) : 0ull;
    float scx[SLOTS + 1], scy[SLOTS + 1], scz[SLOTS + 1], sr[SLOTS + 1], ssp[SLOTS + 1];
    int sk[SLOTS + 1];
#pragma unroll
    for (int q = 0; q < SLOTS; q++) {
      scx[q] = scy[q] = scz[q] = sr[q] = ssp[q] = 0.0f;
      sk[q] = 0;
      if (m) {
        const int k = __builtin_ctzll(m);
        m &= m - 1;
        scx[q] = sph[k].cx; scy[q] = sph[k].cy; scz[q] = sph[k].cz;
        sr[q] = sph[k].r; ssp[q] = sph[k].s_pass;
        sk[q] = k;
      }
    }
    uint64_t rest = m;  // culled spheres beyond the slots (higher indices)
    int trips = 1;
    while (__builtin_amdgcn_ballot_w64(mv > 0.0f)) {
      if (trips == kCullSafeIterations) {  // uniform: leave culling behind, visit all
#pragma unroll
        for (int q = 0; q < SLOTS; q++) ssp[q] = 0.0f;  // slots never pass again
        rest = f.n >= 64 ? ~0ull : ((1ull << f.n) - 1ull);
      }
      float L = 0.0f;
      int dnew = draw;
      // Empty slots hold s_pass = 0 and never pass, so every slot is tested
      // unconditionally: SLOTS independent dependency chains the scheduler
      // can interleave, then the branches in index order.
      float ssq[SLOTS + 1];
#pragma unroll
      for (int q = 0; q < SLOTS; q++) ssq[q] = dist2(px, py, pz, scx[q], scy[q], scz[q]);
#pragma unroll
      for (int q = 0; q < SLOTS; q++) pass_body(ssq[q] < ssp[q], ssq[q], sr[q], sk[q], L, dnew);
      for (uint64_t mm = rest; mm; mm &= mm - 1) {
        const int k = __builtin_ctzll(mm);
        const SphereRec& s = rest_sph[k];
        sphere_step(px, py, pz, s.cx, s.cy, s.cz, s.r, s.s_pass, k, L, dnew);
      }
      if (mv > 0.0f) {
        px = px + dx * L;
        py = py + dy * L;
        pz = pz + dz * L;
        draw = dnew;
        mv = L;  // L >= 0: max(0, r - d) over passing spheres
      }
      if (++trips >= kMaxIterations) {
        if (mv > 0.0f) atomicOr(f.status, 1);
        break;
      }
    }
  } else {
    if (any_march) {
      for (int w = 0; w < nwords; w++) {
        const uint64_t m = word_mask(w);
        if (lane == 0) s_mask[wave][w] = m;
      }
    }
    __builtin_amdgcn_wave_barrier();
    int trips = 1;
    bool full = !(f.cull && any_march);
    while (__builtin_amdgcn_ballot_w64(mv > 0.0f)) {
      if (trips == kCullSafeIterations) full = true;
      float L = 0.0f;
      int dnew = draw;
      for (int w = 0; w < nwords; w++) {
        uint64_t m;
        if (full) {
          const int rem = f.n - w * 64;
          m = rem >= 64 ? ~0ull : ((1ull << rem) - 1ull);
        } else {
          m = uniform_u64(s_mask[wave][w]);
        }
        for (; m; m &= m - 1) {
          const int k = w * 64 + __builtin_ctzll(m);
          const SphereRec& s = sph[k];
          sphere_step(px, py, pz, s.cx, s.cy, s.cz, s.r, s.s_pass, k, L, dnew);
        }
      }
      if (mv > 0.0f) {
        px = px + dx * L;
        py = py + dy * L;
        pz = pz + dz * L;
        draw = dnew;
        mv = L;  // L >= 0: max(0, r - d) over passing spheres
      }
      if (++trips >= kMaxIterations) {
        if (mv > 0.0f) atomicOr(f.status, 1);
        break;
      }
    }
  }
  if (!valid) return;
  const SphereRec d = sph[draw];
  const uint32_t rgba = shade(f, d, px, py, pz, nullptr);
  f.out[(long long)(b - f.sub_row0) * f.out_pitch + a] = rgba;
}

// n <= 64 with the march window: each step visits only the culled spheres
// whose (lo, hi) interval meets the along-ray distances of the wave's
// marching lanes, [min over marching lanes, max over all lanes] of tacc.
// Lanes only move forward, so a sphere left behind by every marching lane is
// never needed again and one not yet reached is not needed yet.
template <int SLOTS, int WPB, int TLO_EVERY = 1>
__device__ __forceinline__ void trace_tile_window(const FrameRec& f,
                                                  const SphereRec* __restrict__ sph) {
  const int lane = threadIdx.x & 63;
  const int wave = WPB == 1 ? 0 : (int)(threadIdx.x >> 6);
  const int tile = blockIdx.x * WPB + wave;
  const int tile_y = tile / f.tiles_x;
  const int tile_x = tile - tile_y * f.tiles_x;
  if (tile_y * kTile >= f.sub_rows) return;  // grid rounding; uniform per wave
  const int a = tile_x * kTile + (lane & 7);
  const int b = f.sub_row0 + tile_y * kTile + (lane >> 3);
  const int b_end = f.sub_row0 + f.sub_rows;
  const bool valid = a < f.sub_w && b < b_end;
  const int ac = a < f.sub_w ? a : f.sub_w - 1;
  const int bc = b < b_end ? b : b_end - 1;
  const int i = f.xstart + ac * f.xadd;
  const int j = f.ystart + bc * f.yadd;

  float dx, dy, dz;
  primary_dir(f, i, j, dx, dy, dz);

  const float l0 = f.first_l;
  float px = f.cam[0] + dx * l0;
  float py = f.cam[1] + dy * l0;
  float pz = f.cam[2] + dz * l0;
  int draw = f.first_draw;
  float mv = (valid && l0 > 0.0f) ? 1.0f : 0.0f;
  float tacc = l0;  // along-ray distance marched (binary32 sum of the steps)

  const uint64_t all = f.n >= 64 ? ~0ull : ((1ull << f.n) - 1ull);
  const bool any_march = __builtin_amdgcn_ballot_w64(mv > 0.0f) != 0;
  const bool windowed = f.cull && any_march;
  uint64_t m = all;
  float lo = -__builtin_inff(), hi = __builtin_inff();
  if (windowed) {
    const Cone cone = tile_cone(f, tile_x, tile_y, dx, dy, dz);
    m = cull_window(f, sph, 0, cone, lo, hi);
  }
  int trips = 1;
  if (SLOTS > 0 && windowed && __builtin_popcountll(m) <= SLOTS) {
    // Few culled spheres: hold them in SGPR slots and test every one each
    // step (cheaper than maintaining the window).
    constexpr int NS = SLOTS > 0 ? SLOTS : 1;
    float scx[NS], scy[NS], scz[NS], sr[NS], ssp[NS];
    int sk[NS];
    uint64_t mm = m;
#pragma unroll
    for (int q = 0; q < SLOTS; q++) {
      scx[q] = scy[q] = scz[q] = sr[q] = ssp[q] = 0.0f;
      sk[q] = 0;
      if (mm) {
        const int k = __builtin_ctzll(mm);
        mm &= mm - 1;
        scx[q] = sph[k].cx; scy[q] = sph[k].cy; scz[q] = sph[k].cz;
        sr[q] = sph[k].r; ssp[q] = sph[k].s_pass;
        sk[q] = k;
      }
    }
    uint64_t rest = 0;
    while (__builtin_amdgcn_ballot_w64(mv > 0.0f)) {
      if (trips == kCullSafeIterations) {  // uniform: leave culling behind, visit all
#pragma unroll
        for (int q = 0; q < SLOTS; q++) ssp[q] = 0.0f;
        rest = all;
      }
      float L = 0.0f;
      int dnew = draw;
      float ssq[NS];
#pragma unroll
      for (int q = 0; q < SLOTS; q++) ssq[q] = dist2(px, py, pz, scx[q], scy[q], scz[q]);
#pragma unroll
      for (int q = 0; q < SLOTS; q++) pass_body(ssq[q] < ssp[q], ssq[q], sr[q], sk[q], L, dnew);
      for (uint64_t r2 = rest; r2; r2 &= r2 - 1) {
        const int k = __builtin_ctzll(r2);
        const SphereRec& s = sph[k];
        sphere_step(px, py, pz, s.cx, s.cy, s.cz, s.r, s.s_pass, k, L, dnew);
      }
      if (mv > 0.0f) {
        px = px + dx * L;
        py = py + dy * L;
        pz = pz + dz * L;
        draw = dnew;
        mv = L;
      }
      if (++trips >= kMaxIterations) {
        if (mv > 0.0f) atomicOr(f.status, 1);
        break;
      }
    }
  } else {
    bool full = !windowed;
    float tlo = 0.0f;
    while (__builtin_amdgcn_ballot_w64(mv > 0.0f)) {
      if (trips == kCullSafeIterations) full = true;  // uniform: visit all from here on
      uint64_t win = all;
      if (!full) {
        // tacc >= +0: reduce the bit patterns (wave_min_u32 / wave_max_u32).  The
        // low end only rises, so an earlier value is a valid lower bound
        // (refreshed every TLO_EVERY steps, as trace_tile_window_r).
        if (TLO_EVERY == 1 || trips % TLO_EVERY == 1)
          tlo = __uint_as_float(wave_min_u32(__float_as_uint(mv > 0.0f ? tacc : __builtin_inff())));
        const float thi = __uint_as_float(wave_max_u32(__float_as_uint(tacc)));
        win = m & __builtin_amdgcn_ballot_w64(lo < thi) & __builtin_amdgcn_ballot_w64(hi > tlo);
      }
      float L = 0.0f;
      int dnew = draw;
      for (uint64_t mm = win; mm; mm &= mm - 1) {
        const int k = __builtin_ctzll(mm);
        const SphereRec& s = sph[k];
        sphere_step(px, py, pz, s.cx, s.cy, s.cz, s.r, s.s_pass, k, L, dnew);
      }
      if (mv > 0.0f) {
        px = px + dx * L;
        py = py + dy * L;
        pz = pz + dz * L;
        draw = dnew;
        mv = L;
        tacc = tacc + L;
      }
      if (++trips >= kMaxIterations) {
        if (mv > 0.0f) atomicOr(f.status, 1);
        break;
      }
    }
  }
  if (!valid) return;
  const SphereRec d = sph[draw];
  const uint32_t rgba = shade(f, d, px, py, pz, nullptr);
  f.out[(long long)(b - f.sub_row0) * f.out_pitch + a] = rgba;
}

// R pixels per lane (an (8R)x8 tile per wave: columns c, c + 8, ...): the
// wave-uniform work of a sphere visit -- record load, window bits, branch --
// is shared by R rays, and each lane carries R independent dependency chains.
// Same exact march as trace_tile_window, per ray.
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
    sin_l = fmaxf(sin_l, __builtin_sqrtf((cx * cx + cy * cy) + cz * cz));
    wide = wide || ((dx[r] * ax + dy[r] * ay) + dz[r] * az) < 0.5f;
  }
  Cone c;
  c.ax = ax; c.ay = ay; c.az = az;
  c.sin_t = fminf(1.0f, __uint_as_float(wave_max_u32(__float_as_uint(sin_l))) + 1e-5f);
  c.cos_t = __builtin_sqrtf(fmaxf(0.0f, 1.0f - c.sin_t * c.sin_t));
  c.wide = __builtin_amdgcn_ballot_w64(wide) != 0;
  return c;
}

// Pass bodies of one sphere for the lane's R rays under one scalar branch.
// (Lane-masked selects through inline asm instead of these exec-masked
// updates were measured slower: 1% at R = 2, 15% at R = 1.)
// NOTINY: sqrt_cr_normal for every passing lane.  Exact also for ss < 2^-96,
// where sqrt_cr_normal is not the correctly rounded sqrt: a pass needs
// rad - sqrtf(ss) > 0.01f, so rad > 2^-7, and rad - q == rad for any q < 2^-33,
// which both roots of such ss are (tests/native/wave_check.hip, every ss).
template <int R, bool NOTINY = false>
__device__ __forceinline__ void pass_body_r(const float (&ss)[R], float s_pass, float rad, int k,
                                            float (&L)[R], int (&dnew)[R]) {
  uint64_t pm[R], any = 0;
#pragma unroll
  for (int r = 0; r < R; r++) {
    pm[r] = __builtin_amdgcn_ballot_w64(ss[r] < s_pass);
    any |= pm[r];
  }
  if (NOTINY) {
    if (any) {
      __asm__ volatile("; sphere passes for some ray of the wave");
#pragma unroll
      for (int r = 0; r < R; r++) {
        if (ss[r] < s_pass) {
          const float t = rad - sqrt_cr_normal(ss[r]);
          L[r] = max_nonneg(L[r], t);
          dnew[r] = k;
        }
      }
    }
    return;
  }
  if (any) {
    __asm__ volatile("; sphere passes for some ray of the wave");
    uint64_t tiny = 0;
#pragma unroll
    for (int r = 0; r < R; r++) tiny |= __builtin_amdgcn_ballot_w64(ss[r] < kTinySqrtArg) & pm[r];
    if (tiny == 0) {
#pragma unroll
      for (int r = 0; r < R; r++) {
        if (ss[r] < s_pass) {
          const float t = rad - sqrt_cr_normal(ss[r]);
          L[r] = max_nonneg(L[r], t);
          dnew[r] = k;
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; r++) {
        if (ss[r] < s_pass) {
          const float t = rad - __builtin_sqrtf(ss[r]);
          L[r] = max_nonneg(L[r], t);
          dnew[r] = k;
        }
      }
    }
  }
}

// FL (A/B flags): kFlMask -- marching masks from a plain f32 compare; kFlFree --
// the advance runs on every lane (exact, see below) and edge lanes march as the
// duplicates they are; kFlPrefetch -- the next visited record is loaded before
// the current visit's arithmetic.
// kFlPair -- visits taken two at a time: both records loaded, both spheres'
// distances computed (four independent chains per lane), then the two pass
// bodies in index order.
// kFlNoShade (timing probe only, wrong bytes): store a hash of the march result
// instead of shading it, to split the kernel time between march and shading.
// kFlNoTiny -- no tiny-argument sqrt branch in the pass body (pass_body_r).
// kFlBits -- the visit loop clears each visited bit with s_bitset0_b64.
constexpr int kFlMask = 1, kFlFree = 2, kFlPrefetch = 4, kFlPair = 8, kFlNoShade = 32,
              kFlNoTiny = 64, kFlBits = 128;
// kFlVisitCost -- the tile-order cost is the wave's sphere visits (slots + window
// bits, summed in SALU), not its march steps.
constexpr int kFlVisitCost = 256;
constexpr int kFlDefault = kFlMask | kFlFree | kFlNoTiny;

template <int SLOTS, int R, int WPB, int TLO_EVERY = 1, int FL = 0>
__device__ __forceinline__ void trace_tile_window_r(const FrameRec& f,
                                                    const SphereRec* __restrict__ sph) {
  const int lane = threadIdx.x & 63;
  const int wave = WPB == 1 ? 0 : (int)(threadIdx.x >> 6);
  // Adaptive tile order (sfrt_trace.h FrameRec): workgroup 0 may be the sorter.
  const int ntiles = f.tiles_x * ((f.sub_rows + kTile - 1) / kTile);
  int slot = (int)blockIdx.x;
  if (WPB == 1 && f.prev_cost) {
    if (blockIdx.x == 0) {
      sort_tiles(f.prev_cost, ntiles, f.next_order);
      return;
    }
    slot -= 1;
  }
  int tile = slot * WPB + wave;
  if (WPB == 1 && f.tile_order) {
    const int t = (int)f.tile_order[slot];
    tile = t < ntiles ? t : slot;  // never outside the grid
  }
  const int tile_y = tile / f.tiles_x;  // f.tiles_x = ceil(sub_w / (8 R)) for this kernel
  const int tile_x = tile - tile_y * f.tiles_x;
  if (tile_y * kTile >= f.sub_rows) return;  // grid rounding; uniform per wave
  const int b = f.sub_row0 + tile_y * kTile + (lane >> 3);
  const int b_end = f.sub_row0 + f.sub_rows;
  const int bc = b < b_end ? b : b_end - 1;
  const int j = f.ystart + bc * f.yadd;
  const float l0 = f.first_l;
  int a[R], draw[R];
  bool valid[R];
  float dx[R], dy[R], dz[R], px[R], py[R], pz[R], mv[R], tacc[R];
  bool marching = false;
#pragma unroll
  for (int r = 0; r < R; r++) {
    a[r] = tile_x * R * kTile + r * kTile + (lane & 7);
    valid[r] = a[r] < f.sub_w && b < b_end;
    const int ac = a[r] < f.sub_w ? a[r] : f.sub_w - 1;
    primary_dir(f, f.xstart + ac * f.xadd, j, dx[r], dy[r], dz[r]);
    px[r] = f.cam[0] + dx[r] * l0;
    py[r] = f.cam[1] + dy[r] * l0;
    pz[r] = f.cam[2] + dz[r] * l0;
    draw[r] = f.first_draw;
    mv[r] = ((FL & kFlFree) || valid[r]) && l0 > 0.0f ? 1.0f : 0.0f;
    tacc[r] = l0;
    marching = marching || mv[r] > 0.0f;
  }
  // mv >= +0 always (0, or the last step length), so "marching" is mv's bits != 0:
  // an integer compare straight into a lane mask
  auto marching_mask = [&](int r) {
    if (FL & kFlMask) return __builtin_amdgcn_ballot_w64(mv[r] > 0.0f);
    return __builtin_amdgcn_ballot_w64(__float_as_uint(mv[r]) != 0u);
  };
  auto any_marching = [&]() {
    uint64_t q = 0;
#pragma unroll
    for (int r = 0; r < R; r++) q |= marching_mask(r);
    return q != 0;
  };
  const uint64_t all = f.n >= 64 ? ~0ull : ((1ull << f.n) - 1ull);
  const bool windowed = f.cull && __builtin_amdgcn_ballot_w64(marching) != 0;
  uint64_t m = all;
  float lo = -__builtin_inff(), hi = __builtin_inff();
  if (windowed) {
    const Cone cone = tile_cone_r<R>(f, tile_x, tile_y, dx, dy, dz);
    m = cull_window(f, sph, 0, cone, lo, hi);
  }

  // pos += dir * L for marching rays (SphereWorld.cpp:371).  kFlFree: on every
  // lane.  A ray that stopped had no passing sphere at its position (its last
  // step visited every sphere that could pass), its position no longer moves,
  // so each later step again has none: L = +0, dnew = draw, tacc + 0 = tacc,
  // and p + d * (+0) = p -- also for p = -0, which a marching wave's ray only
  // reaches through -0 + d * l0 with d of negative sign, so d * (+0) = -0.
  auto advance = [&](const float (&L)[R], const int (&dnew)[R]) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      if ((FL & kFlFree) || mv[r] > 0.0f) {
        px[r] = px[r] + dx[r] * L[r];
        py[r] = py[r] + dy[r] * L[r];
        pz[r] = pz[r] + dz[r] * L[r];
        draw[r] = dnew[r];
        mv[r] = L[r];
        tacc[r] = tacc[r] + L[r];
      }
    }
  };
  auto visit = [&](float cx, float cy, float cz, float rad, float s_pass, int k, float (&L)[R],
                   int (&dnew)[R]) {
    float ss[R];
#pragma unroll
    for (int r = 0; r < R; r++) ss[r] = dist2(px[r], py[r], pz[r], cx, cy, cz);
    pass_body_r<R, (FL & kFlNoTiny) != 0>(ss, s_pass, rad, k, L, dnew);
  };
  int trips = 1;
  uint32_t visits = 0;  // kFlVisitCost: wave-uniform (SGPR) sum of the sphere visits
  if (SLOTS > 0 && windowed && __builtin_popcountll(m) <= SLOTS) {
    constexpr int NS = SLOTS > 0 ? SLOTS : 1;
    float scx[NS], scy[NS], scz[NS], sr[NS], ssp[NS];
    int sk[NS];
    uint64_t mm = m;
#pragma unroll
    for (int q = 0; q < SLOTS; q++) {
      scx[q] = scy[q] = scz[q] = sr[q] = ssp[q] = 0.0f;
      sk[q] = 0;
      if (mm) {
        const int k = __builtin_ctzll(mm);
        mm &= mm - 1;
        scx[q] = sph[k].cx; scy[q] = sph[k].cy; scz[q] = sph[k].cz;
        sr[q] = sph[k].r; ssp[q] = sph[k].s_pass;
        sk[q] = k;
      }
    }
    uint64_t rest = 0;
    // single-exit loop (the march guard is part of the condition): a second
    // exit makes the compiler shuffle every loop-carried register each step
    for (; any_marching() && trips < kMaxIterations; ++trips) {
      if (trips == kCullSafeIterations) {
#pragma unroll
        for (int q = 0; q < SLOTS; q++) ssp[q] = 0.0f;
        rest = all;
      }
      float L[R];
      int dnew[R];
#pragma unroll
      for (int r = 0; r < R; r++) { L[r] = 0.0f; dnew[r] = draw[r]; }
#pragma unroll
      for (int q = 0; q < SLOTS; q++) visit(scx[q], scy[q], scz[q], sr[q], ssp[q], sk[q], L, dnew);
      for (uint64_t r2 = rest; r2; r2 &= r2 - 1) {
        const int k = __builtin_ctzll(r2);
        const SphereRec& s = sph[k];
        visit(s.cx, s.cy, s.cz, s.r, s.s_pass, k, L, dnew);
      }
      if (FL & kFlVisitCost) visits += (uint32_t)SLOTS + (uint32_t)__builtin_popcountll(rest);
      advance(L, dnew);
    }
  } else {
    bool full = !windowed;
    float tlo = 0.0f;
    for (; any_marching() && trips < kMaxIterations; ++trips) {
      if (trips == kCullSafeIterations) full = true;
      uint64_t win = all;
      if (!full) {
        uint32_t th = 0u;  // +0
#pragma unroll
        for (int r = 0; r < R; r++) {
          const uint32_t u = __float_as_uint(tacc[r]);
          th = u > th ? u : th;
        }
        // The low end only rises (rays move forward and leave the march), so a
        // value from an earlier step is a valid lower bound: refreshed every
        // TLO_EVERY steps.
        if (TLO_EVERY == 1 || trips % TLO_EVERY == 1) {
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
        win = m & __builtin_amdgcn_ballot_w64(lo < thi) & __builtin_amdgcn_ballot_w64(hi > tlo);
      }
      if (FL & kFlVisitCost) visits += (uint32_t)__builtin_popcountll(win);
      float L[R];
      int dnew[R];
#pragma unroll
      for (int r = 0; r < R; r++) { L[r] = 0.0f; dnew[r] = draw[r]; }
      if (FL & kFlPair) {
        for (uint64_t mm = win; mm;) {
          const int k1 = __builtin_ctzll(mm);
          mm &= mm - 1;
          const SphereRec& s1 = sph[k1];
          if (mm) {
            const int k2 = __builtin_ctzll(mm);
            mm &= mm - 1;
            const SphereRec& s2 = sph[k2];
            float ss1[R], ss2[R];
#pragma unroll
            for (int r = 0; r < R; r++) {
              ss1[r] = dist2(px[r], py[r], pz[r], s1.cx, s1.cy, s1.cz);
              ss2[r] = dist2(px[r], py[r], pz[r], s2.cx, s2.cy, s2.cz);
            }
            pass_body_r<R>(ss1, s1.s_pass, s1.r, k1, L, dnew);
            pass_body_r<R>(ss2, s2.s_pass, s2.r, k2, L, dnew);
          } else {
            visit(s1.cx, s1.cy, s1.cz, s1.r, s1.s_pass, k1, L, dnew);
          }
        }
      } else if (FL & kFlPrefetch) {
        if (win) {
          int k = __builtin_ctzll(win);
          float cx = sph[k].cx, cy = sph[k].cy, cz = sph[k].cz, rad = sph[k].r, sp = sph[k].s_pass;
          for (uint64_t mm = win & (win - 1);; mm &= mm - 1) {
            const int kn = mm ? __builtin_ctzll(mm) : k;
            const float ncx = sph[kn].cx, ncy = sph[kn].cy, ncz = sph[kn].cz, nr = sph[kn].r,
                        nsp = sph[kn].s_pass;
            visit(cx, cy, cz, rad, sp, k, L, dnew);
            if (!mm) break;
            k = kn; cx = ncx; cy = ncy; cz = ncz; rad = nr; sp = nsp;
          }
        }
      } else if (FL & kFlBits) {
        for (uint64_t mm = win; mm;) {
          const int k = __builtin_ctzll(mm);
          __asm__("s_bitset0_b64 %0, %1" : "+s"(mm) : "s"(k));
          const SphereRec& s = sph[k];
          visit(s.cx, s.cy, s.cz, s.r, s.s_pass, k, L, dnew);
        }
      } else {
        for (uint64_t mm = win; mm; mm &= mm - 1) {
          const int k = __builtin_ctzll(mm);
          const SphereRec& s = sph[k];
          visit(s.cx, s.cy, s.cz, s.r, s.s_pass, k, L, dnew);
        }
      }
      advance(L, dnew);
    }
  }
  if (trips >= kMaxIterations && any_marching() && lane == 0) atomicOr(f.status, 1);
  if (WPB == 1 && f.tile_cost && lane == 0)
    f.tile_cost[tile] = (uint8_t)tile_bucket((FL & kFlVisitCost) ? (visits >> 2) : (uint32_t)trips);
#pragma unroll
  for (int r = 0; r < R; r++) {
    if (valid[r]) {
      if (FL & kFlNoShade) {
        f.out[(long long)(b - f.sub_row0) * f.out_pitch + a[r]] =
            __float_as_uint(px[r]) ^ __float_as_uint(py[r]) ^ __float_as_uint(pz[r]) ^ (uint32_t)draw[r];
        continue;
      }
      const SphereRec d = sph[draw[r]];
      const uint32_t rgba = shade(f, d, px[r], py[r], pz[r], nullptr);
      f.out[(long long)(b - f.sub_row0) * f.out_pitch + a[r]] = rgba;
    }
  }
}

template <int SLOTS, int R, int WPB = kWavesPerBlock, int TLO_EVERY = 1, int FL = 0>
__global__ __launch_bounds__(64 * WPB) void k_trace_window_r(InlineArgs args) {
  trace_tile_window_r<SLOTS, R, WPB, TLO_EVERY, FL>(args.f, args.s);
}

template <int SLOTS, int WPB = kWavesPerBlock, int TLO_EVERY = 1>
__global__ __launch_bounds__(64 * WPB) void k_trace_window(InlineArgs args) {
  trace_tile_window<SLOTS, WPB, TLO_EVERY>(args.f, args.s);
}

template <int SLOTS, bool REST_LDS>
__global__ __launch_bounds__(256) void k_trace_inline(InlineArgs args) {
  if (REST_LDS) {  // spheres beyond the slots read from an LDS copy instead of s_load
    __shared__ SphereRec lsph[kInlineSpheres];
    for (int t = threadIdx.x; t < args.f.n; t += blockDim.x) lsph[t] = args.s[t];
    __syncthreads();
    trace_tile<true, SLOTS>(args.f, args.s, lsph);
  } else {
    trace_tile<true, SLOTS>(args.f, args.s, args.s);
  }
}

// n > 64 with the march window: per culling word, the lanes' (lo, hi) pairs
// live in dynamic LDS ([wave][lo/hi][n rounded up to 64] floats).
__device__ __forceinline__ void trace_tile_window_global(const FrameRec& f,
                                                         const SphereRec* __restrict__ sph,
                                                         float* __restrict__ s_win) {
  __shared__ uint64_t s_mask[kWavesPerBlock][kMaskWords];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tile = blockIdx.x * kWavesPerBlock + wave;
  const int tile_y = tile / f.tiles_x;
  const int tile_x = tile - tile_y * f.tiles_x;
  if (tile_y * kTile >= f.sub_rows) return;  // grid rounding; uniform per wave
  const int a = tile_x * kTile + (lane & 7);
  const int b = f.sub_row0 + tile_y * kTile + (lane >> 3);
  const int b_end = f.sub_row0 + f.sub_rows;
  const bool valid = a < f.sub_w && b < b_end;
  const int ac = a < f.sub_w ? a : f.sub_w - 1;
  const int bc = b < b_end ? b : b_end - 1;
  const int i = f.xstart + ac * f.xadd;
  const int j = f.ystart + bc * f.yadd;

  float dx, dy, dz;
  primary_dir(f, i, j, dx, dy, dz);

  const float l0 = f.first_l;
  float px = f.cam[0] + dx * l0;
  float py = f.cam[1] + dy * l0;
  float pz = f.cam[2] + dz * l0;
  int draw = f.first_draw;
  float mv = (valid && l0 > 0.0f) ? 1.0f : 0.0f;
  float tacc = l0;

  const int nwords = (f.n + 63) >> 6;
  float* const w_lo = s_win + (size_t)wave * 2 * nwords * 64;
  float* const w_hi = w_lo + nwords * 64;
  const bool any_march = __builtin_amdgcn_ballot_w64(mv > 0.0f) != 0;
  const bool windowed = f.cull && any_march;
  if (windowed) {
    const Cone cone = tile_cone(f, tile_x, tile_y, dx, dy, dz);
    for (int w = 0; w < nwords; w++) {
      float lo, hi;
      const uint64_t m = cull_window(f, sph, w * 64, cone, lo, hi);
      if (lane == 0) s_mask[wave][w] = m;
      w_lo[w * 64 + lane] = lo;
      w_hi[w * 64 + lane] = hi;
    }
  }
  __builtin_amdgcn_wave_barrier();
  int trips = 1;
  bool full = !windowed;
  while (__builtin_amdgcn_ballot_w64(mv > 0.0f)) {
    if (trips == kCullSafeIterations) full = true;  // uniform: visit all from here on
    float tlo = 0.0f, thi = 0.0f;
    if (!full) {
      tlo = __uint_as_float(wave_min_u32(__float_as_uint(mv > 0.0f ? tacc : __builtin_inff())));
      thi = __uint_as_float(wave_max_u32(__float_as_uint(tacc)));
    }
    float L = 0.0f;
    int dnew = draw;
    for (int w = 0; w < nwords; w++) {
      uint64_t win;
      if (full) {
        const int rem = f.n - w * 64;
        win = rem >= 64 ? ~0ull : ((1ull << rem) - 1ull);
      } else {
        win = uniform_u64(s_mask[wave][w]) &
              __builtin_amdgcn_ballot_w64(w_lo[w * 64 + lane] < thi) &
              __builtin_amdgcn_ballot_w64(w_hi[w * 64 + lane] > tlo);
      }
      for (; win; win &= win - 1) {
        const int k = w * 64 + __builtin_ctzll(win);
        const SphereRec& s = sph[k];
        sphere_step(px, py, pz, s.cx, s.cy, s.cz, s.r, s.s_pass, k, L, dnew);
      }
    }
    if (mv > 0.0f) {
      px = px + dx * L;
      py = py + dy * L;
      pz = pz + dz * L;
      draw = dnew;
      mv = L;
      tacc = tacc + L;
    }
    if (++trips >= kMaxIterations) {
      if (mv > 0.0f) atomicOr(f.status, 1);
      break;
    }
  }
  if (!valid) return;
  const SphereRec d = sph[draw];
  const uint32_t rgba = shade(f, d, px, py, pz, nullptr);
  f.out[(long long)(b - f.sub_row0) * f.out_pitch + a] = rgba;
}

__global__ __launch_bounds__(256) void k_trace_global_window(FrameRec f) {
  extern __shared__ float s_win[];
  trace_tile_window_global(f, f.spheres, s_win);
}

__global__ __launch_bounds__(256) void k_trace_global(FrameRec f) {
  trace_tile<false, 0>(f, f.spheres, f.spheres);
}

// Debug/parity kernel: one lane per listed pixel, full sphere list, float
// intermediates out (pos, drawSphere, iterations, xcoord, ycoord, brightness).
__global__ __launch_bounds__(256) void k_trace_points(FrameRec f, const int* __restrict__ ij,
                                                      int count, PixelDump* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= count) return;
  const SphereRec* __restrict__ sph = f.spheres;
  float dx, dy, dz;
  primary_dir(f, ij[2 * t], ij[2 * t + 1], dx, dy, dz);
  const float l0 = f.first_l;
  float px = f.cam[0] + dx * l0, py = f.cam[1] + dy * l0, pz = f.cam[2] + dz * l0;
  int draw = f.first_draw;
  int iters = 1;
  float L = l0;
  while (L > 0.0f && iters < kMaxIterations) {
    L = 0.0f;
    for (int k = 0; k < f.n; k++) {
      const SphereRec& s = sph[k];
      const float ex = px - s.cx, ey = py - s.cy, ez = pz - s.cz;
      const float ss = (ex * ex + ey * ey) + ez * ez;
      if (ss < s.s_pass) {
        const float tt = s.r - __builtin_sqrtf(ss);
        L = L < tt ? tt : L;
        draw = k;
      }
    }
    px = px + dx * L;
    py = py + dy * L;
    pz = pz + dz * L;
    ++iters;
  }
  PixelDump dmp;
  dmp.pos[0] = px; dmp.pos[1] = py; dmp.pos[2] = pz;
  dmp.draw = draw;
  dmp.iters = iters;
  shade(f, sph[draw], px, py, pz, &dmp);
  out[t] = dmp;
}

}  // namespace

// Pixels per lane of an ordered launch (adaptive tile order): the widest tile
// -- four pixels per lane (32x8), else three (24x8) -- whose grid still has
// >= 30000 tiles, about four waves per wave slot of the chip, enough for
// longest-first to balance; else two (16x8).  Measured: 4K 64 spheres 177
// (16x8) -> 173.5 (24x8) -> 172.9 us (32x8), 8K 645.6 -> 636.7 us (24x8 ->
// 32x8); 1080p 10 spheres 37.3 us at 16x8 against 39.4 / 41.0 wider.
static int ordered_rays(const FrameRec& f) {
  const long long rows = (f.sub_rows + kTile - 1) / kTile;
  const long long t4 = (long long)((f.sub_w + 4 * kTile - 1) / (4 * kTile)) * rows;
  const long long t3 = (long long)((f.sub_w + 3 * kTile - 1) / (3 * kTile)) * rows;
  return t4 >= 30000 ? 4 : t3 >= 30000 ? 3 : 2;
}

// The kernel choice of launch_trace, shared with trace_tile_key.  Default:
// two pixels per lane (16x8 tiles) above kPairMinSpheres spheres; in the
// adaptive tile order ordered_rays for any scene (1080p, 10 spheres: 16x8 tiles
// 37.4 us against 42.0 with 8x8, which win only in row-major order: 45.7 vs 48.5).
static int trace_rays(const FrameRec& f, bool ordered) {
  return f.variant == 49 ? 1
         : f.variant == 40 || f.variant == 41 || (f.variant >= 44 && f.variant <= 48 && f.variant != 46) ? 2
         : f.variant == 72 || f.variant == 85 || (f.variant >= 94 && f.variant <= 97) ? 3
         : f.variant == 73 || f.variant == 86 ? 4
         : f.variant == 74 || f.variant == 75 || f.variant == 83 || f.variant == 91 ? 1
         : (f.variant >= 60 && f.variant <= 71) || (f.variant >= 80 && f.variant <= 82) || f.variant == 84 ||
                f.variant == 90 ? 2
         : f.variant == 42 ? 3
         : f.variant == 43 ? 4
         : (f.variant == 0 && ordered) ? ordered_rays(f)
         : (f.variant == 0 && f.n > kPairMinSpheres) ? 2 : 1;
}
static bool trace_window_r(const FrameRec& f, int rays) {
  return f.n <= kInlineSpheres &&
         (rays > 1 || f.variant == 0 || f.variant == 49 || f.variant == 74 || f.variant == 75 ||
          f.variant == 83 || f.variant == 91);
}

long long trace_tile_key(const FrameRec& f, long long* tiles) {
  *tiles = 0;
  const int rays = trace_rays(f, true);
  // one wave per workgroup: every R-kernel launch except variants 40-43 and 45
  if (!trace_window_r(f, rays) || (f.variant >= 40 && f.variant <= 43) || f.variant == 45) return 0;
  const long long tiles_x = (f.sub_w + rays * kTile - 1) / (rays * kTile);
  const long long tiles_y = (f.sub_rows + kTile - 1) / kTile;
  if (tiles_x <= 0 || tiles_y <= 0) return 0;
  *tiles = tiles_x * tiles_y;
  return (1ll << 62) | ((long long)rays << 56) | (tiles_x << 28) | tiles_y;
}

int launch_trace(const FrameRec& f, const SphereRec* host_spheres, void* stream) {
  const long long tiles_y = (f.sub_rows + kTile - 1) / kTile;
  const long long tiles = tiles_y * f.tiles_x;
  if (tiles <= 0) return 0;
  const long long blocks = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks > 0x7fffffffLL || tiles > 0x7fffffffLL) return -1;
  hipStream_t s = (hipStream_t)stream;
  // Default for n <= 64: trace_tile_window_r with 16x8 tiles (two pixels per
  // lane) once the scene has more than kPairMinSpheres spheres; with few
  // spheres 8x8 tiles (one pixel per lane) win.  Both run one wave per
  // workgroup (a finished wave's slot is refilled at once), refresh the march
  // window's low end every second step and use kFlMask | kFlFree (measured,
  // DESIGN.md 5).
  const int rays = trace_rays(f, f.tile_cost != nullptr);
  if (trace_window_r(f, rays)) {
    // (8 rays) x 8 tiles: several pixels per lane
    InlineArgs args;
    args.f = f;
    args.f.tiles_x = (f.sub_w + rays * kTile - 1) / (rays * kTile);
    for (int k = 0; k < f.n; k++) args.s[k] = host_spheres[k];
    const long long tiles2 = tiles_y * args.f.tiles_x;
    long long key_tiles = 0;
    if (trace_tile_key(f, &key_tiles) == 0 || key_tiles != tiles2) {  // no adaptive order here
      args.f.tile_order = nullptr; args.f.tile_cost = nullptr; args.f.prev_cost = nullptr;
    }
    // one wave per workgroup (+ the tile-order sorter, sfrt_trace.h FrameRec)
    const dim3 g1((unsigned)(tiles2 + (args.f.prev_cost ? 1 : 0))), b1(64);
    const dim3 g4((unsigned)((tiles2 + kWavesPerBlock - 1) / kWavesPerBlock)), b4(256);
    // SFRT_OPT_VARIANT (A/B only): 40 / 41: four waves per workgroup, low end every
    // step, 4 / 0 slots; 42 / 43: 24x8 / 32x8 tiles; 44 / 45: one / two waves per
    // workgroup, low end every step; 48: low end every 4th step; 49: 8x8 tiles here;
    // 47: no FL flags; 61-71: 60 + FL bits (kFlMask 1, kFlFree 2, kFlPrefetch 4,
    // kFlPair 8); 72 / 73 / 74: 24x8 / 32x8 / 8x8 tiles with FL 3, 75: 8x8 with
    // kFlPair; 81 / 82: FL 3 | kFlBits, default | kFlBits; 80 / 83: the defaults
    // (16x8 / 8x8, kFlDefault); 90 / 91: timing probes without shading (wrong
    // bytes).  Measured: DESIGN.md 5.
    switch (f.variant) {
      case 40: hipLaunchKernelGGL((k_trace_window_r<kSlots, 2>), g4, b4, 0, s, args); break;
      case 41: hipLaunchKernelGGL((k_trace_window_r<0, 2>), g4, b4, 0, s, args); break;
      case 42: hipLaunchKernelGGL((k_trace_window_r<kSlots, 3>), g4, b4, 0, s, args); break;
      case 43: hipLaunchKernelGGL((k_trace_window_r<kSlots, 4>), g4, b4, 0, s, args); break;
      case 44: hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1>), g1, b1, 0, s, args); break;
      case 45:
        hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 2>), dim3((unsigned)((tiles2 + 1) / 2)),
                           dim3(128), 0, s, args);
        break;
      case 48: hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1, 4>), g1, b1, 0, s, args); break;
      case 49: hipLaunchKernelGGL((k_trace_window_r<kSlots, 1, 1, 2>), g1, b1, 0, s, args); break;
      case 61: hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1, 2, 1>), g1, b1, 0, s, args); break;
      case 62: hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1, 2, 2>), g1, b1, 0, s, args); break;
      case 64: hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1, 2, 4>), g1, b1, 0, s, args); break;
      case 67: hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1, 2, 7>), g1, b1, 0, s, args); break;
      case 71: hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1, 2, 11>), g1, b1, 0, s, args); break;
      case 72: hipLaunchKernelGGL((k_trace_window_r<kSlots, 3, 1, 2, 3>), g1, b1, 0, s, args); break;
      case 73: hipLaunchKernelGGL((k_trace_window_r<kSlots, 4, 1, 2, 3>), g1, b1, 0, s, args); break;
      case 74:
        hipLaunchKernelGGL((k_trace_window_r<kSlots, 1, 1, 2, kFlMask | kFlFree>), g1, b1, 0, s, args);
        break;
      case 75: hipLaunchKernelGGL((k_trace_window_r<kSlots, 1, 1, 2, 11>), g1, b1, 0, s, args); break;
      case 81: hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1, 2, 3 | kFlBits>), g1, b1, 0, s, args); break;
      case 82:
        hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1, 2, 3 | kFlNoTiny | kFlBits>), g1, b1, 0, s, args);
        break;
      case 84:
        hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1, 2, kFlDefault | kFlVisitCost>), g1, b1, 0, s, args);
        break;
      case 85: hipLaunchKernelGGL((k_trace_window_r<kSlots, 3, 1, 2, kFlDefault>), g1, b1, 0, s, args); break;
      case 86: hipLaunchKernelGGL((k_trace_window_r<kSlots, 4, 1, 2, kFlDefault>), g1, b1, 0, s, args); break;
      case 94: hipLaunchKernelGGL((k_trace_window_r<kSlots, 3, 1, 1, kFlDefault>), g1, b1, 0, s, args); break;
      case 95: hipLaunchKernelGGL((k_trace_window_r<kSlots, 3, 1, 4, kFlDefault>), g1, b1, 0, s, args); break;
      case 96: hipLaunchKernelGGL((k_trace_window_r<0, 3, 1, 2, kFlDefault>), g1, b1, 0, s, args); break;
      case 97: hipLaunchKernelGGL((k_trace_window_r<8, 3, 1, 2, kFlDefault>), g1, b1, 0, s, args); break;
      case 90: hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1, 2, kFlDefault | kFlNoShade>), g1, b1, 0, s, args); break;
      case 91: hipLaunchKernelGGL((k_trace_window_r<kSlots, 1, 1, 2, kFlDefault | kFlNoShade>), g1, b1, 0, s, args); break;
      case 47: hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1, 2>), g1, b1, 0, s, args); break;
      case 63: hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1, 2, 3>), g1, b1, 0, s, args); break;
      case 80:
      case 83:
      default:
        if (rays == 1)  // default for n <= kPairMinSpheres: 8x8 tiles (= variant 83)
          hipLaunchKernelGGL((k_trace_window_r<kSlots, 1, 1, 2, kFlDefault>), g1, b1, 0, s, args);
        else if (rays == 3)  // large ordered frames (= variant 85)
          hipLaunchKernelGGL((k_trace_window_r<kSlots, 3, 1, 2, kFlDefault>), g1, b1, 0, s, args);
        else if (rays == 4)  // larger ordered frames (= variant 86)
          hipLaunchKernelGGL((k_trace_window_r<kSlots, 4, 1, 2, kFlDefault>), g1, b1, 0, s, args);
        else  // (= variant 80)
          hipLaunchKernelGGL((k_trace_window_r<kSlots, 2, 1, 2, kFlDefault>), g1, b1, 0, s, args);
        break;
    }
  } else if (f.n <= kInlineSpheres) {
    InlineArgs args;
    args.f = f;
    for (int k = 0; k < f.n; k++) args.s[k] = host_spheres[k];
    // SFRT_OPT_VARIANT (tuning A/B only).  Default (8x8 tiles, one wave per
    // workgroup, window low end every second step): march window with the
    // SGPR-slot march for waves with <= kSlots culled spheres; 52: the same
    // whatever n; 46: low end every step; 35: also four waves per workgroup; 2: slots + the rest every step (no window); 1/6/8: slot
    // counts; 16/17: LDS-backed rest; 32/36: window with 0/6 slots.
    const dim3 g((unsigned)blocks), b(256);
    switch (f.variant) {
      case 1: hipLaunchKernelGGL((k_trace_inline<0, false>), g, b, 0, s, args); break;
      case 6: hipLaunchKernelGGL((k_trace_inline<6, false>), g, b, 0, s, args); break;
      case 8: hipLaunchKernelGGL((k_trace_inline<8, false>), g, b, 0, s, args); break;
      case 16: hipLaunchKernelGGL((k_trace_inline<kSlots, true>), g, b, 0, s, args); break;
      case 17: hipLaunchKernelGGL((k_trace_inline<0, true>), g, b, 0, s, args); break;
      case 2: hipLaunchKernelGGL((k_trace_inline<kSlots, false>), g, b, 0, s, args); break;
      case 32: hipLaunchKernelGGL(k_trace_window<0>, g, b, 0, s, args); break;
      case 36: hipLaunchKernelGGL(k_trace_window<6>, g, b, 0, s, args); break;
      case 35: hipLaunchKernelGGL(k_trace_window<kSlots>, g, b, 0, s, args); break;
      case 46:
        hipLaunchKernelGGL((k_trace_window<kSlots, 1>), dim3((unsigned)tiles), dim3(64), 0, s, args);
        break;
      case 52:
      default:
        hipLaunchKernelGGL((k_trace_window<kSlots, 1, 2>), dim3((unsigned)tiles), dim3(64), 0, s, args);
        break;
    }
  } else {
    if (f.variant == 2) {  // A/B: the per-word culled lists visited every step
      hipLaunchKernelGGL(k_trace_global, dim3((unsigned)blocks), dim3(256), 0, s, f);
    } else {
      const size_t lds = (size_t)kWavesPerBlock * 2 * (size_t)((f.n + 63) / 64) * 64 * sizeof(float);
      hipLaunchKernelGGL(k_trace_global_window, dim3((unsigned)blocks), dim3(256), lds, s, f);
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_trace_points(const FrameRec& f, const int* dev_ij, int count, PixelDump* dev_out,
                        void* stream) {
  if (count <= 0) return 0;
  hipLaunchKernelGGL(k_trace_points, dim3((count + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, f, dev_ij, count, dev_out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace sfrt
