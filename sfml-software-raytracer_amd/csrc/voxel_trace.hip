// voxel_trace.hip -- gfx950 kernel for the reference's voxel World frame fill
// (SURVEY 8f row f2): World::Raycast / World::LRaycast,
// /root/reference/Raytracing/World.cpp:302-491, one lane per pixel.
//
// Bit-exact with oracle/voxelworld_oracle.c: binary32 in the reference's
// expression order, -ffp-contract=off, correctly rounded division and sqrt,
// and the x86-64 float->integer conversions of the reference's build
// (out-of-range and NaN give INT_MIN / 0) emulated explicitly.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "sfrt_device.h"
#include "sfrt_math.h"
#include "voxel_trace.h"

#pragma clang fp contract(off)

// cell_hit's buffer descriptor word 3 (0x00020000, DATA_FORMAT_32) is the gfx9 / CDNA encoding;
// gfx10+ lay that word out differently.  This file is built for gfx950 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "voxel_trace.hip: the grid's buffer descriptor is encoded for gfx950 (CDNA4)"
#endif

namespace sfrt {
namespace {

constexpr float kPI = 3.1415926535f;     // World.h:5
constexpr float kPI2 = 6.28318530718f;   // World.h:6

// x86-64 cvttss2si semantics (the reference's build): INT_MIN when out of range or NaN.
__device__ __forceinline__ int32_t to_i32(float f) {
  return (f > -2147483648.0f && f < 2147483648.0f) ? (int32_t)f : (int32_t)0x80000000;
}
// A primary-ray DDA position to its cell coordinate: to_i32, or in the fast DDA (every lane of
// the wave within the host's dda_qlim bound, so |f| < 2^30) the plain conversion it equals
// there -- one v_cvt_i32_f32 instead of a compare, a conversion and a select per axis and step.
template <bool FAST>
__device__ __forceinline__ int32_t pos_i32(float f) {
  return FAST ? (int32_t)f : to_i32(f);
}
// float -> unsigned as x86-64 g++ emits it: 64-bit cvttss2si, low 32 bits.
__device__ __forceinline__ uint32_t to_u32(float f) {
  if (!(f > -9.2233720368547758e18f && f < 9.2233720368547758e18f)) return 0u;
  return (uint32_t)(long long)f;
}
__device__ __forceinline__ uint32_t to_u8(float f) {
  return (uint32_t)to_i32(f) & 0xffu;
}
__device__ __forceinline__ float min255(float v) { return 255.0f < v ? 255.0f : v; }

struct V3 {
  float x, y, z;
};

// blocks.contains((x << 20) + (y << 10) + z) (World.cpp:385, 476).  The reference's map key IS
// a linear index: (x << 20) + (y << 10) + z, in wrapping 32-bit arithmetic, is the offset of cell
// (x, y, z) in a dense [2048][1024][1024] array, and every stored key lies below nx << 20.  So the
// host stores the world as that array of bytes (VoxFrame::cells, nx << 20 bytes: code = id +
// kVoxCellBias, 0 = empty; rows and planes beyond ny / nz stay 0), and a lookup is the key itself
// as the byte offset of a buffer load whose range check (num_records = nx << 20) returns 0 for
// every key at or past the last x-plane -- negative keys included (>= 2^31 as unsigned).  No
// decode of the key, no validity compares, no index arithmetic: two v_lshl_add_u32 and the load
// per step, exactly the reference's contains() (profiles/ab/r5_ab1).  `code` is the cell's code
// when the cell is hit (id = code - kVoxCellBias).
__device__ __forceinline__ bool cell_hit(const VoxFrame& f, int32_t x, int32_t y, int32_t z,
                                         uint32_t& code) {
  // ((x << 10) + y) << 10) + z: two v_lshl_add_u32 (left alone: two shifts and an add3)
  uint32_t key;
  __asm__("v_lshl_add_u32 %0, %1, 10, %2" : "=v"(key) : "v"(x), "v"(y));
  __asm__("v_lshl_add_u32 %0, %1, 10, %2" : "=v"(key) : "v"(key), "v"(z));
  const __amdgpu_buffer_rsrc_t cells =
      __builtin_amdgcn_make_buffer_rsrc((void*)f.cells, (short)0, (int)f.cell_bytes, 0x00020000);
  code = __builtin_amdgcn_raw_buffer_load_b8(cells, (int)key, 0, 0);
  return code != 0u;
}

__device__ __forceinline__ uint32_t texel(const VoxFrame& f, const VoxTex& t, uint32_t x,
                                          uint32_t y) {
  const uint32_t idx = x + y * (uint32_t)t.w;
  if (t.texels == nullptr || idx >= (uint32_t)(t.w * t.h)) {
    atomicOr(f.status, 2);       // the reference reads outside the image here
    return 0xffff00ffu;          // magenta, as the oracle
  }
  return t.texels[idx];
}

// The DDA divides by the same |dir| components at every step.  With their
// correctly rounded reciprocals, sfrt_math::div_recip gives the same bits as
// the division for b in [2^-60, 2^60]; a wave with any lane
// outside that range (an axis-parallel ray has |dir.x| == 0) divides plainly.
__device__ __forceinline__ bool recip_ok(float b) { return b >= 0x1.0p-60f && b <= 0x1.0p60f; }

// dirXadd + sign * (pos - (float)ipos) (World.cpp:330-332, 466-468): sign is +-1, so the product
// is exact and one fma rounds the sum exactly as the reference's add does (NaN and inf alike).
__device__ __forceinline__ float dda_num(float add, float sign, float p, int32_t ip) {
  return __builtin_fmaf(sign, p - (float)ip, add);
}

template <bool RECIP>
__device__ __forceinline__ float dv(float a, float b, float y) {
  return RECIP ? sfrt_math::div_recip(a, b, y) : a / b;
}

// Light j through the constant address space (the table is never written by a launch):
// the wave-uniform loads become scalar loads instead of vector loads into VGPRs.
__device__ __forceinline__ VoxLight light_at(const VoxLight* p, int j) {
  const __attribute__((address_space(4))) uint32_t* q =
      (const __attribute__((address_space(4))) uint32_t*)(p + j);
  uint32_t w[sizeof(VoxLight) / 4];
#pragma unroll
  for (int i = 0; i < (int)(sizeof(VoxLight) / 4); i++) w[i] = q[i];
  VoxLight l;
  __builtin_memcpy(&l, w, sizeof l);
  return l;
}

__device__ __forceinline__ uint32_t pack(uint32_t r, uint32_t g, uint32_t b, uint32_t a) {
  return r | (g << 8) | (b << 16) | (a << 24);
}

// World::LRaycast, World.cpp:455-491.
template <bool RECIP>
__device__ bool lraycast_t(const VoxFrame& f, V3 pos, V3 dir, float maxDist,
                           uint32_t& work) {
  float dist = 0.0f;
  int32_t pix = to_i32(pos.x), piy = to_i32(pos.y), piz = to_i32(pos.z);
  const float dirxadd = dir.x > 0 ? 1.0f : 0.0f, diryadd = dir.y > 0 ? 1.0f : 0.0f,
              dirzadd = dir.z > 0 ? 1.0f : 0.0f;
  const float sx = dir.x > 0 ? -1.0f : 1.0f, sy = dir.y > 0 ? -1.0f : 1.0f,
              sz = dir.z > 0 ? -1.0f : 1.0f;
  const float lx = fabsf(dir.x), ly = fabsf(dir.y), lz = fabsf(dir.z);
  const float yx = RECIP ? 1.0f / lx : 0.0f, yy = RECIP ? 1.0f / ly : 0.0f,
              yz = RECIP ? 1.0f / lz : 0.0f;
  const float m2 = maxDist * 2;
  const uint32_t maxIter = to_u32(m2 < 20.0f ? 20.0f : m2);
  // One way out of the loop, as in raycast_t: the reference's loop test and its block hit
  // (return false) become one stop condition at the bottom of the step, the cell of the next
  // step's top tested there (only while the loop test holds, as the reference tests it).
  bool blocked = false;
  if ((0u < maxIter) & (dist < maxDist)) {
    work++;
    uint32_t code;
    blocked = cell_hit(f, pix, piy, piz, code);
    if (!blocked) {
      for (uint32_t i = 0;;) {
        const float a = dv<RECIP>(dda_num(dirxadd, sx, pos.x, pix), lx, yx);
        const float b = dv<RECIP>(dda_num(diryadd, sy, pos.y, piy), ly, yy);
        const float c = dv<RECIP>(dda_num(dirzadd, sz, pos.z, piz), lz, yz);
        float raySpeed = a;  // std::min({a, b, c})
        if (b < raySpeed) raySpeed = b;
        if (c < raySpeed) raySpeed = c;
        raySpeed += 0.002f;
        dist += raySpeed;
        pos.x = pos.x + dir.x * raySpeed;
        pos.y = pos.y + dir.y * raySpeed;
        pos.z = pos.z + dir.z * raySpeed;
        pix = to_i32(pos.x); piy = to_i32(pos.y); piz = to_i32(pos.z);
        i++;
        const bool more = (i < maxIter) & (dist < maxDist);
        work += more ? 1u : 0u;
        blocked = more & cell_hit(f, pix, piy, piz, code);
        if (!more | blocked) break;
      }
    }
  }
  return !blocked & (dist >= maxDist);
}

__device__ bool lraycast(const VoxFrame& f, V3 pos, V3 dir, float maxDist,
                         uint32_t& work) {
  const bool ok = recip_ok(fabsf(dir.x)) && recip_ok(fabsf(dir.y)) && recip_ok(fabsf(dir.z));
  if (__builtin_amdgcn_ballot_w64(!ok)) return lraycast_t<false>(f, pos, dir, maxDist, work);
  return lraycast_t<true>(f, pos, dir, maxDist, work);
}

// The hit block of World::Raycast (World.cpp:385-450): texel of the face the step crossed,
// light from every light source with shadow rays.  `dist` is the step's tryDist.
template <bool RECIP>
__device__ __forceinline__ uint32_t shade_hit(const VoxFrame& f, V3 pos, int32_t pix, int32_t piy,
                                              int32_t piz, int colRay, float sx, float sy,
                                              float sz, float dist, int id, uint32_t& work) {
  uint32_t c;
  if (id < 0) {
    c = f.colors[-id];
  } else {
    // the reference's three face branches (World.cpp:395-412) as selects of the same
    // expressions: one texel fetch per lane whatever mix of faces the wave's lanes hit
    const VoxTex& t = f.tex[id];
    const float tw = (float)(uint32_t)t.w, th = (float)(uint32_t)t.h;
    const float fx = pos.x - (float)pix, fy = pos.y - (float)piy, fz = pos.z - (float)piz;
    const bool c1 = colRay == 1, c2 = colRay == 2, c3 = !c1 & !c2;
    c = texel(f, t, to_u32(tw * (c1 ? fz : fx)), to_u32(th * (c2 ? fz : fy)));
    pos.x = c1 ? pos.x + sx * 0.01f : pos.x;  // get it off the wall
    pos.y = c2 ? pos.y + sy * 0.01f : pos.y;
    pos.z = c3 ? pos.z + sz * 0.01f : pos.z;
    sx = c1 ? sx : 0.0f;
    sy = c2 ? sy : 0.0f;
    sz = c3 ? sz : 0.0f;
  }
  const float l0 = 0.05f / dist - dist * 0.0001f;
  float litr = l0 < 0.0f ? 0.0f : l0;
  float litg = litr, litb = litr;
  // the record address stepped (a j * 36 product per light was four scalar instructions) and
  // the skip test's fields one scalar load (VoxLight): 4K 201.5 -> 198.0 us (profiles/ab/r5_ab2)
  const VoxLight* const lend = f.lights + f.nlights;
  for (const VoxLight* lp = f.lights; lp != lend; ++lp) {
    const VoxLight L = light_at(lp, 0);
    const float ex = pos.x - L.px, ey = pos.y - L.py, ez = pos.z - L.pz;
    // dd >= dd_pass: the light adds nothing (host threshold, exact); a wave none of whose lanes
    // is that close skips the light's division and the rest.  The test is ours: the squared
    // distance by two fmas against the host's inflated dd_skip (voxel_trace.h), and the body
    // evaluates the reference's dd
    const float ddf = __builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez));
    if (!__builtin_amdgcn_ballot_w64(ddf < L.dd_skip)) continue;
    float dd = ex * ex + ey * ey + ez * ez;  // VLengthS
    float add = (L.intensity / dd - dd * 0.002f);
    if (add > 0) {
      float nx = L.px - pos.x, ny = L.py - pos.y, nz = L.pz - pos.z;
      add *= ((nx * sx + ny * sy + nz * sz) * 0.7f + 0.3f);
      if (add > 0) {
        bool lit = true;
        if (L.shadows && dist < f.shadow_distance) {
          dd = __builtin_sqrtf(nx * nx + ny * ny + nz * nz);  // VLength
          nx = nx / dd; ny = ny / dd; nz = nz / dd;
          lit = lraycast(f, pos, V3{nx, ny, nz}, dd, work);
        }
        if (lit) {
          litr += add * L.r;
          litg += add * L.g;
          litb += add * L.b;
        }
      }
    }
  }
  return pack(to_u8(min255((float)(c & 0xffu) * litr)),
              to_u8(min255((float)((c >> 8) & 0xffu) * litg)),
              to_u8(min255((float)((c >> 16) & 0xffu) * litb)), c >> 24);
}

// World::Raycast, World.cpp:302-453.
template <bool RECIP>
__device__ uint32_t raycast_t(const VoxFrame& f, V3 dir, float yscale,
                              float atan_dir, uint32_t& work) {
  const V3 cam{f.cam[0], f.cam[1], f.cam[2]};
  float dist = 0.0f;
  V3 pos = cam;
  int32_t pix = pos_i32<RECIP>(pos.x), piy = pos_i32<RECIP>(pos.y), piz = pos_i32<RECIP>(pos.z);
  // The reference's tryPos (World.cpp:318) equals pos at the top of every step (pos = tryPos
  // ends each step), so the step advances pos in place after the billboard loop, which works
  // on copies of pos and dist (the reference moves both there and then overwrites them with
  // tryPos / tryDist): no second position carried around the loop and copied back each step.
  const float dirxadd = dir.x > 0 ? 1.0f : 0.0f, diryadd = dir.y > 0 ? 1.0f : 0.0f,
              dirzadd = dir.z > 0 ? 1.0f : 0.0f;
  const float sx = dir.x > 0 ? -1.0f : 1.0f, sy = dir.y > 0 ? -1.0f : 1.0f,
              sz = dir.z > 0 ? -1.0f : 1.0f;   // dir*sign (short, exact as float)
  const float lx = fabsf(dir.x), ly = fabsf(dir.y), lz = fabsf(dir.z);
  const float yx = RECIP ? 1.0f / lx : 0.0f, yy = RECIP ? 1.0f / ly : 0.0f,
              yz = RECIP ? 1.0f / lz : 0.0f;
  int DI = 0;
  float dnext = f.ndyn > 0 ? f.dyn[0].dist : __builtin_nanf("");  // next billboard; NaN: never >=
  int colRay = 0;
  float last_x = 0.0f, last_y = 0.0f, last_z = 0.0f;  // the last step's rays (colRay, below)
  // Shading after the loop: a lane that hits a block (or a billboard's opaque texel) stops
  // stepping, and the wave shades all its hit lanes once, after its last lane has stopped.
  // Shaded inside the loop, the light loop and its shadow rays ran once per distinct hit step
  // of the wave with the lanes of that step only (profiles/ab/r4_ab7: 4K 299 -> 289 us; with
  // the per-wave light skip 265 us).
  //
  //
  // One way out of the step loop: the reference leaves World::Raycast's loop three ways (its
  // loop test, a block hit, a billboard's opaque texel); as three divergent exits the compiler
  // kept a lane mask per exit and merged EXEC around each, ~35 scalar instructions and 3
  // branches per step (tools/isa_block_profile.py).  Here a lane tests one stop condition at the
  // bottom of the step, and what stopped it is read from registers afterwards: `early` != 0 (a
  // billboard's texel, alpha > 127), else `hcode` != 0 (the cell code of a block), else it marched
  // out.  A billboard's texel stops its lane through the loop test (the step's distance made
  // +inf); the lane still advances in that step, and nothing of it but `early` is read afterwards.
  // The first loop test is uniform (dist = 0, i = 0).  4K 234.6 -> 208.7 us, and 208.0 -> 201.5
  // with the outcome read back this way and the axis choice kept out of the loop's lane masks
  // (profiles/ab/r5_ab1, r5_ab2); with the two-instruction key, the billboard stop through the
  // distance and the step counters compiled out when no tile cost is recorded (k_voxel_ordered
  // COST): 200.8 -> 192.3 us (r5_ab4).  The hit face's axis (colRay) is recomputed after the loop
  // from the lane's last step's rays, by the step's own rule: computed in the loop it cost two
  // selects per step, and left for the compiler to sink it carried two lane masks merged with
  // EXEC every step (193.3 -> 188.0 us, r5_ab6).
  uint32_t hcode = 0u, early = 0u;
  if (0.0f < f.view_distance && 0u < f.maxiter) {
    for (uint32_t i = 0;;) {
      work++;
      const float xray = dv<RECIP>(dda_num(dirxadd, sx, pos.x, pix), lx, yx);
      const float yray = dv<RECIP>(dda_num(diryadd, sy, pos.y, piy), ly, yy);
      const float zray = dv<RECIP>(dda_num(dirzadd, sz, pos.z, piz), lz, yz);
      // the reference's if / else-if / else (World.cpp:330-350) as selects: one branch-free
      // step.  In the fast DDA no ray is NaN (finite numerators over |d| >= 2^-60), so the
      // reference's choice is the first axis whose ray equals the minimum (v_min3_f32; +-0
      // compare equal).  The speed can differ from the reference's only in the sign of a zero (a
      // negative ray underflowing to -0 beside a +0 one), which reaches the position only through
      // dir * speed added to a -0.0 component (a -0.0 camera coordinate not yet moved), and no
      // output depends on that sign (to_i32, the fractions, the texel and light offsets all map
      // +-0 alike)
      bool ax, ay;
      float raySpeed;
      if (RECIP) {
        raySpeed = fminf(fminf(xray, yray), zray);
        ax = xray == raySpeed;
        ay = !ax & (yray == raySpeed);
      } else {
        ax = (xray <= yray) & (xray <= zray);
        ay = !ax & (yray <= xray) & (yray <= zray);
        raySpeed = ax ? xray : (ay ? yray : zray);
      }
      const float rs2 = raySpeed + 0.002f;
      last_x = xray; last_y = yray; last_z = zray;
      float tryDist = dist + raySpeed;
      // dynamic billboards in front of the next block (World.cpp:353-378): the next billboard's
      // distance is held in a register (NaN past the last), so the test reads no memory on the
      // steps that pass no billboard (nearly all), and a wave whose lanes all pass none skips
      // the loop, which works on copies of pos and dist (the reference moves both there and then
      // overwrites them with tryPos / tryDist)
      if (__builtin_amdgcn_ballot_w64(tryDist >= dnext)) {
        V3 bp = pos;
        float bdist = dist;
        while (tryDist >= dnext) {
          const VoxDyn& d = f.dyn[DI];
          const float bs = d.dist - bdist;
          bdist = d.dist;
          bp.x = bp.x + dir.x * bs;
          bp.y = bp.y + dir.y * bs;
          bp.z = bp.z + dir.z * bs;
          const float to = d.py - bp.y;
          const float sizey = d.sy * yscale;
          if (fabsf(to) < sizey) {
            float ang = d.atan_b - atan_dir;  // VAngleXZ(dir, VNormalizeXZ(d->pos - cam.pos))
            ang = ang > kPI ? ang - kPI2 : (ang < -kPI ? ang + kPI2 : ang);
            ang = ang * bdist;
            const VoxTex& t = f.dyn_tex[d.tex];
            const float xf = (0.5f + ang / kPI * 0.5f / d.sx);
            if (xf > 0 && xf < 1) {
              int32_t x = to_i32(xf * (float)(uint32_t)t.w);
              int32_t y = to_i32((sizey + to) / sizey / 2 * (float)(uint32_t)t.h);
              x = x < 0 ? 0 : x;
              y = y < 0 ? 0 : y;
              const uint32_t c = texel(f, t, (uint32_t)x, (uint32_t)y);
              if ((c >> 24) > 127u) {
                early = pack(to_u8(min255((float)(c & 0xffu) * d.r)),
                             to_u8(min255((float)((c >> 8) & 0xffu) * d.g)),
                             to_u8(min255((float)((c >> 16) & 0xffu) * d.b)), c >> 24);
                tryDist = __builtin_inff();  // stops the lane through the loop test
                break;
              }
            }
          }
          DI++;
          dnext = DI < f.ndyn ? f.dyn[DI].dist : __builtin_nanf("");
        }
      }
      dist = tryDist;
      pos.x += dir.x * (ax ? rs2 : raySpeed);  // tryPos (World.cpp:330-350)
      pos.y += dir.y * (ay ? rs2 : raySpeed);
      pos.z += dir.z * ((ax | ay) ? raySpeed : rs2);
      pix = pos_i32<RECIP>(pos.x); piy = pos_i32<RECIP>(pos.y); piz = pos_i32<RECIP>(pos.z);
      cell_hit(f, pix, piy, piz, hcode);  // hcode != 0: hit a block (World.cpp:385)
      i++;
      if ((hcode != 0u) | !(dist < f.view_distance) | !(i < f.maxiter)) break;
    }
  }
  if (early != 0u) return early;  // a billboard's texel with alpha > 127: never 0
  // the axis of the lane's last step, from that step's rays (kept in registers: the loop's last
  // assignment is its exit value), by the step's own rule
  if (RECIP) {
    const float rs = fminf(fminf(last_x, last_y), last_z);
    colRay = last_x == rs ? 1 : (last_y == rs ? 2 : 3);
  } else {
    const bool ax = (last_x <= last_y) & (last_x <= last_z);
    const bool ay = !ax & (last_y <= last_x) & (last_y <= last_z);
    colRay = ax ? 1 : (ay ? 2 : 3);
  }
  if (hcode != 0u)
    return shade_hit<RECIP>(f, pos, pix, piy, piz, colRay, sx, sy, sz, dist,
                            (int)hcode - kVoxCellBias, work);
  return pack(0, 0, 0, 255);  // sf::Color::Black
}

__device__ uint32_t raycast(const VoxFrame& f, V3 dir, float yscale,
                            float atan_dir, uint32_t& work) {
  // the reciprocal divisions and, within the host's bound on the direction's spread, the plain
  // position conversions (pos_i32)
  const float lx = fabsf(dir.x), ly = fabsf(dir.y), lz = fabsf(dir.z);
  const bool ok = recip_ok(lx) && recip_ok(ly) && recip_ok(lz) &&
                  fmaxf(fmaxf(lx, ly), lz) <= f.dda_qlim * fminf(fminf(lx, ly), lz);
  if (__builtin_amdgcn_ballot_w64(!ok)) return raycast_t<false>(f, dir, yscale, atan_dir, work);
  return raycast_t<true>(f, dir, yscale, atan_dir, work);
}

// 8x8 pixels per one-wave workgroup (a finished wave's slot refills at once;
// 0.7-1.5% faster than 16x16 per 256 threads).
// The default: 8x8 tiles on a 1-D grid of one-wave workgroups in the adaptive
// tile order (sfrt_device.h sort_tiles; workgroup 0 is the sorter when
// prev_cost is set).
// Eight waves per SIMD: 58 VGPRs since the shading left the DDA loop (72 before, seven waves).
#ifndef SFRT_VOX_WAVES
#define SFRT_VOX_WAVES 8
#endif
// COST: record the tile's cost for the adaptive order (f.tile_cost set); without it the step
// counters are dead code and compiled out (one VALU per DDA and shadow-ray step)
template <bool COST>
__global__ __launch_bounds__(64, SFRT_VOX_WAVES) void k_voxel_ordered(VoxFrame f, int tiles_x, int ntiles) {
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
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int a = tx * 8 + (lane & 7);
  const int b = f.sub_row0 + ty * 8 + (lane >> 3);
  // Edge lanes trace a clamped duplicate pixel and store nothing (a divergent
  // branch around raycast() would make its wave-uniform choices divergent).
  const int ac = a < f.sub_w ? a : f.sub_w - 1;
  const int bc = b < f.sub_row0 + f.sub_rows ? b : f.sub_row0 + f.sub_rows - 1;
  uint32_t work = 0;
  const int i = f.xstart + ac * f.xadd;
  const int j = f.ystart + bc * f.yadd;
  const V3 dir{f.col[3 * i], f.row[2 * j], f.col[3 * i + 1]};
  const uint32_t rgba = raycast(f, dir, f.row[2 * j + 1], f.col[3 * i + 2], work);
  // The store's pixel from the lane id again (mbcnt, not threadIdx): kept live across
  // raycast(), a, b and `in` were spilled to scratch (16 bytes per lane).
  const int lane2 = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int a2 = tx * 8 + (lane2 & 7), r2 = ty * 8 + (lane2 >> 3);
  if (a2 < f.sub_w && r2 < f.sub_rows) f.out[(long long)r2 * f.out_pitch + a2] = rgba;
  if (COST) {
    // the tile's slowest ray, in DDA + shadow steps / 4 (the classes' scale)
    const uint32_t w = wave_max_u32(work);
    if (lane == 0) store_cost(f.tile_cost, tile, tile_bucket(w >> 2), cls, f.cost_diff);
  }
}

// The grid rewrite of launch_voxel_cells: one 256-lane workgroup per (x, y) row of the box, four
// bytes of the row per lane (a row starts at a 1 KiB boundary, so the full words are aligned
// dword stores).
__global__ __launch_bounds__(256) void k_voxel_cells(uint8_t* __restrict__ cells,
                                                     const uint8_t* __restrict__ codes, int nx, int ny,
                                                     int nz, int by, int bz) {
  const int x = (int)blockIdx.x / by, y = (int)blockIdx.x - x * by;
  const int z0 = 4 * (int)threadIdx.x;
  if (z0 >= bz) return;
  const bool row_in = x < nx && y < ny;
  const uint8_t* src = codes + ((size_t)x * ny + y) * nz;
  uint8_t b[4];
#pragma unroll
  for (int k = 0; k < 4; k++) b[k] = row_in && z0 + k < nz ? src[z0 + k] : (uint8_t)0;
  uint8_t* dst = cells + ((size_t)x << 20) + ((size_t)y << 10) + z0;
  if (z0 + 4 <= bz) {
    *reinterpret_cast<uint32_t*>(dst) =
        (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
  } else {
    for (int k = 0; z0 + k < bz; k++) dst[k] = b[k];
  }
}

}  // namespace

long long voxel_tile_key(const VoxFrame& f, long long* tiles) {
  *tiles = 0;
  if (f.sub_w <= 0 || f.sub_rows <= 0) return 0;
  const long long tx = (f.sub_w + 7) / 8, ty = (f.sub_rows + 7) / 8;
  *tiles = tx * ty;
  return (1ll << 62) | (tx << 28) | ty;
}

int launch_voxel(const VoxFrame& f, void* stream, void* done_event) {
  long long tiles = 0;
  if (voxel_tile_key(f, &tiles) == 0) return 0;
  // the kernel reads the grid through a buffer resource over f.cells (f.cell_bytes) and the tables
  // unguarded: refuse a record whose device pointers were not filled
  if (!f.cells || f.cell_bytes == 0 || !f.col || !f.row || !f.out || !f.status ||
      (f.ndyn > 0 && !f.dyn) || (f.nlights > 0 && !f.lights))
    return -1;
  if (tiles > 0x7ffffffeLL) return -1;
  // row-major unless the host linked this launch into its tile-order chain
  const dim3 grid((unsigned)(tiles + (f.prev_cost ? 1 : 0)));
  if (f.tile_cost)
    hipExtLaunchKernelGGL(k_voxel_ordered<true>, grid, dim3(64), 0, (hipStream_t)stream, nullptr,
                          (hipEvent_t)done_event, 0, f, (int)((f.sub_w + 7) / 8), (int)tiles);
  else
    hipExtLaunchKernelGGL(k_voxel_ordered<false>, grid, dim3(64), 0, (hipStream_t)stream, nullptr,
                          (hipEvent_t)done_event, 0, f, (int)((f.sub_w + 7) / 8), (int)tiles);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_voxel_cells(uint8_t* cells, const uint8_t* codes, int nx, int ny, int nz, int bx, int by,
                       int bz, void* stream) {
  // the box must hold the world and stay inside the key space (kVoxMax*), the rows inside 1 KiB
  if (!cells || (nx > 0 && !codes) || nx < 0 || ny < 0 || nz < 0 || bx < nx || by < ny || bz < nz ||
      bx > kVoxMaxX || by > kVoxMaxY || bz > kVoxMaxZ)
    return -1;
  if (bx == 0 || by == 0 || bz == 0) return 0;
  hipLaunchKernelGGL(k_voxel_cells, dim3((unsigned)((long long)bx * by)), dim3(256), 0,
                     (hipStream_t)stream, cells, codes, nx, ny, nz, by, bz);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace sfrt
