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

#include "sfrt_math.h"
#include "sfrt_trace.h"

#pragma clang fp contract(off)

namespace sfrt {
namespace {

constexpr float kPI = 3.1415926535f;     // SphereWorld.h:6
constexpr float kPI2 = 6.28318530718f;   // SphereWorld.h:7

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}

// Primary direction of pixel (i, j), normalised (SphereWorld.cpp:95-106, :358).
__device__ __forceinline__ void primary_dir(const FrameRec& f, int i, int j, float& dx,
                                            float& dy, float& dz) {
  const float h = f.h_start + f.h_inc * (float)i;
  const float v = f.v_start + (float)j * f.v_inc;
  float x = (f.fwd[0] + f.right[0] * h) + f.up[0] * v;
  float y = (f.fwd[1] + f.right[1] * h) + f.up[1] * v;
  float z = (f.fwd[2] + f.right[2] * h) + f.up[2] * v;
  const float len = __builtin_sqrtf((x * x + y * y) + z * z);
  dx = x / len;
  dy = y / len;
  dz = z / len;
}

// Shading tail, SphereWorld.cpp:373-381.  Returns RGBA8 packed (r in byte 0).
__device__ __forceinline__ uint32_t shade(const FrameRec& f, const SphereRec& d, float px,
                                         float py, float pz, PixelDump* dump) {
  float ang = d.atan_c - sfrt_math::atan2f(pz, px);
  ang = ang > kPI ? ang - kPI2 : (ang < -kPI ? ang + kPI2 : ang);
  const float xcoord = ang / kPI2 + 1.0f;
  const float ex = px - d.cx, ey = py - d.cy, ez = pz - d.cz;
  const float ny = ey / __builtin_sqrtf((ex * ex + ey * ey) + ez * ez);
  const float ycoord = sfrt_math::asinf(ny) / kPI + 0.5f;
  const float bx = px - f.cam[0], by = py - f.cam[1], bz = pz - f.cam[2];
  const float bl = __builtin_sqrtf((bx * bx + by * by) + bz * bz);
  const float brightness = 3.0f / (bl < 3.0f ? 3.0f : bl);
  // fmodf(v, 1.0f) == v - truncf(v) exactly for every binary32 v (NaN/inf -> NaN).
  float u = xcoord * 4.0f * d.r;
  u = (u - __builtin_truncf(u)) * f.tex_wf;
  float w = ycoord * 2.0f * d.r;
  w = (w - __builtin_truncf(w)) * f.tex_hf;
  // float -> unsigned: v_cvt_u32_f32 (NaN -> 0), as x86's cvttss2si for [0, 2^31).
  const uint32_t tx = __float2uint_rz(u), ty = __float2uint_rz(w);
  const uint32_t idx = tx + ty * (uint32_t)f.tex_w;
  uint32_t texel = 0;
  if (idx < (uint32_t)(f.tex_w * f.tex_h)) {
    texel = f.tex[idx];
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

// Wave-level cull: bit k of the result is set when sphere (base + k) can pass
// the march test for some ray of this wave's tile.  Every lane holds one unit
// ray (dx, dy, dz) of the tile.  A sphere is dropped only when the whole
// cone around those rays misses the sphere inflated by a margin that covers
// binary32 rounding of the march positions (|error| << 1e-3 * (|c-cam| + r)
// for < 10^4 steps) -- inside that margin the reference test r - d > 0.01f
// cannot hold.  Spheres whose threshold is 0 never pass and are dropped.
__device__ __forceinline__ uint64_t cull_chunk(const FrameRec& f, const SphereRec* __restrict__ sph,
                                               int base, double ax, double ay, double az,
                                               double theta) {
  const int lane = threadIdx.x & 63;
  const int k = base + lane;
  bool inc = false;
  if (k < f.n) {
    const SphereRec s = sph[k];
    if (s.s_pass > 0.0f) {
      const double wx = (double)s.cx - (double)f.cam[0];
      const double wy = (double)s.cy - (double)f.cam[1];
      const double wz = (double)s.cz - (double)f.cam[2];
      const double dist = sqrt(wx * wx + wy * wy + wz * wz);
      const double rr = (double)s.r + 1e-3 * (dist + (double)s.r) + 1e-4;
      if (dist <= rr) {
        inc = true;
      } else {
        const double beta = asin(rr / dist);
        const double c = fmin(1.0, fmax(-1.0, (wx * ax + wy * ay + wz * az) / dist));
        inc = acos(c) <= theta + beta + 1e-6;
      }
    }
  }
  return __builtin_amdgcn_ballot_w64(inc);
}

template <bool INLINE>
__device__ __forceinline__ void trace_tile(const FrameRec& f, const SphereRec* __restrict__ sph) {
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

  // ---- per-wave sphere cull (the "wavefront ballot") ----
  const int nwords = (f.n + 63) >> 6;
  uint64_t mask0 = ~0ull;
  if (f.cull) {
    const double ddx = dx, ddy = dy, ddz = dz;
    double ax = wave_sum(ddx), ay = wave_sum(ddy), az = wave_sum(ddz);
    const double an = sqrt(ax * ax + ay * ay + az * az);
    ax /= an; ay /= an; az /= an;
    const double dn = sqrt(ddx * ddx + ddy * ddy + ddz * ddz);
    const double cmin = wave_min((ddx * ax + ddy * ay + ddz * az) / dn);
    const double theta = acos(fmin(1.0, cmin)) + 1e-6;
    if (INLINE) {
      mask0 = cull_chunk(f, sph, 0, ax, ay, az, theta);
    } else {
      for (int w = 0; w < nwords; w++) {
        const uint64_t m = cull_chunk(f, sph, w * 64, ax, ay, az, theta);
        if (lane == 0) s_mask[wave][w] = m;
      }
    }
  } else {
    if (!INLINE && lane < nwords) {
      const int rem = f.n - lane * 64;
      s_mask[wave][lane] = rem >= 64 ? ~0ull : ((1ull << rem) - 1ull);
    }
    if (INLINE) mask0 = f.n >= 64 ? ~0ull : ((1ull << f.n) - 1ull);
  }
  if (!INLINE) __builtin_amdgcn_wave_barrier();

  // ---- march, SphereWorld.cpp:362-372; iteration 1 (pos == cam) came from the host ----
  const float l0 = f.first_l;
  float px = f.cam[0] + dx * l0;
  float py = f.cam[1] + dy * l0;
  float pz = f.cam[2] + dz * l0;
  int draw = f.first_draw;
  int iters = 1;
  bool active = valid && l0 > 0.0f;
  while (__builtin_amdgcn_ballot_w64(active)) {
    float L = 0.0f;
    int dnew = draw;
    for (int w = 0; w < (INLINE ? 1 : nwords); w++) {
      uint64_t m = INLINE ? mask0 : s_mask[wave][w];
      m = __builtin_amdgcn_readfirstlane((unsigned)m) |
          ((uint64_t)__builtin_amdgcn_readfirstlane((unsigned)(m >> 32)) << 32);
      while (m) {
        const int k = w * 64 + __builtin_ctzll(m);
        m &= m - 1;
        const SphereRec& s = sph[k];
        const float ex = px - s.cx, ey = py - s.cy, ez = pz - s.cz;
        const float ss = (ex * ex + ey * ey) + ez * ez;
        if (ss < s.s_pass) {
          const float t = s.r - __builtin_sqrtf(ss);
          L = L < t ? t : L;  // std::max(largestDist, t)
          dnew = k;
        }
      }
    }
    if (active) {
      px = px + dx * L;
      py = py + dy * L;
      pz = pz + dz * L;
      draw = dnew;
      ++iters;
      active = L > 0.0f;
      if (iters >= kMaxIterations) {
        active = false;
        atomicOr(f.status, 1);
      }
    }
  }
  if (!valid) return;
  const SphereRec d = sph[draw];
  const uint32_t rgba = shade(f, d, px, py, pz, nullptr);
  f.out[(long long)(b - f.sub_row0) * f.out_pitch + a] = rgba;
}

__global__ __launch_bounds__(256) void k_trace_inline(InlineArgs args) {
  trace_tile<true>(args.f, args.s);
}

__global__ __launch_bounds__(256) void k_trace_global(FrameRec f) {
  trace_tile<false>(f, f.spheres);
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

int launch_trace(const FrameRec& f, const SphereRec* host_spheres, void* stream) {
  const long long tiles_y = (f.sub_rows + kTile - 1) / kTile;
  const long long tiles = tiles_y * f.tiles_x;
  if (tiles <= 0) return 0;
  const long long blocks = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks > 0x7fffffffLL) return -1;
  hipStream_t s = (hipStream_t)stream;
  if (f.n <= kInlineSpheres) {
    InlineArgs args;
    args.f = f;
    for (int k = 0; k < f.n; k++) args.s[k] = host_spheres[k];
    hipLaunchKernelGGL(k_trace_inline, dim3((unsigned)blocks), dim3(256), 0, s, args);
  } else {
    hipLaunchKernelGGL(k_trace_global, dim3((unsigned)blocks), dim3(256), 0, s, f);
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
