// sfrt_probe.h -- diagnostic hooks of the sphere kernel (sphere_trace.hip), out of its body.
//
// trace_tile_window_r<R, LIST, DUMP, P> calls a handful of hooks on a probe object of type P.
// The shipped library instantiates it with NoProbe, whose hooks are empty (no state, no
// instructions: the release ISA is the probe-free kernel's, tools/isa_compare.py).  A build with
// -DSFRT_EXP=<bits> (sfrt_build_flavour() "diagnostic"; bench.py refuses it) instantiates
// DiagProbe<bits> instead, which writes probe values over each tile's first pixels -- wrong
// image bytes by design.  Bits (tools/tile_timeline.py, tools/visit_counts.py, tools/gpu/diag.sh):
//    16  per-tile wall clock: pixels 0..3 of the tile's first row = start, end, trips, slot
//   512  (with 16) the wave's entry time in place of its slot
//  1024  (with 16) the tile's shader clocks (s_memtime) in place of its trips
//    32  per-tile march counters: trips, sphere visits, visits that passed for some ray,
//        window mode (0 slots / 1 window), culled spheres
//    64  the march without the shading tail (a hash of the final positions is stored)
//   128  the shading's atan2f replaced by one multiply (timing probe)
//   256  the shading's asinf replaced by one multiply (timing probe)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "sfrt_device.h"
#include "sfrt_math.h"

#ifndef SFRT_EXP
#define SFRT_EXP 0
#endif

namespace sfrt {

// The release probe: every hook is empty and the shading is the reference's.
struct NoProbe {
  static constexpr bool kShade = true;
  __device__ __forceinline__ static float hit_atan2(float y, float x) { return atan2f_wave(y, x); }
  __device__ __forceinline__ static float hit_asin(float v) { return sfrt_math::asinf(v); }
  __device__ __forceinline__ void wave_entry() {}
  __device__ __forceinline__ void tile_begin() {}
  __device__ __forceinline__ void window_mode() {}
  __device__ __forceinline__ void visit(bool) {}
  __device__ __forceinline__ void march_only(uint32_t*, uint32_t) {}
  __device__ __forceinline__ void tile_end(uint32_t*, int, bool, int, int, uint64_t) {}
};

template <int EXP>
struct DiagProbe {
  static constexpr bool kShade = (EXP & 64) == 0;
  __device__ __forceinline__ static float hit_atan2(float y, float x) {
    if constexpr (EXP & 128) return y * x;
    else return atan2f_wave(y, x);
  }
  __device__ __forceinline__ static float hit_asin(float v) {
    if constexpr (EXP & 256) return v * 0.7f;
    else return sfrt_math::asinf(v);
  }
  uint64_t entry = 0, t0 = 0, c0 = 0;
  uint32_t visits = 0, passes = 0, mode = 0;
  __device__ __forceinline__ void wave_entry() {
    if constexpr (EXP & 512) entry = __builtin_amdgcn_s_memrealtime();
  }
  __device__ __forceinline__ void tile_begin() {
    if constexpr (EXP & 16) {
      t0 = __builtin_amdgcn_s_memrealtime();
      if constexpr (EXP & 1024) c0 = __builtin_amdgcn_s_memtime();
    }
  }
  __device__ __forceinline__ void window_mode() {
    if constexpr (EXP & 32) mode = 1;
  }
  __device__ __forceinline__ void visit(bool passed) {
    if constexpr (EXP & 32) {
      visits++;
      passes += passed ? 1u : 0u;
    }
  }
  // bit 64: the value stored in place of the shaded pixel
  __device__ __forceinline__ void march_only(uint32_t* out, uint32_t hash) { *out = hash; }
  // Overwrites pixels 0..4 of the tile's first row (lane l < 5 holds pixel l of ray 0).
  __device__ __forceinline__ void tile_end(uint32_t* out0, int lane, bool valid0, int trips, int slot,
                                           uint64_t culled) {
    if constexpr (EXP & 32) {
      if (lane < 5 && valid0) {
        *out0 = lane == 0 ? (uint32_t)trips : lane == 1 ? visits : lane == 2 ? passes
              : lane == 3 ? mode : (uint32_t)__builtin_popcountll(culled);
      }
    }
    if constexpr (EXP & 16) {
      const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
      uint32_t third = (uint32_t)trips;
      if constexpr (EXP & 1024) third = (uint32_t)(__builtin_amdgcn_s_memtime() - c0);
      uint32_t fourth = (uint32_t)slot;
      if constexpr (EXP & 512) fourth = (uint32_t)entry;
      if (lane < 4 && valid0)
        *out0 = lane == 0 ? (uint32_t)t0 : lane == 1 ? (uint32_t)t1 : lane == 2 ? third : fourth;
    }
  }
};

using ActiveProbe = std::conditional_t<(SFRT_EXP != 0), DiagProbe<SFRT_EXP>, NoProbe>;
constexpr bool kDiagnosticBuild = SFRT_EXP != 0;

}  // namespace sfrt
