// sfrt_host.h -- host-side helpers shared by the C-ABI translation units
// (sfrt_world.cpp, sfrt_glsl.cpp, sfrt_voxel.cpp, sfrt_multi.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include "sfrt.h"

namespace sfrt {

// Makes `dev` the calling thread's current HIP device for the guard's scope and
// restores the caller's device afterwards (a C-ABI call must not move it).
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

}  // namespace sfrt

// Any HIP failure becomes SFRT_E_HIP at the boundary.
#define HIP_TRY(expr)                            \
  do {                                           \
    if ((expr) != hipSuccess) return SFRT_E_HIP; \
  } while (0)
