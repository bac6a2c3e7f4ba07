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

// One slot of a per-frame table ring (sfrt_voxel.cpp, sfrt_glsl.cpp): device tables, their
// pinned staging copy, and one event that every earlier user of the slot -- the staging copy and
// each launch that read it, on whatever stream -- completes before.  A launch on another stream
// than the slot's last user first makes its stream wait on that event, so (1) it never reads the
// tables before the staging copy landed and (2) the event it records afterwards still covers the
// earlier users: restaging waits on it alone.
struct TableSlot {
  void* d = nullptr;
  void* h = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  hipStream_t last = nullptr;  // stream of the last record of ev (valid while pending)
  bool pending = false;

  // Before restaging: every earlier user has finished with the slot.
  hipError_t reclaim() {
    if (pending) {
      const hipError_t e = hipEventSynchronize(ev);
      if (e != hipSuccess) return e;
    }
    pending = false;
    return ev ? hipSuccess : hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  }
  // After the staging copy was queued on s (a later reader on another stream waits for it).
  hipError_t staged(hipStream_t s) { return mark(s); }
  // Before queuing a launch on s that reads the slot.
  hipError_t use_on(hipStream_t s) {
    return (pending && last != s) ? hipStreamWaitEvent(s, ev, 0) : hipSuccess;
  }
  // After queuing a launch on s that reads the slot (use_on(s) came first).
  hipError_t launched(hipStream_t s) { return mark(s); }
  void release() {
    (void)hipFree(d);
    (void)hipHostFree(h);
    if (ev) (void)hipEventDestroy(ev);
    d = h = nullptr;
    ev = nullptr;
    cap = 0;
    pending = false;
  }

 private:
  hipError_t mark(hipStream_t s) {
    const hipError_t e = hipEventRecord(ev, s);
    if (e != hipSuccess) return e;
    last = s;
    pending = true;
    return hipSuccess;
  }
};

}  // namespace sfrt

// Any HIP failure becomes SFRT_E_HIP at the boundary.
#define HIP_TRY(expr)                            \
  do {                                           \
    if ((expr) != hipSuccess) return SFRT_E_HIP; \
  } while (0)
