// sfrt_host.h -- host-side helpers shared by the C-ABI translation units
// (sfrt_world.cpp, sfrt_glsl.cpp, sfrt_voxel.cpp, sfrt_multi.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

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

// A device buffer that every launch reads, on whatever stream, and that is rewritten in place now
// and then (the voxel grid, sfrt_voxel.cpp): stream-ordered both ways, with no host or device-wide
// synchronisation.  One event per reading stream, re-recorded after each launch on it; a rewrite
// queued on stream w first makes w wait for each of them on the device (hipStreamWaitEvent), and
// records `written` after itself, which the next launch on each other stream waits for once.
struct SharedBuffer {
  struct Reader {
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;
    bool read = false;     // ev covers a launch that read the current contents
    bool current = false;  // s is ordered after the last rewrite
  };
  std::vector<Reader> readers;
  hipEvent_t written = nullptr;
  hipStream_t writer = nullptr;
  bool have_written = false;

  // Before queuing a launch on s that reads the buffer.
  hipError_t before_read(hipStream_t s) {
    Reader* r = nullptr;
    const hipError_t e = reader(s, &r);
    if (e != hipSuccess) return e;
    if (have_written && !r->current && s != writer) {
      const hipError_t w = hipStreamWaitEvent(s, written, 0);
      if (w != hipSuccess) return w;
    }
    r->current = true;
    return hipSuccess;
  }
  // After queuing that launch.
  hipError_t after_read(hipStream_t s) {
    Reader* r = nullptr;
    hipError_t e = reader(s, &r);
    if (e != hipSuccess) return e;
    if ((e = hipEventRecord(r->ev, s)) != hipSuccess) return e;
    r->read = true;
    return hipSuccess;
  }
  // Before queuing a rewrite on w: w waits, on the device, for every launch that read the buffer.
  hipError_t before_write(hipStream_t w) {
    if (have_written && writer != w) {  // and for the last rewrite, if no read came between
      const hipError_t e = hipStreamWaitEvent(w, written, 0);
      if (e != hipSuccess) return e;
    }
    for (Reader& r : readers)
      if (r.read && r.s != w) {
        const hipError_t e = hipStreamWaitEvent(w, r.ev, 0);
        if (e != hipSuccess) return e;
      }
    return hipSuccess;
  }
  // After queuing the rewrite on w: later launches on other streams wait for it.
  hipError_t after_write(hipStream_t w) {
    hipError_t e;
    if (!written && (e = hipEventCreateWithFlags(&written, hipEventDisableTiming)) != hipSuccess)
      return e;
    if ((e = hipEventRecord(written, w)) != hipSuccess) return e;
    writer = w;
    have_written = true;
    for (Reader& r : readers) {
      r.current = r.s == w;
      r.read = false;  // the rewrite on w came after each of them
    }
    return hipSuccess;
  }
  void release() {
    for (Reader& r : readers)
      if (r.ev) (void)hipEventDestroy(r.ev);
    readers.clear();
    if (written) (void)hipEventDestroy(written);
    written = nullptr;
    have_written = false;
  }

 private:
  static constexpr size_t kMaxReaders = 16;
  hipError_t reader(hipStream_t s, Reader** out) {
    for (Reader& r : readers)
      if (r.s == s) {
        *out = &r;
        return hipSuccess;
      }
    if (readers.size() >= kMaxReaders) {  // forget streams whose last read has completed
      for (size_t k = readers.size(); k-- > 0;)
        if (!readers[k].read || hipEventQuery(readers[k].ev) == hipSuccess) {
          (void)hipEventDestroy(readers[k].ev);
          readers.erase(readers.begin() + (long)k);
        }
      if (readers.size() >= kMaxReaders) {  // all busy: wait for the oldest
        const hipError_t e = hipEventSynchronize(readers.front().ev);
        if (e != hipSuccess) return e;
        (void)hipEventDestroy(readers.front().ev);
        readers.erase(readers.begin());
      }
    }
    Reader r;
    r.s = s;
    const hipError_t e = hipEventCreateWithFlags(&r.ev, hipEventDisableTiming);
    if (e != hipSuccess) return e;
    // a stream new to the buffer is ordered after the last rewrite once before_read has run
    readers.push_back(r);
    *out = &readers.back();
    return hipSuccess;
  }
};

}  // namespace sfrt

// Any HIP failure becomes SFRT_E_HIP at the boundary.
#define HIP_TRY(expr)                            \
  do {                                           \
    if ((expr) != hipSuccess) return SFRT_E_HIP; \
  } while (0)
