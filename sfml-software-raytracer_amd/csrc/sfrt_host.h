// sfrt_host.h -- host-side helpers shared by the C-ABI translation units
// (sfrt_world.cpp, sfrt_glsl.cpp, sfrt_voxel.cpp, sfrt_multi.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "sfrt.h"

namespace sfrt {

// hipFree and hipHostFree wait for the whole device: each returned only after 20 ms of work queued
// on an unrelated stream had drained (tools/gpu/probe_hostalloc.py, profiles/r6u_hip_alloc_calls.txt),
// while hipMalloc, hipHostMalloc, hipMallocAsync and hipFreeAsync did not.  So buffers that grow
// while frames run -- per-frame tables, staging, device frames -- are stream-ordered device memory
// (hipMallocAsync / hipFreeAsync behind the waits that make the old buffer idle), and a replaced
// pinned host buffer is retired until its owner is destroyed (capacities grow geometrically, so the
// retired bytes stay below the live ones).
struct RetiredHost {
  std::vector<void*> bufs;
  void add(void* h) {
    if (h) bufs.push_back(h);
  }
  void release() {
    for (void* h : bufs) (void)hipHostFree(h);
    bufs.clear();
  }
};
inline size_t grown_capacity(size_t cap, size_t need) {
  size_t c = cap > 256 ? cap : 256;
  while (c < need) c += c / 2;
  return c;
}

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
  // Room for `bytes` (after reclaim(): every earlier user has finished), waiting for no other
  // stream: the device tables reallocated in the order of s, the staging stream; the old pinned
  // copy retired (RetiredHost).
  hipError_t grow(size_t bytes, hipStream_t s) {
    if (cap >= bytes) return hipSuccess;
    const size_t c = grown_capacity(cap, bytes);
    hipError_t e;
    if (d && (e = hipFreeAsync(d, s)) != hipSuccess) return e;
    d = nullptr;
    retired.add(h);
    h = nullptr;
    cap = 0;
    if ((e = hipMallocAsync(&d, c, s)) != hipSuccess) return e;
    if ((e = hipHostMalloc(&h, c, hipHostMallocDefault)) != hipSuccess) return e;
    cap = c;
    return hipSuccess;
  }
  // The same through the launch itself: the event to pass to the kernel launch as its stop event
  // (hipExtLaunchKernelGGL: the dispatch packet's own completion signal records it, so no marker
  // packet sits between two frames -- a hipEventRecord after every launch cost the 1080p voxel
  // frame ~5 us, profiles/ab/r6_ab3), then launched_with(s) once the launch is queued on s.
  hipEvent_t launch_event() const { return ev; }
  void launched_with(hipStream_t s) {
    last = s;
    pending = true;
  }
  void release() {
    (void)hipFree(d);
    (void)hipHostFree(h);
    retired.release();
    if (ev) (void)hipEventDestroy(ev);
    d = h = nullptr;
    ev = nullptr;
    cap = 0;
    pending = false;
  }

 private:
  RetiredHost retired;
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
// synchronisation and no per-frame work.  Every launch that reads the buffer also reads a table
// slot and re-records the slot's event, which by TableSlot's rule covers every earlier user of the
// slot; so a rewrite queued on stream w is ordered after every reader by w waiting, on the device,
// for each pending slot event (and for the previous rewrite).  `written`, recorded after the
// rewrite, orders the first later launch on each other stream after it.  (A second event recorded
// after every launch, one per reading stream, had cost the 1080p voxel frame 5 us: ab/r6_ab3.)
struct SharedBuffer {
  hipEvent_t written = nullptr;
  hipStream_t writer = nullptr;
  bool have_written = false;
  std::vector<hipStream_t> current;  // other streams already ordered after the last rewrite

  // Before queuing a launch on s that reads the buffer.
  hipError_t before_read(hipStream_t s) {
    if (!have_written || s == writer) return hipSuccess;
    for (hipStream_t c : current)
      if (c == s) return hipSuccess;
    const hipError_t e = hipStreamWaitEvent(s, written, 0);
    if (e != hipSuccess) return e;
    if (current.size() >= 64) current.clear();  // (a forgotten stream only waits once more)
    current.push_back(s);
    return hipSuccess;
  }
  // Before queuing a rewrite on w: w waits for every launch that read the buffer, through the
  // table slots those launches read.
  template <int N>
  hipError_t before_write(hipStream_t w, const TableSlot (&readers)[N]) {
    if (have_written && writer != w) {
      const hipError_t e = hipStreamWaitEvent(w, written, 0);
      if (e != hipSuccess) return e;
    }
    for (const TableSlot& t : readers)
      if (t.pending && t.last != w) {
        const hipError_t e = hipStreamWaitEvent(w, t.ev, 0);
        if (e != hipSuccess) return e;
      }
    return hipSuccess;
  }
  // After queuing the rewrite on w.
  hipError_t after_write(hipStream_t w) {
    hipError_t e;
    if (!written && (e = hipEventCreateWithFlags(&written, hipEventDisableTiming)) != hipSuccess)
      return e;
    if ((e = hipEventRecord(written, w)) != hipSuccess) return e;
    writer = w;
    have_written = true;
    current.clear();
    return hipSuccess;
  }
  void release() {
    if (written) (void)hipEventDestroy(written);
    written = nullptr;
    have_written = false;
    current.clear();
  }
};

// Pinned staging for a stream-ordered upload from the caller's (pageable) memory: the bytes are
// copied into the staging buffer on the host, then to the device on a stream; the buffer is reused
// only after its last device copy has run (a host wait on that copy alone, never on the device).
struct PinnedStage {
  void* h = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  bool pending = false;

  // The staging buffer holding a copy of src[0, bytes).
  hipError_t fill(const void* src, size_t bytes, void** out) {
    const hipError_t e = take(bytes, out);
    if (e == hipSuccess) std::memcpy(*out, src, bytes);
    return e;
  }
  // The staging buffer, room for `bytes`, for the caller to write (its last copy has run).
  hipError_t take(size_t bytes, void** out) {
    hipError_t e;
    if (pending) {
      if ((e = hipEventSynchronize(ev)) != hipSuccess) return e;
      pending = false;
    }
    if (cap < bytes) {  // the old buffer retired, not freed (RetiredHost)
      const size_t c = grown_capacity(cap, bytes);
      retired.add(h);
      h = nullptr;
      cap = 0;
      if ((e = hipHostMalloc(&h, c, hipHostMallocDefault)) != hipSuccess) return e;
      cap = c;
    }
    if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
    *out = h;
    return hipSuccess;
  }
  // After the device copy from the staging buffer was queued on s.
  hipError_t copied(hipStream_t s) {
    const hipError_t e = hipEventRecord(ev, s);
    if (e == hipSuccess) pending = true;
    return e;
  }
  void release() {
    (void)hipHostFree(h);
    retired.release();
    if (ev) (void)hipEventDestroy(ev);
    h = nullptr;
    ev = nullptr;
    cap = 0;
    pending = false;
  }

 private:
  RetiredHost retired;
};

}  // namespace sfrt

// Any HIP failure becomes SFRT_E_HIP at the boundary.
#define HIP_TRY(expr)                            \
  do {                                           \
    if ((expr) != hipSuccess) return SFRT_E_HIP; \
  } while (0)
