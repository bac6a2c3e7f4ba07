// sfrt_host.h -- host-side helpers shared by the C-ABI translation units
// (sfrt_world.cpp, sfrt_glsl.cpp, sfrt_voxel.cpp, sfrt_multi.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
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

// Events recorded on a caller's stream are not used once the call returns: HIP's event calls read
// the stream an event was last recorded on, and a caller may destroy that stream once its frames
// are done (hipEventSynchronize on an event last recorded on a destroyed stream returned
// hipErrorStreamCaptureUnsupported now and then, tests/test_streams.py
// test_random_interleavings_long).  So each such event is relayed at once, while the caller's
// stream is alive, to an event recorded on a stream the object owns, which completes after it;
// only relayed events are waited on later.
struct Relay {
  hipStream_t stream = nullptr;
  hipEvent_t scratch = nullptr;
  hipError_t ensure() {
    hipError_t e;
    if (!stream && (e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking)) != hipSuccess) return e;
    if (!scratch && (e = hipEventCreateWithFlags(&scratch, hipEventDisableTiming)) != hipSuccess) return e;
    return hipSuccess;
  }
  // `to` completes after `from`, recorded just now on a caller's stream.
  hipError_t pass(hipEvent_t from, hipEvent_t to) {
    hipError_t e;
    if ((e = ensure()) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(stream, from, 0)) != hipSuccess) return e;
    return hipEventRecord(to, stream);
  }
  // `to` completes after the work queued on s so far.
  hipError_t record(hipStream_t s, hipEvent_t to) {
    hipError_t e;
    if ((e = ensure()) != hipSuccess) return e;
    if ((e = hipEventRecord(scratch, s)) != hipSuccess) return e;
    return pass(scratch, to);
  }
  void release() {
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    if (scratch) (void)hipEventDestroy(scratch);
    stream = nullptr;
    scratch = nullptr;
  }
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
  hipEvent_t ev = nullptr;     // relayed (Relay): completes after every earlier user
  hipEvent_t stop = nullptr;   // the launch's own stop event, on the caller's stream
  hipStream_t last = nullptr;  // stream of the last user (compared only, valid while pending)
  bool pending = false;
  Relay* relay = nullptr;      // the owner's (set at its creation)

  // Before restaging: every earlier user has finished with the slot.
  hipError_t reclaim() {
    hipError_t e;
    if (pending && (e = hipEventSynchronize(ev)) != hipSuccess) return e;
    pending = false;
    if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
    if (!stop && (e = hipEventCreateWithFlags(&stop, hipEventDisableTiming)) != hipSuccess) return e;
    return hipSuccess;
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
  hipEvent_t launch_event() const { return stop; }
  hipError_t launched_with(hipStream_t s) {
    const hipError_t e = relay->pass(stop, ev);
    if (e != hipSuccess) return e;
    last = s;
    pending = true;
    return hipSuccess;
  }
  void release() {
    (void)hipFree(d);
    (void)hipHostFree(h);
    retired.release();
    if (ev) (void)hipEventDestroy(ev);
    if (stop) (void)hipEventDestroy(stop);
    d = h = nullptr;
    ev = stop = nullptr;
    cap = 0;
    pending = false;
  }

 private:
  RetiredHost retired;
  hipError_t mark(hipStream_t s) {
    const hipError_t e = relay->record(s, ev);
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
  hipEvent_t written = nullptr;  // relayed (Relay): the rewrite may run on a caller's stream
  hipStream_t writer = nullptr;  // compared only
  bool have_written = false;
  Relay* relay = nullptr;        // the owner's (set at its creation)
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
    if ((e = relay->record(w, written)) != hipSuccess) return e;
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
// The copy runs on a stream the owner keeps alive (its own): `ev` is waited on later (Relay).
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

namespace sfrt {
// With SFRT_DEBUG set in the environment, a failing HIP call names itself on stderr (the ABI
// returns only SFRT_E_HIP).
inline void report_hip_error(hipError_t e, const char* expr, const char* file, int line) {
  static const bool on = std::getenv("SFRT_DEBUG") != nullptr;
  if (on) std::fprintf(stderr, "sfrt: %s:%d: %s -> %s\n", file, line, expr, hipGetErrorName(e));
}
}  // namespace sfrt

// Any HIP failure becomes SFRT_E_HIP at the boundary.
#define HIP_TRY(expr)                                                 \
  do {                                                                \
    const hipError_t hip_try_e = (expr);                              \
    if (hip_try_e != hipSuccess) {                                    \
      sfrt::report_hip_error(hip_try_e, #expr, __FILE__, __LINE__);   \
      return SFRT_E_HIP;                                              \
    }                                                                 \
  } while (0)
