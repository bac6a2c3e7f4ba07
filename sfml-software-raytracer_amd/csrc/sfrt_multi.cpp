// sfrt_multi.cpp -- one frame over several GPUs of a node, behind the C ABI
// (include/sfrt.h "One frame over several GPUs").
//
// The reference fills one sf::Image from one C++ process (Source.cpp:17-28,
// 47-52: eight RenderThreads, each UpdateImage(&gameImage, num, 8, cycle, 4),
// SphereWorld.cpp:94-98).  Here the same process fills it on n GPUs: one
// sfrt_world per device renders a contiguous row band with global row indices
// (sfrt_world_render_band), and the bands travel to devices[0] -- the path's one
// exchange step -- by RCCL (one ncclGather for equal bands, grouped
// ncclSend/ncclRecv otherwise) or by peer copies over xGMI.  Per rank: a render
// stream, a copy stream (RCCL's stream), two band buffers, so the transfer of
// frame k overlaps the render of frame k + 1.  Bands of alpha-binary worlds cross
// the link packed (band_pack.hip: 3.125 B per pixel instead of 4) and are unpacked
// into the frame on devices[0].
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "sfrt.h"
#include "sfrt_host.h"

namespace {

// RCCL entry points, resolved from librccl.so.1 by the first RCCL context (a
// process that already loaded RCCL -- e.g. torch's copy -- gets that one), so
// the single-GPU library carries no RCCL dependency.  A test may name another library
// with the same C API instead, explicitly and before that first context
// (sfrt_multi_use_test_transport: the tests' loopback transport,
// tests/native/rccl_loopback.cpp, which -- unlike RCCL -- accepts a device listed twice, so
// the RCCL branch below runs with n > 1 on a one-GPU box).  Nothing in the environment
// selects it, and sfrt_multi_transport_library reports which library is in use.
struct Rccl {
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGather) gather = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  bool ok = false;
  bool override_lib = false;  // a test transport, not librccl
  std::string name;           // the library the entry points came from
};

std::mutex g_rccl_mu;
std::string g_test_transport;  // sfrt_multi_use_test_transport
bool g_rccl_resolved = false;

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    std::string alt;
    {
      std::lock_guard<std::mutex> lk(g_rccl_mu);
      alt = g_test_transport;
      g_rccl_resolved = true;
    }
    void* h = nullptr;
    if (!alt.empty()) {
      h = dlopen(alt.c_str(), RTLD_NOW | RTLD_LOCAL);
      r.override_lib = true;
      r.name = alt;
    } else {
      r.name = "librccl.so.1";
      h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
      if (!h) {
        r.name = "librccl.so";
        h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
      }
    }
    if (!h) return;
    r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
    r.gather = (decltype(r.gather))dlsym(h, "ncclGather");
    r.send = (decltype(r.send))dlsym(h, "ncclSend");
    r.recv = (decltype(r.recv))dlsym(h, "ncclRecv");
    r.ok = r.comm_init_all && r.comm_destroy && r.group_start && r.group_end && r.gather &&
           r.send && r.recv;
  });
  return r;
}

#define NCCL_TRY(expr)                              \
  do {                                              \
    if ((expr) != ncclSuccess) return SFRT_E_HIP;   \
  } while (0)

constexpr int kAlign = 8;  // rows per kernel tile (bands.py ALIGN)

// bands.py root_weighted_spans, restated (the Python tuner and this agree row for row).
void split_rows(int height, int n, double factor, int* row0, int* rows) {
  auto equal = [&] {
    for (int r = 0; r < n; r++) {
      row0[r] = (int)((int64_t)r * height / n);
      rows[r] = (int)((int64_t)(r + 1) * height / n) - row0[r];
    }
  };
  if (n == 1 || factor == 1.0) return equal();
  int other = (int)((double)height / ((double)(n - 1) + factor));
  other -= other % kAlign;
  if (other <= 0 || (int64_t)other * (n - 1) >= height) return equal();
  rows[0] = height - (n - 1) * other;
  row0[0] = 0;
  for (int r = 1; r < n; r++) {
    row0[r] = rows[0] + (r - 1) * other;
    rows[r] = other;
  }
}

// bands.py cost_weighted_spans, restated (row for row the same partition): rank 0 gets
// `factor` shares of the frame's march cost, every other rank one share (SURVEY 8e
// "Balance": cost-weighted band edges), with band edges on 8-row tile boundaries (or
// the last row).  Each edge is the boundary whose cost prefix (a double sum over the rows
// in order) is closest to its target, never before the previous edge.  Costs that are
// negative, non-finite or sum to zero give split_rows' partition.
void cost_rows(const float* cost, int height, int n, double factor, int* row0, int* rows) {
  std::vector<int> at;  // candidate edges 0, 8, 16, ..., height
  std::vector<double> pre;
  double sum = 0.0;
  bool ok = true;
  for (int j = 0; j <= height; j++) {
    if (j % kAlign == 0 || j == height) {
      at.push_back(j);
      pre.push_back(sum);
    }
    if (j < height) {
      const double c = (double)cost[j];
      if (!(c >= 0.0) || !std::isfinite(c)) ok = false;
      sum += c;
    }
  }
  if (n == 1 || !ok || !(sum > 0.0)) return split_rows(height, n, factor, row0, rows);
  const double denom = (double)(n - 1) + factor;
  size_t i = 0;
  row0[0] = 0;
  for (int r = 1; r < n; r++) {
    const double target = sum * (factor + (double)(r - 1)) / denom;
    size_t k = i;
    while (k + 1 < at.size() && pre[k] < target) k++;
    if (k > i && pre[k] - target > target - pre[k - 1]) k--;
    i = k;
    row0[r] = at[i];
    rows[r - 1] = row0[r] - row0[r - 1];
  }
  rows[n - 1] = height - row0[n - 1];
}

struct Rank {
  int device = 0;
  sfrt_world* world = nullptr;
  hipStream_t render_s = nullptr, copy_s = nullptr;
  uint8_t* band[2] = {};
  size_t band_bytes = 0;
  uint8_t* packed[2] = {};  // this rank's packed band (its device)
  uint8_t* stage[2] = {};   // where it lands on devices[0]
  size_t packed_bytes = 0;
  hipEvent_t rendered[2] = {}, copied[2] = {};
  bool copy_pending[2] = {};
  ncclComm_t comm = nullptr;
  // Replaced buffers, freed with the object: hipFree waits for the whole device (sfrt_host.h),
  // and the capacities grow geometrically, so these stay below the live ones.
  std::vector<void*> retired;        // on its device
  std::vector<void*> retired_stage;  // on devices[0]
};

}  // namespace

struct sfrt_multi {
  std::vector<Rank> ranks;
  int transport = SFRT_MULTI_PEER;
  std::vector<int> rows_set;  // sfrt_multi_set_bands (empty: equal split)
  std::vector<int> last_rows; // the bands of the last render (sfrt_multi_row_costs)
  int transfer = SFRT_TRANSFER_AUTO;
  bool last_packed = false;   // the format of the last render's transfers
  hipEvent_t unpacked[2] = {};  // devices[0]: the unpacks that read stage[slot]
  bool unpack_pending[2] = {};
  int64_t k = 0;              // frames rendered (band buffer k % 2)
  hipEvent_t start = nullptr;  // on devices[0]: the caller's stream position at render
  hipStream_t out_s = nullptr;  // devices[0]: update_image's frame stream
  uint8_t* d_frame = nullptr;   // devices[0]: update_image's frame
  size_t d_frame_bytes = 0;
  std::vector<void*> retired_frames;  // replaced d_frame buffers (see Rank::retired)
  std::mutex mu;

  ~sfrt_multi() {
    for (Rank& r : ranks) {
      sfrt::DeviceGuard g(r.device);
      if (r.render_s) (void)hipStreamSynchronize(r.render_s);
      if (r.copy_s) (void)hipStreamSynchronize(r.copy_s);
    }
    for (Rank& r : ranks)
      if (r.comm) (void)rccl().comm_destroy(r.comm);
    for (Rank& r : ranks) {
      sfrt::DeviceGuard g(r.device);
      for (int q = 0; q < 2; q++) {
        (void)hipFree(r.band[q]);
        (void)hipFree(r.packed[q]);
        if (r.rendered[q]) (void)hipEventDestroy(r.rendered[q]);
        if (r.copied[q]) (void)hipEventDestroy(r.copied[q]);
      }
      for (void* p : r.retired) (void)hipFree(p);
      if (r.render_s) (void)hipStreamDestroy(r.render_s);
      if (r.copy_s) (void)hipStreamDestroy(r.copy_s);
      sfrt_world_destroy(r.world);
    }
    if (!ranks.empty()) {
      sfrt::DeviceGuard g(ranks[0].device);
      for (Rank& r : ranks) {
        for (int q = 0; q < 2; q++) (void)hipFree(r.stage[q]);
        for (void* p : r.retired_stage) (void)hipFree(p);
      }
      for (int q = 0; q < 2; q++)
        if (unpacked[q]) (void)hipEventDestroy(unpacked[q]);
      if (out_s) {
        (void)hipStreamSynchronize(out_s);
        (void)hipStreamDestroy(out_s);
      }
      (void)hipFree(d_frame);
      for (void* p : retired_frames) (void)hipFree(p);
      if (start) (void)hipEventDestroy(start);
    }
  }

  template <class F>
  int each(F&& fn) {
    for (Rank& r : ranks) {
      const int rc = fn(r.world);
      if (rc) return rc;
    }
    return SFRT_OK;
  }

  int spans(int height, std::vector<int>& row0, std::vector<int>& rows) const {
    const int n = (int)ranks.size();
    row0.assign(n, 0);
    rows.assign(n, 0);
    if (rows_set.empty()) {
      split_rows(height, n, 1.0, row0.data(), rows.data());
      return SFRT_OK;
    }
    int64_t at = 0;
    for (int r = 0; r < n; r++) {
      row0[r] = (int)at;
      rows[r] = rows_set[r];
      at += rows_set[r];
    }
    return at == height ? SFRT_OK : SFRT_E_INVALID;
  }

  // Packed transfer buffers for bands of rows[r] x width pixels: rank r's packed[2] on
  // its device, stage[2] on devices[0].  Growing them first drains this object's streams; the
  // old buffers are retired (Rank::retired), not freed.
  int packed_buffers(const std::vector<int>& rows, int width) {
    for (size_t r = 1; r < ranks.size(); r++) {
      Rank& R = ranks[r];
      const int64_t b = sfrt_band_packed_bytes((int64_t)rows[r] * width);
      if (b < 0) return SFRT_E_INVALID;
      if ((size_t)b <= R.packed_bytes) continue;
      for (Rank& Q : ranks) {
        sfrt::DeviceGuard g(Q.device);
        HIP_TRY(hipStreamSynchronize(Q.render_s));
        HIP_TRY(hipStreamSynchronize(Q.copy_s));
      }
      const size_t cap = sfrt::grown_capacity(R.packed_bytes, (size_t)b);
      {
        sfrt::DeviceGuard g(R.device);
        for (int q = 0; q < 2; q++) {
          if (R.packed[q]) R.retired.push_back(R.packed[q]);
          R.packed[q] = nullptr;
        }
        R.packed_bytes = 0;
        for (int q = 0; q < 2; q++) HIP_TRY(hipMalloc(&R.packed[q], cap));
      }
      {
        sfrt::DeviceGuard g(ranks[0].device);
        for (int q = 0; q < 2; q++) {
          if (R.stage[q]) R.retired_stage.push_back(R.stage[q]);
          R.stage[q] = nullptr;
        }
        for (int q = 0; q < 2; q++) HIP_TRY(hipMalloc(&R.stage[q], cap));
      }
      R.packed_bytes = cap;
    }
    return SFRT_OK;
  }

  // Queue one frame: renders after `stream`'s queued work, complete at its next position.
  int render(uint8_t* frame, int64_t pitch, hipStream_t stream) {
    int width = 0, height = 0;
    int rc = sfrt_world_get_size(ranks[0].world, &width, &height);
    if (rc) return rc;
    if (pitch != (int64_t)width * 4) return SFRT_E_INVALID;  // bands are contiguous rows
    std::vector<int> row0, rows;
    if ((rc = spans(height, row0, rows))) return rc;
    last_rows = rows;
    const int n = (int)ranks.size();
    bool equal = true;
    for (int r = 1; r < n; r++) equal = equal && rows[r] == rows[0];
    equal = equal && rows[0] > 0;
    const int slot = (int)(k & 1);
    bool packed = false;
    if (n > 1 && transfer != SFRT_TRANSFER_RGBA) {
      bool binary = true;
      for (Rank& R : ranks) {
        int b = 0;
        if ((rc = sfrt_world_alpha_binary(R.world, &b))) return rc;
        binary = binary && b;
      }
      if (transfer == SFRT_TRANSFER_PACKED && !binary) return SFRT_E_INVALID;
      packed = binary;
    }
    if (packed && (rc = packed_buffers(rows, width))) return rc;
    last_packed = packed;
    {
      sfrt::DeviceGuard g(ranks[0].device);
      HIP_TRY(hipEventRecord(start, stream));
    }
    // renders: rank 0 straight into its rows of the frame, the others into a band buffer
    for (int r = 0; r < n; r++) {
      Rank& R = ranks[r];
      sfrt::DeviceGuard g(R.device);
      HIP_TRY(hipStreamWaitEvent(R.render_s, start, 0));
      if (rows[r] == 0) continue;
      uint8_t* target = frame;
      if (r > 0) {
        const size_t bytes = (size_t)rows[r] * (size_t)pitch;
        if (R.band_bytes < bytes) {
          HIP_TRY(hipStreamSynchronize(R.render_s));
          HIP_TRY(hipStreamSynchronize(R.copy_s));
          const size_t cap = sfrt::grown_capacity(R.band_bytes, bytes);
          for (int q = 0; q < 2; q++) {
            if (R.band[q]) R.retired.push_back(R.band[q]);  // not freed: Rank::retired
            R.band[q] = nullptr;
            R.copy_pending[q] = false;
          }
          R.band_bytes = 0;
          for (int q = 0; q < 2; q++) HIP_TRY(hipMalloc(&R.band[q], cap));
          R.band_bytes = cap;
        }
        // the transfer that last read this buffer must be done before it is overwritten
        if (R.copy_pending[slot]) HIP_TRY(hipStreamWaitEvent(R.render_s, R.copied[slot], 0));
        target = R.band[slot];
      }
      if ((rc = sfrt_world_render_band(R.world, target, pitch, row0[r], rows[r], R.render_s)))
        return rc;
      if (packed && r > 0 &&
          (rc = sfrt_band_pack(target, (int64_t)rows[r] * width, R.packed[slot], R.render_s)))
        return rc;
      HIP_TRY(hipEventRecord(R.rendered[slot], R.render_s));
      HIP_TRY(hipStreamWaitEvent(R.copy_s, R.rendered[slot], 0));
    }
    // the exchange step
    if (transport == SFRT_MULTI_RCCL) {
      const Rccl& nc = rccl();
      NCCL_TRY(nc.group_start());
      for (int r = 0; r < n; r++) {
        Rank& R = ranks[r];
        if (rows[r] == 0) continue;
        const size_t count = (size_t)rows[r] * (size_t)pitch;
        uint8_t* send = r == 0 ? frame : R.band[slot];
        if (packed) {  // rank 0's rows are already in the frame
          if (r > 0) {
            const size_t bytes = (size_t)sfrt_band_packed_bytes((int64_t)rows[r] * width);
            if (nc.send(R.packed[slot], bytes, ncclUint8, 0, R.comm, R.copy_s) != ncclSuccess ||
                nc.recv(R.stage[slot], bytes, ncclUint8, r, ranks[0].comm, ranks[0].copy_s) !=
                    ncclSuccess) {
              (void)nc.group_end();
              return SFRT_E_HIP;
            }
          }
        } else if (equal) {  // in place on the root: its send buffer is frame + 0 * count
          if (nc.gather(send, r == 0 ? frame : send, count, ncclUint8, 0, R.comm, R.copy_s) !=
              ncclSuccess) {
            (void)nc.group_end();
            return SFRT_E_HIP;
          }
        } else if (r > 0) {
          if (nc.send(send, count, ncclUint8, 0, R.comm, R.copy_s) != ncclSuccess ||
              nc.recv(frame + (size_t)row0[r] * (size_t)pitch, count, ncclUint8, r, ranks[0].comm,
                      ranks[0].copy_s) != ncclSuccess) {
            (void)nc.group_end();
            return SFRT_E_HIP;
          }
        }
      }
      NCCL_TRY(nc.group_end());
      if (packed) {  // after the receives on the root's copy stream
        sfrt::DeviceGuard g(ranks[0].device);
        for (int r = 1; r < n; r++)
          if (rows[r] > 0 &&
              (rc = sfrt_band_unpack(ranks[r].stage[slot], (int64_t)rows[r] * width,
                                     frame + (size_t)row0[r] * (size_t)pitch, ranks[0].copy_s)))
            return rc;
      }
      for (int r = 0; r < n; r++) {
        Rank& R = ranks[r];
        sfrt::DeviceGuard g(R.device);
        HIP_TRY(hipEventRecord(R.copied[slot], R.copy_s));
        R.copy_pending[slot] = true;
      }
      // the root's copy stream saw its own render and every receive
      sfrt::DeviceGuard g(ranks[0].device);
      HIP_TRY(hipStreamWaitEvent(stream, ranks[0].copied[slot], 0));
    } else {
      for (int r = 1; r < n; r++) {
        Rank& R = ranks[r];
        if (rows[r] == 0) continue;
        sfrt::DeviceGuard g(R.device);
        if (packed) {
          // stage[slot] is free once the unpacks of two frames back have read it
          if (unpack_pending[slot]) HIP_TRY(hipStreamWaitEvent(R.copy_s, unpacked[slot], 0));
          HIP_TRY(hipMemcpyPeerAsync(R.stage[slot], ranks[0].device, R.packed[slot], R.device,
                                     (size_t)sfrt_band_packed_bytes((int64_t)rows[r] * width),
                                     R.copy_s));
        } else {
          HIP_TRY(hipMemcpyPeerAsync(frame + (size_t)row0[r] * (size_t)pitch, ranks[0].device,
                                     R.band[slot], R.device, (size_t)rows[r] * (size_t)pitch,
                                     R.copy_s));
        }
        HIP_TRY(hipEventRecord(R.copied[slot], R.copy_s));
        R.copy_pending[slot] = true;
      }
      sfrt::DeviceGuard g(ranks[0].device);
      if (rows[0] > 0) HIP_TRY(hipStreamWaitEvent(stream, ranks[0].rendered[slot], 0));
      if (packed) {  // unpack on the root's copy stream, after every band landed
        hipStream_t us = ranks[0].copy_s;
        for (int r = 1; r < n; r++)
          if (rows[r] > 0) HIP_TRY(hipStreamWaitEvent(us, ranks[r].copied[slot], 0));
        for (int r = 1; r < n; r++)
          if (rows[r] > 0 &&
              (rc = sfrt_band_unpack(ranks[r].stage[slot], (int64_t)rows[r] * width,
                                     frame + (size_t)row0[r] * (size_t)pitch, us)))
            return rc;
        HIP_TRY(hipEventRecord(unpacked[slot], us));
        unpack_pending[slot] = true;
        HIP_TRY(hipStreamWaitEvent(stream, unpacked[slot], 0));
      } else {
        for (int r = 1; r < n; r++)
          if (rows[r] > 0) HIP_TRY(hipStreamWaitEvent(stream, ranks[r].copied[slot], 0));
      }
    }
    k++;
    return SFRT_OK;
  }

  int check() {
    int first = SFRT_OK;
    for (Rank& r : ranks) {
      sfrt::DeviceGuard g(r.device);
      const int rc = sfrt_world_check(r.world, r.render_s);
      if (rc && !first) first = rc;
      if (hipStreamSynchronize(r.copy_s) != hipSuccess && !first) first = SFRT_E_HIP;
    }
    return first;
  }
};

extern "C" {

int sfrt_multi_use_test_transport(const char* library_path) {
  if (!library_path || !*library_path) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (g_rccl_resolved) return SFRT_E_INVALID;  // the process already resolved its transport
  g_test_transport = library_path;
  return SFRT_OK;
}

int sfrt_multi_transport_library(char* buf, int size) {
  if (!buf || size <= 0) return SFRT_E_INVALID;
  bool resolved;
  {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    resolved = g_rccl_resolved;
  }
  std::string name;
  if (resolved) {
    const Rccl& r = rccl();
    name = (r.override_lib ? "test:" : "") + r.name + (r.ok ? "" : " (not loaded)");
  }
  std::snprintf(buf, (size_t)size, "%s", name.c_str());
  return (int)name.size() < size ? SFRT_OK : SFRT_E_INVALID;
}

int sfrt_multi_create(const int* hip_devices, int n, int transport, sfrt_multi** out) {
  if (!out) return SFRT_E_INVALID;
  *out = nullptr;
  if (!hip_devices || n <= 0 || n > 64 || transport < SFRT_MULTI_AUTO || transport > SFRT_MULTI_PEER)
    return SFRT_E_INVALID;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) return SFRT_E_HIP;
  bool distinct = true;
  for (int r = 0; r < n; r++) {
    if (hip_devices[r] < 0 || hip_devices[r] >= count) return SFRT_E_INVALID;
    for (int q = 0; q < r; q++) distinct = distinct && hip_devices[q] != hip_devices[r];
  }
  if (transport == SFRT_MULTI_AUTO) transport = distinct ? SFRT_MULTI_RCCL : SFRT_MULTI_PEER;
  // RCCL refuses a device listed twice (the tests' loopback transport does not)
  if (transport == SFRT_MULTI_RCCL && (!rccl().ok || (!distinct && !rccl().override_lib)))
    return SFRT_E_INVALID;
  sfrt_multi* m = new sfrt_multi();
  m->transport = transport;
  m->ranks.resize((size_t)n);
  for (int r = 0; r < n; r++) {
    Rank& R = m->ranks[r];
    R.device = hip_devices[r];
    if (sfrt_world_create(R.device, &R.world) != SFRT_OK) {
      delete m;
      return SFRT_E_HIP;
    }
    sfrt::DeviceGuard g(R.device);
    bool ok = hipStreamCreateWithFlags(&R.render_s, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&R.copy_s, hipStreamNonBlocking) == hipSuccess;
    for (int q = 0; q < 2 && ok; q++)
      ok = hipEventCreateWithFlags(&R.rendered[q], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&R.copied[q], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
      delete m;
      return SFRT_E_HIP;
    }
  }
  {
    sfrt::DeviceGuard g(hip_devices[0]);
    if (hipEventCreateWithFlags(&m->start, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m->unpacked[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m->unpacked[1], hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&m->out_s, hipStreamNonBlocking) != hipSuccess) {
      delete m;
      return SFRT_E_HIP;
    }
  }
  if (transport == SFRT_MULTI_RCCL) {
    std::vector<ncclComm_t> comms((size_t)n, nullptr);
    if (rccl().comm_init_all(comms.data(), n, hip_devices) != ncclSuccess) {
      delete m;
      return SFRT_E_HIP;
    }
    for (int r = 0; r < n; r++) m->ranks[r].comm = comms[r];
  }
  *out = m;
  return SFRT_OK;
}

void sfrt_multi_destroy(sfrt_multi* m) { delete m; }

int sfrt_multi_count(const sfrt_multi* m, int* n, int* transport) {
  if (!m || !n || !transport) return SFRT_E_INVALID;
  *n = (int)m->ranks.size();
  *transport = m->transport;
  return SFRT_OK;
}

int sfrt_multi_world(sfrt_multi* m, int rank, sfrt_world** out) {
  if (!m || !out || rank < 0 || rank >= (int)m->ranks.size()) return SFRT_E_INVALID;
  *out = m->ranks[rank].world;
  return SFRT_OK;
}

int sfrt_multi_set_size(sfrt_multi* m, int width, int height) {
  if (!m) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  return m->each([&](sfrt_world* w) { return sfrt_world_set_size(w, width, height); });
}

int sfrt_multi_set_camera(sfrt_multi* m, const sfrt_camera* cam) {
  if (!m) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  return m->each([&](sfrt_world* w) { return sfrt_world_set_camera(w, cam); });
}

int sfrt_multi_load_texture(sfrt_multi* m, int slot, const uint8_t* rgba, int tex_w, int tex_h) {
  if (!m) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  return m->each([&](sfrt_world* w) { return sfrt_world_load_texture(w, slot, rgba, tex_w, tex_h); });
}

int sfrt_multi_set_spheres(sfrt_multi* m, const sfrt_sphere* spheres, int count) {
  if (!m) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  return m->each([&](sfrt_world* w) { return sfrt_world_set_spheres(w, spheres, count); });
}

int sfrt_multi_add_sphere(sfrt_multi* m, float x, float y, float z, float radius) {
  if (!m) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  return m->each([&](sfrt_world* w) { return sfrt_world_add_sphere(w, x, y, z, radius); });
}

int sfrt_multi_update_spheres(sfrt_multi* m) {
  if (!m) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  return m->each([&](sfrt_world* w) { return sfrt_world_update_spheres(w); });
}

int sfrt_multi_set_sphere_textures(sfrt_multi* m, const int32_t* slots, int count) {
  if (!m) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  return m->each([&](sfrt_world* w) { return sfrt_world_set_sphere_textures(w, slots, count); });
}

int sfrt_multi_set_option(sfrt_multi* m, int option, int value) {
  if (!m) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  return m->each([&](sfrt_world* w) { return sfrt_world_set_option(w, option, value); });
}

int sfrt_multi_set_transfer(sfrt_multi* m, int format) {
  if (!m || format < SFRT_TRANSFER_AUTO || format > SFRT_TRANSFER_PACKED) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  m->transfer = format;
  return SFRT_OK;
}

int sfrt_multi_get_transfer(sfrt_multi* m, int* format, int* last_packed) {
  if (!m || !format || !last_packed) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  *format = m->transfer;
  *last_packed = m->last_packed ? 1 : 0;
  return SFRT_OK;
}

int sfrt_multi_set_bands(sfrt_multi* m, const int* rows, int n) {
  if (!m) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  if (!rows) {
    m->rows_set.clear();
    return SFRT_OK;
  }
  if (n != (int)m->ranks.size()) return SFRT_E_INVALID;
  for (int r = 0; r < n; r++)
    if (rows[r] < 0) return SFRT_E_INVALID;
  m->rows_set.assign(rows, rows + n);
  return SFRT_OK;
}

int sfrt_multi_bands(int height, int n, float root_factor, int* row0, int* rows) {
  if (height < 0 || n <= 0 || !row0 || !rows || !std::isfinite(root_factor) || root_factor <= 0.0f)
    return SFRT_E_INVALID;
  split_rows(height, n, (double)root_factor, row0, rows);
  return SFRT_OK;
}

int sfrt_multi_cost_bands(const float* row_cost, int height, int n, float root_factor, int* row0,
                          int* rows) {
  if (height < 0 || n <= 0 || !row0 || !rows || (height > 0 && !row_cost) ||
      !std::isfinite(root_factor) || root_factor <= 0.0f)
    return SFRT_E_INVALID;
  cost_rows(row_cost, height, n, (double)root_factor, row0, rows);
  return SFRT_OK;
}

int sfrt_multi_row_costs(sfrt_multi* m, float* costs, int height) {
  if (!m || height < 0 || (height > 0 && !costs)) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  std::vector<char> seen((size_t)height, 0);
  for (size_t q = 0; q < m->ranks.size(); q++) {
    auto& R = m->ranks[q];
    if (q < m->last_rows.size() && m->last_rows[q] == 0) continue;  // rendered nothing
    int r0 = 0, nr = 0, w = 0, h = 0;
    int rc = sfrt_world_get_size(R.world, &w, &h);
    if (rc) return rc;
    if (h != height) return SFRT_E_INVALID;
    std::vector<float> c((size_t)height);
    if ((rc = sfrt_world_row_costs(R.world, c.data(), height, &r0, &nr))) return rc;
    if (r0 < 0 || nr < 0 || (int64_t)r0 + nr > height) return SFRT_E_INVALID;
    for (int j = 0; j < nr; j++) {
      costs[r0 + j] = c[(size_t)j];
      seen[(size_t)(r0 + j)] = 1;
    }
  }
  for (char v : seen)
    if (!v) return SFRT_E_INVALID;  // some row was not in any rank's last band
  return SFRT_OK;
}

int sfrt_multi_balance(sfrt_multi* m, float root_factor) {
  if (!m || !std::isfinite(root_factor) || root_factor <= 0.0f) return SFRT_E_INVALID;
  int width = 0, height = 0;
  int rc = sfrt_world_get_size(m->ranks[0].world, &width, &height);
  if (rc) return rc;
  std::vector<float> cost((size_t)height);
  if ((rc = sfrt_multi_row_costs(m, cost.data(), height))) return rc;
  const int n = (int)m->ranks.size();
  std::vector<int> row0((size_t)n), rows((size_t)n);
  cost_rows(cost.data(), height, n, (double)root_factor, row0.data(), rows.data());
  return sfrt_multi_set_bands(m, rows.data(), n);
}

int sfrt_multi_render(sfrt_multi* m, void* dev_frame, int64_t pitch_bytes, void* hip_stream) {
  if (!m || !dev_frame) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  return m->render((uint8_t*)dev_frame, pitch_bytes, (hipStream_t)hip_stream);
}

int sfrt_multi_check(sfrt_multi* m) {
  if (!m) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  return m->check();
}

int sfrt_multi_update_image(sfrt_multi* m, uint8_t* pixels) {
  if (!m || !pixels) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(m->mu);
  int width = 0, height = 0;
  int rc = sfrt_world_get_size(m->ranks[0].world, &width, &height);
  if (rc) return rc;
  const size_t bytes = (size_t)width * (size_t)height * 4;
  sfrt::DeviceGuard g(m->ranks[0].device);
  if (m->d_frame_bytes < bytes) {
    HIP_TRY(hipStreamSynchronize(m->out_s));
    if (m->d_frame) m->retired_frames.push_back(m->d_frame);  // not freed: Rank::retired
    m->d_frame = nullptr;
    m->d_frame_bytes = 0;
    const size_t cap = sfrt::grown_capacity(0, bytes);
    HIP_TRY(hipMalloc(&m->d_frame, cap));
    m->d_frame_bytes = cap;
  }
  if ((rc = m->render(m->d_frame, (int64_t)width * 4, m->out_s))) return rc;
  HIP_TRY(hipMemcpyAsync(pixels, m->d_frame, bytes, hipMemcpyDeviceToHost, m->out_s));
  HIP_TRY(hipStreamSynchronize(m->out_s));
  return m->check();
}

}  // extern "C"
