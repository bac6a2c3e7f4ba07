// sfrt_world.cpp -- host side of the drop-in: a C++ mirror of the scene state
// that SphereWorld::UpdateImage reads, the per-frame preparation the kernel
// needs, and the extern "C" boundary declared in include/sfrt.h.
//
// Reference interface mirrored (paths under /root/reference/Raytracing/):
//   SphereWorld::width/height/cam     SphereWorld.h:50-52 (defaults 320x180, fov 75/47 deg)
//   SphereWorld::SphereWorld          SphereWorld.cpp:43-77 (fov -> radians :72-73)
//   SphereWorld::AddSphere            SphereWorld.cpp:177-190
//   SphereWorld::UpdateSpheres (sort) SphereWorld.cpp:199-212
//   SphereWorld::UpdateImage          SphereWorld.cpp:83-112
//   textures[0]                       SphereWorld.h:74, SphereWorld.cpp:52
// Compiled with -ffp-contract=off: every float expression below is
// evaluated exactly as the reference writes it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <utility>
#include <vector>

#include "sfrt.h"
#include "sfrt_host.h"
#include "sfrt_math.h"
#include "sfrt_sched.h"
#include "sfrt_trace.h"

#pragma clang fp contract(off)


namespace {

constexpr float kPI = 3.1415926535f;  // SphereWorld.h:6

struct V3 {
  float x, y, z;
};
inline V3 vsub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
// SphereWorld.cpp:340-343
inline float vlength(V3 v) { return std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z); }
// SphereWorld.cpp:27-31
inline V3 rot_x(V3 v, float amount) {
  const float s = std::sin(amount);
  const float c = std::cos(amount);
  return {v.x, v.y * c - v.z * s, v.y * s + v.z * c};
}
// SphereWorld.cpp:32-36
inline V3 rot_y(V3 v, float amount) {
  const float s = std::sin(amount);
  const float c = std::cos(amount);
  return {v.x * c + v.z * s, v.y, -v.x * s + v.z * c};
}
inline V3 center(const sfrt_sphere& s) { return {s.x, s.y, s.z}; }

bool finite3(const float* v) { return std::isfinite(v[0]) && std::isfinite(v[1]) && std::isfinite(v[2]); }
bool sphere_ok(const sfrt_sphere& s) {
  return std::isfinite(s.x) && std::isfinite(s.y) && std::isfinite(s.z) && std::isfinite(s.radius) &&
         s.radius > 0.0f;
}

// Stable insertion by |c - cam| + r, inserted after equal keys (SphereWorld.cpp:201-212).
// Returns the permutation (new position -> old index).
std::vector<size_t> sort_spheres(std::vector<sfrt_sphere>& spheres, V3 cam) {
  std::vector<sfrt_sphere> temp = spheres;
  std::vector<size_t> order;
  spheres.clear();
  for (size_t k = 0; k < temp.size(); k++) {
    const sfrt_sphere& t = temp[k];
    const float dist = vlength(vsub(center(t), cam)) + t.radius;
    size_t ins = 0;
    for (size_t j = 0; j < spheres.size(); j++) {
      if (dist < vlength(vsub(center(spheres[j]), cam)) + spheres[j].radius) break;
      ins++;
    }
    spheres.insert(spheres.begin() + (long)ins, t);
    order.insert(order.begin() + (long)ins, k);
  }
  return order;
}

template <class T>
void permute(std::vector<T>& v, const std::vector<size_t>& order) {
  std::vector<T> out(order.size());
  for (size_t i = 0; i < order.size(); i++) out[i] = v[order[i]];
  v.swap(out);
}

bool passes(float r, float s) { return r - std::sqrt(s) > 0.01f; }  // SphereWorld.cpp:365-366

// Smallest binary32 s >= 0 for which the reference test fails; the test is
// monotone in s (sqrtf and the subtraction are monotone), so
// passes(r, s) <=> s < threshold for every s >= 0 (and NaN s fails both).
float pass_threshold(float r) {
  if (!passes(r, 0.0f)) return 0.0f;
  uint32_t lo = 0, hi = 0x7f800000u;  // passes(lo), !passes(hi = +inf)
  while (hi - lo > 1) {
    const uint32_t mid = lo + (hi - lo) / 2;
    float s;
    std::memcpy(&s, &mid, 4);
    if (passes(r, s)) lo = mid; else hi = mid;
  }
  float t;
  std::memcpy(&t, &hi, 4);
  return t;
}

}  // namespace

struct sfrt_world {
  int device = 0;
  // --- SphereWorld state read by UpdateImage ---
  int width = 320;   // SphereWorld.h:50
  int height = 180;  // SphereWorld.h:51
  sfrt_camera cam{};
  std::vector<sfrt_sphere> spheres;
  // Per-sphere texture slot, parallel to `spheres` (the "all textures" extension
  // of SURVEY 8d config 3; 0 everywhere = the reference, textures[0]).
  std::vector<int32_t> sphere_tex;
  std::vector<uint8_t> tex_host[SFRT_TEXTURE_SLOTS];
  int tex_w[SFRT_TEXTURE_SLOTS] = {};
  int tex_h[SFRT_TEXTURE_SLOTS] = {};
  bool tex_alpha01[SFRT_TEXTURE_SLOTS] = {};  // every texel's alpha is 0 or 255
  uint32_t tex_off[SFRT_TEXTURE_SLOTS] = {};  // texel offset of each slot in the atlas
  int cull = 1;
  int rays = 0;           // SFRT_OPT_RAYS_PER_LANE (0 = automatic)
  int tile_order_on = 1;  // SFRT_OPT_TILE_ORDER
  // --- device resources ---
  hipStream_t stream = nullptr;
  uint32_t* d_tex = nullptr;  // texture atlas: every loaded slot, back to back
  size_t d_tex_texels = 0;
  // A new texture goes into a new atlas, uploaded on `stream` from pinned staging; launches
  // queued earlier keep reading the old one (its pointer is in their arguments), launches queued
  // later on another stream wait for the upload once (tex_written).  The old atlases are freed
  // once the device has drained anyway (the destructor), or in one sweep per kRetiredTexBytes.
  sfrt::SharedBuffer tex_written;
  sfrt::PinnedStage tex_stage;
  std::vector<void*> retired_tex;
  size_t retired_tex_bytes = 0;
  static constexpr size_t kRetiredTexBytes = 64u << 20;
  int* d_status = nullptr;
  sfrt::TileChains scheds;  // adaptive tile order (sfrt_sched.h), one chain per stream
  sfrt::TileSched dump_sched;  // sfrt_world_trace_points' own chain (never the frames')
  int cur_chain = 0;        // the chain of the launch between sched_begin and sched_end
  // Device copies of the sphere records for launches that read them from memory
  // (> 64 spheres, trace_points): a ring of slots, each with pinned staging and
  // the event of the last launch that read it, so a slot is never overwritten
  // while a launch on any stream may still read it.
  static constexpr int kRing = 8;
  sfrt::SphereRec* d_spheres[kRing] = {};
  sfrt::SphereRec* h_spheres[kRing] = {};
  hipEvent_t spheres_ev[kRing] = {};    // relayed (sfrt_host.h Relay): the slot's last reader done
  hipEvent_t spheres_stop[kRing] = {};  // that reader's own stop event, on the caller's stream
  sfrt::Relay relay;
  bool spheres_pending[kRing] = {};
  int d_spheres_cap = 0;
  int ring = 0;
  int staged = -1;  // slot staged for the launch being prepared, or -1
  uint32_t* d_frame = nullptr;  // compact subset buffer for the host path
  size_t d_frame_px = 0;
  uint32_t* h_stage = nullptr;  // pinned D2H staging
  size_t h_stage_px = 0;
  sfrt::RetiredHost retired_host;  // replaced pinned buffers (sfrt_host.h)
  std::vector<void*> retired_device;  // replaced record rings, freed with the world
  // --- frame pipeline (display path): render k+1 while frame k is copied ---
  struct PipeSlot {
    uint32_t* d_buf = nullptr;
    size_t px = 0;
    hipEvent_t rendered = nullptr, copied = nullptr;
    int* d_status = nullptr;    // this frame's march/texel flags
    int* h_status = nullptr;    // pinned copy, valid once `copied` completes
    bool used = false;
  };
  static constexpr int kPipe = 2;
  PipeSlot pipe[kPipe];
  hipStream_t copy_stream = nullptr;
  int64_t next_ticket = 0;
  mutable std::mutex mu;  // every entry point, getters included (RenderThreads call concurrently)

  ~sfrt_world() {
    sfrt::DeviceGuard g(device);
    if (stream) (void)hipStreamSynchronize(stream);
    if (copy_stream) (void)hipStreamSynchronize(copy_stream);
    for (PipeSlot& p : pipe) {
      (void)hipFree(p.d_buf);
      (void)hipFree(p.d_status);
      (void)hipHostFree(p.h_status);
      if (p.rendered) (void)hipEventDestroy(p.rendered);
      if (p.copied) (void)hipEventDestroy(p.copied);
    }
    if (copy_stream) (void)hipStreamDestroy(copy_stream);
    scheds.release();
    dump_sched.release();
    (void)hipFree(d_tex);
    for (void* p : retired_tex) (void)hipFree(p);
    tex_written.release();
    tex_stage.release();
    (void)hipFree(d_status);
    (void)hipDeviceSynchronize();
    for (int k = 0; k < kRing; k++) {
      (void)hipFree(d_spheres[k]);
      (void)hipHostFree(h_spheres[k]);
      if (spheres_ev[k]) (void)hipEventDestroy(spheres_ev[k]);
      if (spheres_stop[k]) (void)hipEventDestroy(spheres_stop[k]);
    }
    relay.release();
    (void)hipFree(d_frame);
    (void)hipHostFree(h_stage);
    retired_host.release();
    for (void* p : retired_device) (void)hipFree(p);
    if (stream) (void)hipStreamDestroy(stream);
  }

  int validate() const {
    if (spheres.empty()) return SFRT_E_EMPTY;
    if ((int)spheres.size() > SFRT_MAX_SPHERES) return SFRT_E_TOO_MANY;
    if (tex_host[0].empty() || !d_tex) return SFRT_E_NO_TEXTURE;
    for (int32_t k : sphere_tex)
      if (tex_host[k].empty()) return SFRT_E_NO_TEXTURE;
    if (width <= 0 || height <= 0) return SFRT_E_INVALID;
    return SFRT_OK;
  }

  // Per-frame records: everything uniform over the frame, computed with the
  // reference's expressions (see sfrt_trace.h).
  void prepare(sfrt::FrameRec& f, std::vector<sfrt::SphereRec>& recs) const {
    std::memset(&f, 0, sizeof f);
    const V3 campos{cam.pos[0], cam.pos[1], cam.pos[2]};
    f.cam[0] = campos.x; f.cam[1] = campos.y; f.cam[2] = campos.z;
    // SphereWorld.cpp:100-104
    V3 up = rot_x({0, -1, 0}, -cam.hrotation);
    V3 forward = rot_x({0, 0, 1}, -cam.hrotation);
    const V3 right = rot_y({1, 0, 0}, cam.rotation);
    forward = rot_y(forward, cam.rotation);
    up = rot_y(up, cam.rotation);
    f.fwd[0] = forward.x; f.fwd[1] = forward.y; f.fwd[2] = forward.z;
    f.right[0] = right.x; f.right[1] = right.y; f.right[2] = right.z;
    f.up[0] = up.x; f.up[1] = up.y; f.up[2] = up.z;
    // SphereWorld.cpp:85-89
    f.v_start = -cam.fov_v;
    f.v_inc = cam.fov_v / height * 2;
    f.h_start = -cam.fov_h;
    f.h_inc = cam.fov_h / width * 2;
    // First march iteration (pos == cam.pos for every pixel), SphereWorld.cpp:362-370.
    float largest = 0.0f;
    int draw = 0;
    for (size_t i = 0; i < spheres.size(); i++) {
      const float dist = vlength(vsub(campos, center(spheres[i])));
      if (spheres[i].radius - dist > 0.01f) {
        const float t = spheres[i].radius - dist;
        largest = largest < t ? t : largest;
        draw = (int)i;
      }
    }
    f.first_l = largest;
    f.first_draw = draw;
    f.n = (int)spheres.size();
    f.width = width;
    f.height = height;
    f.cull = cull;
    f.rays = rays;
    // Culling margin (sphere_trace.hip, cull_mask).  A march step
    // pos += dir * L rounds twice per component, so each step moves the
    // position off the ray's exact line by at most ~2.1e-7 * (|pos| + L) <=
    // 4.2e-7 * R, where R bounds every |coordinate| the march can reach (the
    // camera and every sphere's |c| + r).  Over kCullSafeIterations (1024)
    // steps that is < 4.3e-4 * R, inside the 1e-3 * R margin added to every
    // radius; the reference test additionally needs r - |p - c| > 0.01.
    const V3 origin{0.0f, 0.0f, 0.0f};
    float reach = vlength(campos);
    for (const sfrt_sphere& s : spheres) {
      const float e = vlength(vsub(center(s), origin)) + s.radius;
      reach = reach < e ? e : reach;
    }
    f.cull_margin = 1e-3f * reach + 1e-4f;
    // Non-finite inputs void the drift bound and the cone: visit every sphere.
    bool finite = std::isfinite(f.cull_margin) && std::isfinite(f.first_l) &&
                  std::isfinite(f.h_start) && std::isfinite(f.h_inc) &&
                  std::isfinite(f.v_start) && std::isfinite(f.v_inc);
    for (int q = 0; q < 3; q++)
      finite = finite && std::isfinite(f.cam[q]) && std::isfinite(f.fwd[q]) &&
               std::isfinite(f.right[q]) && std::isfinite(f.up[q]);
    if (!finite) f.cull = 0;
    f.tex = d_tex;
    f.status = d_status;
    recs.resize(spheres.size());
    for (size_t i = 0; i < spheres.size(); i++) {
      const sfrt_sphere& s = spheres[i];
      sfrt::SphereRec& r = recs[i];
      r.cx = s.x; r.cy = s.y; r.cz = s.z; r.r = s.radius;
      r.s_pass = pass_threshold(s.radius);
      r.atan_c = sfrt_math::atan2f(s.z, s.x);  // == libm atan2f (tests/test_math_exhaustive.py)
      const int k = sphere_tex[i];
      r.tex_off = tex_off[k];
      r.tex_wh = (uint32_t)tex_w[k] | ((uint32_t)tex_h[k] << 16);
    }
  }

  // A larger record ring, waiting for no stream (sfrt_host.h: hipFree / hipHostFree would wait for
  // the whole device): launches queued on any stream may still read the old slots, so the old
  // buffers are retired until the world is destroyed (the ring grows geometrically, and only past
  // the largest sphere count seen); the new ones are plain allocations every stream may use.
  int ensure_sphere_buffers(int n) {
    if (n <= d_spheres_cap) return SFRT_OK;
    const int cap = (int)sfrt::grown_capacity((size_t)d_spheres_cap, (size_t)n);
    for (int k = 0; k < kRing; k++) {
      if (d_spheres[k]) retired_device.push_back(d_spheres[k]);
      retired_host.add(h_spheres[k]);
      d_spheres[k] = nullptr;
      h_spheres[k] = nullptr;
      spheres_pending[k] = false;
    }
    d_spheres_cap = 0;
    for (int k = 0; k < kRing; k++) {
      HIP_TRY(hipMalloc(&d_spheres[k], sizeof(sfrt::SphereRec) * (size_t)cap));
      HIP_TRY(hipHostMalloc(&h_spheres[k], sizeof(sfrt::SphereRec) * (size_t)cap,
                            hipHostMallocDefault));
      if (!spheres_ev[k]) HIP_TRY(hipEventCreateWithFlags(&spheres_ev[k], hipEventDisableTiming));
      if (!spheres_stop[k]) HIP_TRY(hipEventCreateWithFlags(&spheres_stop[k], hipEventDisableTiming));
    }
    d_spheres_cap = cap;
    return SFRT_OK;
  }

  // Upload sphere records when the kernel reads them from device memory.
  int stage_spheres(sfrt::FrameRec& f, const std::vector<sfrt::SphereRec>& recs, hipStream_t s,
                    bool force) {
    staged = -1;
    if (!force && f.n <= sfrt::kInlineSpheres) {
      f.spheres = nullptr;
      return SFRT_OK;
    }
    int rc = ensure_sphere_buffers(f.n);
    if (rc) return rc;
    const int k = ring;
    ring = (ring + 1) % kRing;
    if (spheres_pending[k]) HIP_TRY(hipEventSynchronize(spheres_ev[k]));
    spheres_pending[k] = false;
    std::memcpy(h_spheres[k], recs.data(), sizeof(sfrt::SphereRec) * recs.size());
    HIP_TRY(hipMemcpyAsync(d_spheres[k], h_spheres[k], sizeof(sfrt::SphereRec) * recs.size(),
                           hipMemcpyHostToDevice, s));
    f.spheres = d_spheres[k];
    staged = k;
    return SFRT_OK;
  }

  // After the launch that reads the staged slot has been queued on s.
  int launched(hipStream_t s) {
    if (staged < 0) return SFRT_OK;
    HIP_TRY(relay.record(s, spheres_ev[staged]));
    spheres_pending[staged] = true;
    staged = -1;
    return SFRT_OK;
  }
  // The same through the launch itself: the staged slot's event for launch_trace to record as
  // the kernel's stop event (no marker packet between frames, sfrt_host.h
  // TableSlot::launch_event), then launched_with() once the launch is queued.
  void* ring_event() const { return staged >= 0 ? spheres_stop[staged] : nullptr; }
  int launched_with() {
    if (staged < 0) return SFRT_OK;
    HIP_TRY(relay.pass(spheres_stop[staged], spheres_ev[staged]));
    spheres_pending[staged] = true;
    staged = -1;
    return SFRT_OK;
  }

  // Before a render_band / submit_frame launch on s: link f into the tile-order chain.
  int sched_begin(sfrt::FrameRec& f, hipStream_t s) {
    long long tiles = 0;
    const long long key = tile_order_on ? sfrt::trace_tile_key(f, &tiles) : 0;
    sfrt::TileSchedPtrs p;
    cur_chain = scheds.pick(s);
    sfrt::TileSched& sched = scheds.chain[cur_chain];
    const ChainCam& chain_last = chain_cam[cur_chain];
    const long long cap0 = sched.cap;
    HIP_TRY(sched.begin(key, tiles, s, tile_order_on, p));
    if (sched.cap != cap0 && last_fill.chain == cur_chain)
      last_fill.valid = false;  // the cost buffers were reallocated
    f.tile_order = p.tile_order;
    f.tile_cost = p.tile_cost;
    f.prev_cost = p.prev_cost;
    f.next_order = p.next_order;
    f.cost_diff = p.cost_diff ? 1 : 0;
    // a moving camera: the recorded classes are a frame or two off
    f.order_dilate = p.prev_cost && chain_last.valid &&
                     std::memcmp(&chain_last.cam, &cam, sizeof cam) != 0;
    return SFRT_OK;
  }

  // After launch_trace for f returned (queued = false: it failed).
  int sched_end(const sfrt::FrameRec& f, hipStream_t s, bool queued) {
    sfrt::TileSchedPtrs p;
    p.tile_cost = f.tile_cost;
    sfrt::TileSched& sched = scheds.chain[cur_chain];
    HIP_TRY(sched.end(p, s, queued));
    if (!queued) {
      chain_cam[cur_chain].valid = false;
      if (last_fill.chain == cur_chain) last_fill.valid = false;
      return SFRT_E_HIP;
    }
    if (sched.committed) {
      chain_cam[cur_chain] = ChainCam{true, cam, f.sub_row0};
      // that launch wrote its classes into cost[k % 2] before end() advanced k
      last_fill = LastFill{true, f.sub_row0, f.sub_rows, f.sub_w, sched.key_prev,
                           (int)((sched.k - 1) & 1), cur_chain};
    } else {
      last_fill.valid = false;  // this fill recorded no classes (tile order off, probe)
    }
    return SFRT_OK;
  }

  // The last launch that recorded its per-tile march-step classes (sfrt_world_row_costs).
  struct LastFill {
    bool valid = false;
    int row0 = 0, rows = 0, width = 0;
    long long key = 0;  // trace_tile_key: pixels per lane and the tile grid
    int buf = 0;        // scheds.chain[chain].cost[buf]
    int chain = -1;
  };
  LastFill last_fill;

  // The camera of the last launch that joined the tile-order chain: its costs are the
  // ones the next launch's sorter ranks.
  struct ChainCam {
    bool valid = false;
    sfrt_camera cam{};
    int sub_row0 = 0;
  };
  ChainCam chain_cam[sfrt::TileChains::kChains];  // per chain

  // On s itself: hipMemcpy / hipMemset run on the null stream, which also waits for every blocking
  // stream of the process (a caller's hipStreamCreate streams), not just s.
  int read_status(hipStream_t s) {
    int st = 0;
    HIP_TRY(hipMemcpyAsync(&st, d_status, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (st) {
      HIP_TRY(hipMemsetAsync(d_status, 0, sizeof(int), s));
      HIP_TRY(hipStreamSynchronize(s));
    }
    if (st & 1) return SFRT_E_MARCH_LIMIT;
    if (st & 2) return SFRT_E_TEXEL;
    return SFRT_OK;
  }
};

namespace {

// Representative march steps of a tile-order class (the inverse of sfrt_device.h
// tile_bucket: class 15 - c holds steps < 4 for c = 0, 2c + 2 .. 2c + 3 for c = 1..6,
// 16 + 4 (c - 7) .. + 3 for c = 7..10, then 32-39, 40-47, 48-63, 64-95, >= 96).
double class_steps(uint8_t cls) {
  const int c = 15 - (int)(cls & 15);
  if (c == 0) return 3.0;
  if (c <= 6) return 2.0 * c + 2.5;
  if (c <= 10) return 16.0 + 4.0 * (c - 7) + 1.5;
  static const double tail[5] = {35.5, 43.5, 55.5, 79.5, 128.0};
  return tail[c - 11];
}

// The shading tail costs about as much as four march steps per pixel (22% of
// the 4K frame, whose tiles march ~14 steps).
constexpr double kShadeSteps = 4.0;

}  // namespace

extern "C" {

int sfrt_world_row_costs(sfrt_world* w, float* costs, int capacity, int* row0, int* rows) {
  if (!w || !row0 || !rows || capacity < 0 || (capacity > 0 && !costs)) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  *row0 = 0;
  *rows = 0;
  const auto& L = w->last_fill;
  if (!L.valid) return SFRT_E_INVALID;
  const int tile_w = (int)((L.key >> 56) & 0x3f) * sfrt::kTile;
  const long long tiles_x = (L.key >> 28) & 0xfffffff, tiles_y = L.key & 0xfffffff;
  const sfrt::TileSched& sched = w->scheds.chain[L.chain];
  if (tile_w <= 0 || tiles_x * tiles_y > sched.cap) return SFRT_E_INVALID;
  if (capacity < L.rows) return SFRT_E_INVALID;
  sfrt::DeviceGuard g(w->device);
  // the chain's last launch may still be running on a stream the caller has since destroyed
  // (its handle must not be used, sfrt_sched.h): a tuning call, it waits for the device
  if (sched.have_last) HIP_TRY(hipDeviceSynchronize());
  std::vector<uint8_t> cls((size_t)(tiles_x * tiles_y));
  HIP_TRY(hipMemcpy(cls.data(), sched.cost[L.buf], cls.size(), hipMemcpyDeviceToHost));
  for (long long ty = 0; ty < tiles_y; ty++) {
    double c = 0.0;
    for (long long tx = 0; tx < tiles_x; tx++) {
      const long long x0 = tx * tile_w;
      const long long px = std::min<long long>(tile_w, L.width - x0);
      c += (class_steps(cls[(size_t)(ty * tiles_x + tx)]) + kShadeSteps) * (double)px;
    }
    for (int j = (int)ty * sfrt::kTile; j < std::min(L.rows, (int)(ty + 1) * sfrt::kTile); j++)
      costs[j] = (float)c;
  }
  *row0 = L.row0;
  *rows = L.rows;
  return SFRT_OK;
}

int sfrt_world_create(int hip_device, sfrt_world** out) {
  if (!out) return SFRT_E_INVALID;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || hip_device < 0 || hip_device >= count)
    return SFRT_E_HIP;
  sfrt_world* w = new sfrt_world();
  w->device = hip_device;
  w->tex_written.relay = &w->relay;
  // Camera defaults (SphereWorld.h:10-21) and the constructor's conversion (:72-73).
  w->cam.fov_h = sfrt_deg_to_rad(75.0f);
  w->cam.fov_v = sfrt_deg_to_rad(47.0f);
  sfrt::DeviceGuard g(hip_device);
  if (hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&w->d_status, sizeof(int)) != hipSuccess ||
      hipMemset(w->d_status, 0, sizeof(int)) != hipSuccess) {
    delete w;
    return SFRT_E_HIP;
  }
  *out = w;
  return SFRT_OK;
}

void sfrt_world_destroy(sfrt_world* w) { delete w; }

int sfrt_world_set_size(sfrt_world* w, int width, int height) {
  if (!w || width <= 0 || height <= 0) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  if (width != w->width || height != w->height) {
    // the last fill's rows and tile grid belong to the old frame (sfrt_world_row_costs)
    w->last_fill.valid = false;
    for (auto& c : w->chain_cam) c.valid = false;
  }
  w->width = width;
  w->height = height;
  return SFRT_OK;
}

int sfrt_world_get_size(const sfrt_world* w, int* width, int* height) {
  if (!w || !width || !height) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  *width = w->width;
  *height = w->height;
  return SFRT_OK;
}

int sfrt_world_set_camera(sfrt_world* w, const sfrt_camera* cam) {
  if (!w || !cam || !finite3(cam->pos) || !std::isfinite(cam->rotation) ||
      !std::isfinite(cam->hrotation) || !std::isfinite(cam->fov_h) || !std::isfinite(cam->fov_v))
    return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  w->cam = *cam;
  return SFRT_OK;
}

int sfrt_world_get_camera(const sfrt_world* w, sfrt_camera* cam) {
  if (!w || !cam) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  *cam = w->cam;
  return SFRT_OK;
}

int sfrt_world_load_texture(sfrt_world* w, int slot, const uint8_t* rgba, int tex_w, int tex_h) {
  if (!w || !rgba || slot < 0 || slot >= SFRT_TEXTURE_SLOTS || tex_w <= 0 || tex_h <= 0 ||
      tex_w > 0xffff || tex_h > 0xffff || (int64_t)tex_w * tex_h > (1 << 28))
    return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  const size_t bytes = (size_t)tex_w * tex_h * 4;
  w->tex_host[slot].assign(rgba, rgba + bytes);
  w->tex_w[slot] = tex_w;
  w->tex_h[slot] = tex_h;
  bool a01 = true;
  for (size_t i = 3; i < bytes && a01; i += 4) a01 = rgba[i] == 0 || rgba[i] == 255;
  w->tex_alpha01[slot] = a01;
  // Rebuild the device atlas: textures[0] (SphereWorld.cpp:376-377) first, then
  // the extension slots.  Draws on any stream may still read the old atlas.
  size_t total = 0;
  for (int k = 0; k < SFRT_TEXTURE_SLOTS; k++) {
    w->tex_off[k] = (uint32_t)total;
    total += (size_t)w->tex_w[k] * w->tex_h[k];
  }
  if (total > 0xffffffffull) return SFRT_E_INVALID;
  sfrt::DeviceGuard g(w->device);
  // Stream-ordered (no device-wide wait): a new atlas (hipMalloc waits for no stream,
  // profiles/r6u_hip_alloc_calls.txt), uploaded on the world's stream from pinned staging.
  void* staged = nullptr;
  HIP_TRY(w->tex_stage.take(total * 4, &staged));
  for (int k = 0; k < SFRT_TEXTURE_SLOTS; k++)
    if (!w->tex_host[k].empty())
      std::memcpy((uint8_t*)staged + (size_t)w->tex_off[k] * 4, w->tex_host[k].data(),
                  w->tex_host[k].size());
  uint32_t* fresh = nullptr;
  HIP_TRY(hipMalloc(&fresh, total * 4));
  if (hipMemcpyAsync(fresh, staged, total * 4, hipMemcpyHostToDevice, w->stream) != hipSuccess ||
      w->tex_stage.copied(w->stream) != hipSuccess || w->tex_written.after_write(w->stream) != hipSuccess) {
    (void)hipStreamSynchronize(w->stream);
    (void)hipFree(fresh);
    return SFRT_E_HIP;
  }
  if (w->d_tex) {
    w->retired_tex.push_back(w->d_tex);
    w->retired_tex_bytes += w->d_tex_texels * 4;
  }
  w->d_tex = fresh;
  w->d_tex_texels = total;
  if (w->retired_tex_bytes > sfrt_world::kRetiredTexBytes) {  // a texture reloaded every frame
    HIP_TRY(hipDeviceSynchronize());
    for (void* p : w->retired_tex) (void)hipFree(p);
    w->retired_tex.clear();
    w->retired_tex_bytes = 0;
  }
  return SFRT_OK;
}

int sfrt_world_alpha_binary(const sfrt_world* w, int* binary) {
  if (!w || !binary) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  bool any = false, all = true;
  for (int k = 0; k < SFRT_TEXTURE_SLOTS; k++) {
    if (w->tex_host[k].empty()) continue;
    any = true;
    all = all && w->tex_alpha01[k];
  }
  *binary = any && all ? 1 : 0;
  return SFRT_OK;
}

int sfrt_world_add_sphere(sfrt_world* w, float x, float y, float z, float radius) {
  const sfrt_sphere add{x, y, z, radius};
  if (!w || !sphere_ok(add)) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  std::vector<sfrt_sphere>& s = w->spheres;
  std::vector<int32_t>& st = w->sphere_tex;
  s.push_back(add);
  st.push_back(0);
  // SphereWorld.cpp:180-188: drop every sphere contained in another one.
  for (int i = 0; i < (int)s.size(); i++) {
    for (int j = 0; j < (int)s.size(); j++) {
      if (i != j && vlength(vsub(center(s[i]), center(s[j]))) + s[i].radius <= s[j].radius) {
        s.erase(s.begin() + i);
        st.erase(st.begin() + i);
        i--;
        break;
      }
    }
  }
  permute(st, sort_spheres(s, {w->cam.pos[0], w->cam.pos[1], w->cam.pos[2]}));
  if ((int)s.size() > SFRT_MAX_SPHERES) return SFRT_E_TOO_MANY;
  return SFRT_OK;
}

int sfrt_world_set_spheres(sfrt_world* w, const sfrt_sphere* spheres, int count) {
  if (!w || count < 0 || (count > 0 && !spheres)) return SFRT_E_INVALID;
  if (count > SFRT_MAX_SPHERES) return SFRT_E_TOO_MANY;
  for (int i = 0; i < count; i++)
    if (!sphere_ok(spheres[i])) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  w->spheres.assign(spheres, spheres + count);
  w->sphere_tex.assign((size_t)count, 0);
  return SFRT_OK;
}

int sfrt_world_set_sphere_textures(sfrt_world* w, const int32_t* slots, int count) {
  if (!w || count < 0 || (count > 0 && !slots)) return SFRT_E_INVALID;
  for (int i = 0; i < count; i++)
    if (slots[i] < 0 || slots[i] >= SFRT_TEXTURE_SLOTS) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  if ((size_t)count != w->spheres.size()) return SFRT_E_INVALID;
  w->sphere_tex.assign(slots, slots + count);
  return SFRT_OK;
}

int sfrt_world_get_sphere_textures(sfrt_world* w, int32_t* out, int capacity, int* count) {
  if (!w || !count) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  *count = (int)w->sphere_tex.size();
  if (out) {
    const int n = capacity < *count ? capacity : *count;
    std::memcpy(out, w->sphere_tex.data(), sizeof(int32_t) * (size_t)(n > 0 ? n : 0));
  }
  return SFRT_OK;
}

int sfrt_world_get_spheres(const sfrt_world* w, sfrt_sphere* out, int capacity, int* count) {
  if (!w || !count) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  *count = (int)w->spheres.size();
  if (out) {
    const int n = capacity < *count ? capacity : *count;
    std::memcpy(out, w->spheres.data(), sizeof(sfrt_sphere) * (size_t)(n > 0 ? n : 0));
  }
  return SFRT_OK;
}

int sfrt_world_update_spheres(sfrt_world* w) {
  if (!w) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  permute(w->sphere_tex, sort_spheres(w->spheres, {w->cam.pos[0], w->cam.pos[1], w->cam.pos[2]}));
  return SFRT_OK;
}

int sfrt_world_set_option(sfrt_world* w, int option, int value) {
  if (!w) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  if (option == SFRT_OPT_CULL) {
    w->cull = value ? 1 : 0;
    return SFRT_OK;
  }
  if (option == SFRT_OPT_RAYS_PER_LANE) {
    if (value < 0 || value > 4) return SFRT_E_INVALID;
    w->rays = value;
    return SFRT_OK;
  }
  if (option == SFRT_OPT_TILE_ORDER) {
    w->tile_order_on = value == 2 ? 2 : value ? 1 : 0;  // 2: timing probe (see sched_begin)
    return SFRT_OK;
  }
  return SFRT_E_INVALID;
}

int sfrt_world_update_image(sfrt_world* w, uint8_t* pixels, int ystart, int yadd, int xstart,
                            int xadd) {
  if (!w || !pixels || ystart < 0 || xstart < 0 || yadd <= 0 || xadd <= 0) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  int rc = w->validate();
  if (rc) return rc;
  // SphereWorld.cpp:94,97: i = xstart, xstart + xadd, ... < width (same for j).
  const int sub_w = xstart < w->width ? (w->width - xstart + xadd - 1) / xadd : 0;
  const int sub_h = ystart < w->height ? (w->height - ystart + yadd - 1) / yadd : 0;
  if (sub_w == 0 || sub_h == 0) return SFRT_OK;
  sfrt::DeviceGuard g(w->device);
  const size_t px = (size_t)sub_w * sub_h;
  // Growth waits for no other stream (sfrt_host.h: hipFree / hipHostFree wait for the whole
  // device): the device frame stream-ordered on the world's stream, behind the last update_image
  // (which waited for its own copy); the old pinned staging retired.
  if (w->d_frame_px < px) {
    if (w->d_frame) HIP_TRY(hipFreeAsync(w->d_frame, w->stream));
    w->d_frame = nullptr;
    w->d_frame_px = 0;
    HIP_TRY(hipMallocAsync((void**)&w->d_frame, px * 4, w->stream));
    w->d_frame_px = px;
  }
  if (w->h_stage_px < px) {
    w->retired_host.add(w->h_stage);
    w->h_stage = nullptr;
    w->h_stage_px = 0;
    HIP_TRY(hipHostMalloc(&w->h_stage, px * 4, hipHostMallocDefault));
    w->h_stage_px = px;
  }
  sfrt::FrameRec f;
  std::vector<sfrt::SphereRec> recs;
  w->prepare(f, recs);
  f.xstart = xstart; f.xadd = xadd; f.ystart = ystart; f.yadd = yadd;
  f.sub_w = sub_w;
  f.sub_row0 = 0;
  f.sub_rows = sub_h;
  f.tiles_x = (sub_w + sfrt::kTile - 1) / sfrt::kTile;
  f.out = w->d_frame;
  f.out_pitch = sub_w;
  rc = w->stage_spheres(f, recs, w->stream, false);
  if (rc) return rc;
  if (sfrt::launch_trace(f, recs.data(), w->stream, nullptr, w->ring_event())) return SFRT_E_HIP;
  if ((rc = w->launched_with())) return rc;
  HIP_TRY(hipMemcpyAsync(w->h_stage, w->d_frame, px * 4, hipMemcpyDeviceToHost, w->stream));
  rc = w->read_status(w->stream);
  if (rc) return rc;
  // Scatter the subset into the caller's frame: only addressed pixels are written.
  const size_t W = (size_t)w->width;
  for (int bb = 0; bb < sub_h; bb++) {
    const size_t j = (size_t)ystart + (size_t)bb * yadd;
    const uint32_t* src = w->h_stage + (size_t)bb * sub_w;
    uint8_t* row = pixels + j * W * 4;
    if (xadd == 1) {
      std::memcpy(row + (size_t)xstart * 4, src, (size_t)sub_w * 4);
    } else {
      for (int a = 0; a < sub_w; a++)
        std::memcpy(row + ((size_t)xstart + (size_t)a * xadd) * 4, src + a, 4);
    }
  }
  return SFRT_OK;
}

int sfrt_world_render_band(sfrt_world* w, void* dev_pixels, int64_t pitch_bytes, int row0,
                           int rows, void* hip_stream) {
  if (!w || !dev_pixels || row0 < 0 || rows < 0 || pitch_bytes % 4 != 0) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  int rc = w->validate();
  if (rc) return rc;
  if (pitch_bytes < (int64_t)w->width * 4 || row0 + rows > w->height) return SFRT_E_INVALID;
  if (rows == 0) {
    w->last_fill.valid = false;  // the last fill covered no rows (sfrt_world_row_costs)
    return SFRT_OK;
  }
  sfrt::DeviceGuard g(w->device);
  hipStream_t s = (hipStream_t)hip_stream;  // HIP convention: NULL = the null stream
  sfrt::FrameRec f;
  std::vector<sfrt::SphereRec> recs;
  w->prepare(f, recs);
  f.xstart = 0; f.xadd = 1; f.ystart = 0; f.yadd = 1;
  f.sub_w = w->width;
  f.sub_row0 = row0;
  f.sub_rows = rows;
  f.tiles_x = (w->width + sfrt::kTile - 1) / sfrt::kTile;
  f.out = (uint32_t*)dev_pixels;
  f.out_pitch = pitch_bytes / 4;
  rc = w->stage_spheres(f, recs, s, false);
  if (rc) return rc;
  // after the last texture upload (queued on w->stream, where the other launches run)
  HIP_TRY(w->tex_written.before_read(s));
  if ((rc = w->sched_begin(f, s))) return rc;
  if ((rc = w->sched_end(f, s, sfrt::launch_trace(f, recs.data(), s, nullptr, w->ring_event()) == 0)))
    return rc;
  if ((rc = w->launched_with())) return rc;
  return SFRT_OK;
}

int sfrt_world_check(sfrt_world* w, void* hip_stream) {
  if (!w) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  sfrt::DeviceGuard g(w->device);
  return w->read_status((hipStream_t)hip_stream);
}

int sfrt_world_trace_points(sfrt_world* w, const int32_t* ij, int count, sfrt_pixel_dump* out) {
  if (!w || count < 0 || (count > 0 && (!ij || !out))) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  int rc = w->validate();
  if (rc) return rc;
  for (int k = 0; k < count; k++)
    if (ij[2 * k] < 0 || ij[2 * k] >= w->width || ij[2 * k + 1] < 0 || ij[2 * k + 1] >= w->height)
      return SFRT_E_INVALID;
  if (count == 0) return SFRT_OK;
  static_assert(sizeof(sfrt_pixel_dump) == sizeof(sfrt::PixelDump), "dump layout");
  // The listed pixels come out of the frame-fill kernel itself (its DUMP instantiation,
  // sphere_trace.hip): a whole frame with the world's options -- the kernel table's tile
  // shape or SFRT_OPT_RAYS_PER_LANE, culling -- in the adaptive tile order when that is
  // on (three launches, so the last one runs in a sorted order), row-major otherwise.
  // Memory is O(count): the kernel binary-searches the sorted distinct pixel ids and
  // stores no frame.  The launches run on a private tile-order chain (dump_sched), so
  // the world's own chains, its last fill (sfrt_world_row_costs) and the next frame's
  // order are those of the caller's last render, untouched by the dump.
  std::vector<std::pair<int64_t, int>> ids((size_t)count);
  for (int k = 0; k < count; k++)
    ids[k] = {(int64_t)ij[2 * k + 1] * w->width + ij[2 * k], k};
  std::sort(ids.begin(), ids.end());
  std::vector<int64_t> pix;
  std::vector<int> slot((size_t)count);  // listed position -> distinct entry
  for (const auto& e : ids) {
    if (pix.empty() || pix.back() != e.first) pix.push_back(e.first);
    slot[e.second] = (int)pix.size() - 1;
  }
  sfrt::DeviceGuard g(w->device);
  sfrt::DumpArgs dump{};
  dump.npix = (int)pix.size();
  std::vector<sfrt::PixelDump> got(pix.size());
  int64_t* d_pix = nullptr;
  if (hipMalloc((void**)&d_pix, sizeof(int64_t) * pix.size()) != hipSuccess ||
      hipMalloc(&dump.out, sizeof(sfrt::PixelDump) * pix.size()) != hipSuccess) {
    (void)hipFree(d_pix);
    return SFRT_E_HIP;
  }
  dump.pix = d_pix;
  auto run = [&]() -> int {
    HIP_TRY(hipMemcpyAsync(d_pix, pix.data(), sizeof(int64_t) * pix.size(), hipMemcpyHostToDevice,
                           w->stream));
    const int passes = w->tile_order_on ? 3 : 1;
    w->dump_sched.reset();  // this frame's own order: record, sort, use
    for (int q = 0; q < passes; q++) {
      sfrt::FrameRec f;
      std::vector<sfrt::SphereRec> recs;
      w->prepare(f, recs);
      f.xstart = 0; f.xadd = 1; f.ystart = 0; f.yadd = 1;
      f.sub_w = w->width;
      f.sub_row0 = 0;
      f.sub_rows = w->height;
      f.tiles_x = (w->width + sfrt::kTile - 1) / sfrt::kTile;
      f.out = nullptr;  // the DUMP kernels store records only
      f.out_pitch = w->width;
      int rc2 = w->stage_spheres(f, recs, w->stream, false);
      if (rc2) return rc2;
      sfrt::TileSchedPtrs p;
      if (w->tile_order_on) {
        long long tiles = 0;
        const long long key = sfrt::trace_tile_key(f, &tiles);
        HIP_TRY(w->dump_sched.begin(key, tiles, w->stream, w->tile_order_on, p));
        f.tile_order = p.tile_order;
        f.tile_cost = p.tile_cost;
        f.prev_cost = p.prev_cost;
        f.next_order = p.next_order;
        f.cost_diff = p.cost_diff ? 1 : 0;
      }
      const bool queued = sfrt::launch_trace(f, recs.data(), w->stream, &dump) == 0;
      if (w->tile_order_on) HIP_TRY(w->dump_sched.end(p, w->stream, queued));
      if (!queued) return SFRT_E_HIP;
      if ((rc2 = w->launched(w->stream))) return rc2;
    }
    HIP_TRY(hipMemcpyAsync(got.data(), dump.out, sizeof(sfrt::PixelDump) * pix.size(),
                           hipMemcpyDeviceToHost, w->stream));
    return SFRT_OK;
  };
  rc = run();
  const int st = w->read_status(w->stream);
  (void)hipFree(d_pix);
  (void)hipFree(dump.out);
  if (rc || st) return rc ? rc : st;
  for (int k = 0; k < count; k++) std::memcpy(&out[k], &got[slot[k]], sizeof(sfrt_pixel_dump));
  return SFRT_OK;
}

int sfrt_host_alloc(void** ptr, int64_t bytes) {
  if (!ptr || bytes <= 0) return SFRT_E_INVALID;
  *ptr = nullptr;
  return hipHostMalloc(ptr, (size_t)bytes, hipHostMallocDefault) == hipSuccess ? SFRT_OK
                                                                               : SFRT_E_HIP;
}

int sfrt_host_free(void* ptr) {
  if (!ptr) return SFRT_OK;
  return hipHostFree(ptr) == hipSuccess ? SFRT_OK : SFRT_E_HIP;
}

int sfrt_world_submit_frame(sfrt_world* w, uint8_t* pixels, int64_t* ticket) {
  if (!w || !pixels || !ticket) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(w->mu);
  int rc = w->validate();
  if (rc) return rc;
  sfrt::DeviceGuard g(w->device);
  if (!w->copy_stream && hipStreamCreateWithFlags(&w->copy_stream, hipStreamNonBlocking) != hipSuccess)
    return SFRT_E_HIP;
  const int64_t t = w->next_ticket;
  sfrt_world::PipeSlot& slot = w->pipe[t % sfrt_world::kPipe];
  if (!slot.rendered) {
    HIP_TRY(hipEventCreateWithFlags(&slot.rendered, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&slot.copied, hipEventDisableTiming));
    HIP_TRY(hipMalloc(&slot.d_status, sizeof(int)));
    HIP_TRY(hipHostMalloc(&slot.h_status, sizeof(int), hipHostMallocDefault));
  }
  const size_t px = (size_t)w->width * w->height;
  if (slot.px < px) {  // stream-ordered: freed behind its last copy, no device-wide wait
    if (slot.used) HIP_TRY(hipStreamWaitEvent(w->stream, slot.copied, 0));
    if (slot.d_buf) HIP_TRY(hipFreeAsync(slot.d_buf, w->stream));
    slot.d_buf = nullptr;
    slot.px = 0;
    HIP_TRY(hipMallocAsync(&slot.d_buf, px * 4, w->stream));
    slot.px = px;
  }
  // The slot's previous frame must have left d_buf before this render writes it.
  if (slot.used) HIP_TRY(hipStreamWaitEvent(w->stream, slot.copied, 0));
  HIP_TRY(hipMemsetAsync(slot.d_status, 0, sizeof(int), w->stream));
  sfrt::FrameRec f;
  std::vector<sfrt::SphereRec> recs;
  w->prepare(f, recs);
  f.xstart = 0; f.xadd = 1; f.ystart = 0; f.yadd = 1;
  f.sub_w = w->width;
  f.sub_row0 = 0;
  f.sub_rows = w->height;
  f.tiles_x = (w->width + sfrt::kTile - 1) / sfrt::kTile;
  f.out = slot.d_buf;
  f.out_pitch = w->width;
  f.status = slot.d_status;
  rc = w->stage_spheres(f, recs, w->stream, false);
  if (rc) return rc;
  if ((rc = w->sched_begin(f, w->stream))) return rc;  // adaptive tile order, as render_band
  if ((rc = w->sched_end(f, w->stream,
                         sfrt::launch_trace(f, recs.data(), w->stream, nullptr, w->ring_event()) == 0)))
    return rc;
  if ((rc = w->launched_with())) return rc;
  HIP_TRY(hipEventRecord(slot.rendered, w->stream));
  HIP_TRY(hipStreamWaitEvent(w->copy_stream, slot.rendered, 0));
  HIP_TRY(hipMemcpyAsync(pixels, slot.d_buf, px * 4, hipMemcpyDeviceToHost, w->copy_stream));
  HIP_TRY(hipMemcpyAsync(slot.h_status, slot.d_status, sizeof(int), hipMemcpyDeviceToHost,
                         w->copy_stream));
  HIP_TRY(hipEventRecord(slot.copied, w->copy_stream));
  slot.used = true;
  *ticket = t;
  w->next_ticket = t + 1;
  return SFRT_OK;
}

int sfrt_world_wait_frame(sfrt_world* w, int64_t ticket) {
  if (!w || ticket < 0) return SFRT_E_INVALID;
  hipEvent_t ev;
  int* h_status;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    if (ticket >= w->next_ticket) return SFRT_E_INVALID;
    sfrt_world::PipeSlot& slot = w->pipe[ticket % sfrt_world::kPipe];
    // A slot reused by a newer ticket records a later event on the same
    // in-order copy stream, so waiting on it also covers this ticket.
    ev = slot.copied;
    h_status = slot.h_status;
  }
  sfrt::DeviceGuard g(w->device);
  HIP_TRY(hipEventSynchronize(ev));
  const int st = *h_status;
  if (st & 1) return SFRT_E_MARCH_LIMIT;
  if (st & 2) return SFRT_E_TEXEL;
  return SFRT_OK;
}

int sfrt_sort_spheres(sfrt_sphere* spheres, int count, const float cam_pos[3]) {
  if (count < 0 || (count > 0 && !spheres) || !cam_pos) return SFRT_E_INVALID;
  std::vector<sfrt_sphere> v(spheres, spheres + count);
  sort_spheres(v, {cam_pos[0], cam_pos[1], cam_pos[2]});
  std::memcpy(spheres, v.data(), sizeof(sfrt_sphere) * (size_t)count);
  return SFRT_OK;
}

float sfrt_deg_to_rad(float deg) { return deg * (kPI / 180.0f); }

float sfrt_pass_threshold(float radius) { return pass_threshold(radius); }

const char* sfrt_error_string(int code) {
  switch (code) {
    case SFRT_OK: return "ok";
    case SFRT_E_INVALID: return "invalid argument";
    case SFRT_E_EMPTY: return "no spheres (reference: std::out_of_range from spheres.at)";
    case SFRT_E_NO_TEXTURE: return "texture slot 0 not loaded";
    case SFRT_E_TOO_MANY: return "too many spheres";
    case SFRT_E_HIP: return "HIP runtime error";
    case SFRT_E_MARCH_LIMIT: return "march iteration limit exceeded";
    case SFRT_E_TEXEL: return "texel index outside the texture";
    default: return "unknown error";
  }
}

int sfrt_version(void) { return 3; }

const char* sfrt_build_flavour(void) { return sfrt::trace_build_flavour(); }

}  // extern "C"
