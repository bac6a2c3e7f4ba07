// sfrt_voxel.cpp -- host side of the voxel World frame fill:
// a C++ mirror of the state World::UpdateImage reads and the extern "C"
// entry points sfrt_voxel_* of include/sfrt.h.
//
// Reference (paths under /root/reference/Raytracing/):
//   class World                     World.h:58-97 (width/height 320x180, shadowDistance 16,
//                                   viewDistance 24, Camera defaults World.h:9-19)
//   World::World (fov -> radians)   World.cpp:55-56
//   World::UpdateImage              World.cpp:62-87 (per-column / per-row terms below)
//   blocks, textures, dynTextures,  World.h:75, 90-95
//   colors, dyn, alights
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <algorithm>
#include <vector>

#include "sfrt.h"
#include "sfrt_host.h"
#include "sfrt_sched.h"
#include "sfrt_math.h"
#include "voxel_trace.h"

#pragma clang fp contract(off)

namespace {

constexpr float kPI = 3.1415926535f;  // World.h:5

// The light's contribution test of World::Raycast, `intensity / dd - dd * 0.002f > 0`
// (World.cpp:425-426), for a squared distance dd >= 0: true for dd below a threshold and false
// from it on (intensity / dd never increases with dd, dd * 0.002f never decreases, and each
// rounds monotonically), so the smallest non-negative float where it is false is found by
// bisection over the bit patterns of [+0, +inf].  The kernel skips a light for a wave none of
// whose lanes has dd below it (VoxLight::dd_skip).
static bool light_adds(float intensity, float dd) {
  volatile float q = intensity / dd;   // binary32, correctly rounded (no contraction: FLAGS)
  volatile float p = dd * 0.002f;
  return q - p > 0.0f;
}
float light_dd_pass(float intensity) {
  uint32_t lo = 0u, hi = 0x7f800000u;  // light_adds(+inf) is false for every intensity
  if (!light_adds(intensity, 0.0f)) return 0.0f;
  while (hi - lo > 1u) {               // invariant: adds at lo, not at hi
    const uint32_t mid = lo + (hi - lo) / 2u;
    float m;
    std::memcpy(&m, &mid, 4);
    if (light_adds(intensity, m)) lo = mid; else hi = mid;
  }
  float t;
  std::memcpy(&t, &hi, 4);
  return t;
}

// VoxLight::dd_skip from dd_pass: RU(dd_pass / (1 - 2^-20)), so that a squared distance
// evaluated with fmas (relative error within 2^-20 of the reference's three products and two
// sums, all terms non-negative) at or above it implies the reference's dd >= dd_pass.
float light_dd_skip(float dd_pass) {
  const double t = (double)dd_pass / (1.0 - 0x1.0p-20);
  const float f = (float)t;
  return (double)f >= t ? f : std::nextafter(f, INFINITY);
}

// The fast primary DDA's bound (VoxFrame::dda_qlim, voxel_trace.hip pos_i32).  At a position
// with |p| < 2^30, a step of World::Raycast (World.cpp:330-350) divides a numerator in (-1, 2)
// (dirXadd + sign * (p - (int)p)) by |d_k|, so |raySpeed| <= 2 (1 + 2^-23) / m with
// m = min_k |d_k| (a negative fraction can make it negative), and moves axis j by at most
// |d_j| (|raySpeed| + 0.002)(1 + 2^-21) <= 2.0001 X / m + 0.0021 X (X = max_k |d_k| <= xmax),
// plus the add's rounding, <= 32 below 2^30.  So with Q = X / m, S = 2.001 Q + 0.003 xmax + 33
// bounds one step and |cam| + (maxiter + 1) S <= 2^30 keeps every position of the walk below
// 2^30, where the plain conversion equals to_i32 (only +2^31 and beyond and NaN differ).  The
// kernel takes the fast DDA for a wave whose every lane has X <= qlim * m (the float product
// rounds up at most 2^-24, absorbed by rounding qlim down by 2^-20); 0 disables it.
float dda_qlim(const float cam[3], uint32_t maxiter, float xmax) {
  const double p = std::max({std::fabs((double)cam[0]), std::fabs((double)cam[1]),
                             std::fabs((double)cam[2])});
  const double q = ((1073741824.0 - p) / ((double)maxiter + 1.0) - 33.0 - 0.003 * xmax) / 2.001;
  if (!(q > 1.0) || !std::isfinite(xmax)) return 0.0f;
  const float f = (float)(q * (1.0 - 0x1.0p-20));
  return (double)f <= q * (1.0 - 0x1.0p-20) ? f : std::nextafter(f, 0.0f);
}

// float -> unsigned as the reference's x86-64 build converts it.
uint32_t to_u32(float f) {
  if (!(f > -9.2233720368547758e18f && f < 9.2233720368547758e18f)) return 0u;
  return (uint32_t)(int64_t)f;
}

struct DevTex {
  uint32_t* d = nullptr;
  int w = 0, h = 0;
  size_t cap = 0;
};


}  // namespace

struct sfrt_voxel {
  int device = 0;
  // --- World state read by UpdateImage ---
  int width = 320, height = 180;            // World.h:67-68
  sfrt_camera cam{};
  float shadow_distance = 16.0f;            // World.h:70
  float view_distance = 24.0f;              // World.h:71
  std::vector<int16_t> blocks;
  int nx = 0, ny = 0, nz = 0;
  uint32_t colors[sfrt::kVoxSlots] = {};
  std::vector<sfrt_dynamic> dyn;
  std::vector<sfrt_light> lights;
  // --- device resources ---
  hipStream_t stream = nullptr;
  DevTex tex[sfrt::kVoxSlots], dyn_tex[sfrt::kVoxSlots];
  uint8_t* d_cells = nullptr;  // the key-indexed byte grid (voxel_trace.h, cell_hit)
  size_t d_cells_cap = 0;
  // Every byte of d_cells outside planes x < box[0], rows y < box[1], columns z < box[2] is 0.
  int box[3] = {0, 0, 0};
  bool blocks_dirty = true;
  // The codes of a set_blocks on their way to the grid: pinned staging, its device copy, and the
  // event after the rewrite that read them.  Two in turn, so that blocks set on consecutive frames
  // do not wait on the host for the previous rewrite (which may sit behind other work on its
  // stream); an upload reuses a pair only after that pair's previous rewrite has run.
  struct CodeStage {
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    bool pending = false;
  };
  CodeStage stage[2];
  int stage_next = 0;
  sfrt::RetiredHost retired_host;  // replaced pinned buffers (sfrt_host.h: hipHostFree waits for all)
  // d_cells' and the textures' rewrites ordered against their readers (sfrt_host.h)
  sfrt::SharedBuffer shared;
  sfrt::PinnedStage tex_stage;  // texture uploads from the caller's memory
  // Per-frame tables (columns | rows | dyn | lights) in a ring of slots, each
  // with pinned staging and the event of the last launch that read it, so
  // launches on different streams never see a table overwritten under them.
  // (sfrt::TableSlot, sfrt_host.h: a reuse on another stream waits for the slot's last user.)
  static constexpr int kSlots = 4;
  sfrt::TableSlot slots[kSlots];
  int next_slot = 0;
  int cur_slot = -1;
  // The tables depend only on the size, the camera, the billboards and the lights: every
  // setter of those bumps tables_version, and a launch whose tables are unchanged since the
  // last staging reuses that slot (no host recomputation, no copy).
  uint64_t tables_version = 1, staged_version = 0;
  size_t staged_off[3] = {0, 0, 0};  // byte offsets of row | dyn | lights in the staged slot
  float staged_xmax = 0.0f;          // max finite |component| of the staged ray directions
  int* d_status = nullptr;
  uint32_t* d_frame = nullptr;
  size_t d_frame_px = 0;
  int tile_order_on = 0;     // SFRT_OPT_TILE_ORDER: off by default here (slower)
  sfrt::TileChains scheds;   // adaptive tile order (sfrt_sched.h), render_band; one chain per stream
  sfrt::Relay relay;         // events recorded on callers' streams, relayed (sfrt_host.h)
  std::mutex mu;

  sfrt_voxel() {
    for (auto& t : slots) t.relay = &relay;
    shared.relay = &relay;
  }

  ~sfrt_voxel() {
    sfrt::DeviceGuard g(device);
    if (stream) (void)hipStreamSynchronize(stream);
    (void)hipDeviceSynchronize();
    scheds.release();
    for (auto& t : tex) (void)hipFree(t.d);
    for (auto& t : dyn_tex) (void)hipFree(t.d);
    (void)hipDeviceSynchronize();
    (void)hipFree(d_cells);
    for (CodeStage& c : stage) {
      (void)hipFree(c.d);
      (void)hipHostFree(c.h);
      if (c.ev) (void)hipEventDestroy(c.ev);
    }
    retired_host.release();
    shared.release();
    tex_stage.release();
    for (auto& t : slots) t.release();
    relay.release();
    (void)hipFree(d_status);
    (void)hipFree(d_frame);
    if (stream) (void)hipStreamDestroy(stream);
  }

  // Builds the frame record and uploads the per-frame arrays on stream s.
  // Everything the reference recomputes per pixel but that depends only on the
  // column, the row or the object is evaluated here, with its expressions.
  int prepare(sfrt::VoxFrame& f, hipStream_t s) {
    if (blocks.empty()) return SFRT_E_EMPTY;
    if (width <= 0 || height <= 0) return SFRT_E_INVALID;
    std::memset(&f, 0, sizeof f);
    f.cam[0] = cam.pos[0]; f.cam[1] = cam.pos[1]; f.cam[2] = cam.pos[2];
    f.view_distance = view_distance;
    f.shadow_distance = shadow_distance;
    f.maxiter = to_u32(view_distance * 1.5f);                       // World.cpp:322
    // World.cpp:64-87
    const float vStart = cam.fov_v / 2;
    const float vIncreaseBy = cam.fov_v / height;
    const float vOff = std::sin(cam.hrotation);
    const float hStart = cam.rotation - cam.fov_h / 2;
    const float hIncreaseBy = cam.fov_h / width;
    if (staged_version == tables_version && cur_slot >= 0) {
      sfrt::TableSlot& t = slots[cur_slot];  // still holds this scene's tables; launched() re-marks it
      const int rc = blocks_upload(s);  // first: fill_frame reads d_cells
      if (rc != SFRT_OK) return rc;
      HIP_TRY(shared.before_read(s));
      HIP_TRY(t.use_on(s));  // staged, or last read, on another stream: wait for it
      fill_frame(f, (uint8_t*)t.d, staged_off);
      return SFRT_OK;
    }
    std::vector<float> col((size_t)width * 3), row((size_t)height * 2);
    float xmax = 0.0f;
    for (int i = 0; i < width; i++) {
      const float hray = (hStart + hIncreaseBy * i);
      const float fix = std::cos(cam.rotation - hray);
      const float dx = std::sin(hray) / fix, dz = std::cos(hray) / fix;
      col[3 * (size_t)i] = dx;
      col[3 * (size_t)i + 1] = dz;
      col[3 * (size_t)i + 2] = sfrt_math::atan2f(dz, dx);  // VAngleXZ's ray term (World.cpp:272)
      for (float c : {dx, dz})
        if (std::isfinite(c)) xmax = std::max(xmax, std::fabs(c));
    }
    for (int j = 0; j < height; j++) {
      const float vray = (vStart - j * vIncreaseBy);
      row[2 * (size_t)j] = (vOff + std::sin(vray));
      row[2 * (size_t)j + 1] = std::cos(cam.hrotation + vray);   // r->yscale
      if (std::isfinite(row[2 * (size_t)j])) xmax = std::max(xmax, std::fabs(row[2 * (size_t)j]));
    }
    std::vector<sfrt::VoxDyn> vd(dyn.size());
    for (size_t k = 0; k < dyn.size(); k++) {
      const sfrt_dynamic& d = dyn[k];
      sfrt::VoxDyn& o = vd[k];
      o.px = d.pos[0]; o.py = d.pos[1]; o.pz = d.pos[2];
      o.sx = d.size[0]; o.sy = d.size[1];
      o.r = d.r; o.g = d.g; o.b = d.b;
      o.dist = d.dist_to_camera;
      // VNormalizeXZ(d->pos - cam.pos) (World.cpp:282-285, 361)
      const float ex = d.pos[0] - cam.pos[0], ez = d.pos[2] - cam.pos[2];
      const float l = std::sqrt(ex * ex + ez * ez);
      o.atan_b = sfrt_math::atan2f(ez / l, ex / l);
      o.tex = d.texture_id;
      o.pad = 0;
    }
    std::vector<sfrt::VoxLight> vl(lights.size());
    for (size_t k = 0; k < lights.size(); k++) {
      const sfrt_light& L = lights[k];
      sfrt::VoxLight& o = vl[k];
      o.px = L.pos[0]; o.py = L.pos[1]; o.pz = L.pos[2];
      o.dd_skip = light_dd_skip(light_dd_pass(L.intensity));
      o.intensity = L.intensity; o.r = L.r; o.g = L.g; o.b = L.b;
      o.shadows = L.shadows;
    }
    // one blob per launch: col | row | dyn | lights, 16-byte aligned parts
    auto up16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    const size_t b_col = up16(col.size() * sizeof(float)), b_row = up16(row.size() * sizeof(float)),
                 b_dyn = up16(vd.size() * sizeof(sfrt::VoxDyn)),
                 b_lit = up16(vl.size() * sizeof(sfrt::VoxLight));
    const size_t bytes = b_col + b_row + b_dyn + b_lit + 16;
    sfrt::TableSlot& t = slots[next_slot];
    HIP_TRY(t.reclaim());
    HIP_TRY(t.grow(bytes, s));  // no wait on other streams (sfrt_host.h)
    uint8_t* h = (uint8_t*)t.h;
    std::memcpy(h, col.data(), col.size() * sizeof(float));
    std::memcpy(h + b_col, row.data(), row.size() * sizeof(float));
    if (!vd.empty()) std::memcpy(h + b_col + b_row, vd.data(), vd.size() * sizeof(sfrt::VoxDyn));
    if (!vl.empty())
      std::memcpy(h + b_col + b_row + b_dyn, vl.data(), vl.size() * sizeof(sfrt::VoxLight));
    HIP_TRY(hipMemcpyAsync(t.d, t.h, bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(t.staged(s));
    cur_slot = next_slot;
    next_slot = (next_slot + 1) % kSlots;
    staged_version = tables_version;
    staged_xmax = xmax;
    staged_off[0] = b_col;
    staged_off[1] = b_col + b_row;
    staged_off[2] = b_col + b_row + b_dyn;
    const int rc = blocks_upload(s);  // first: fill_frame reads d_cells
    if (rc != SFRT_OK) return rc;
    HIP_TRY(shared.before_read(s));
    fill_frame(f, (uint8_t*)t.d, staged_off);
    return SFRT_OK;
  }

  // The world as the kernel reads it: byte (x << 20) + (y << 10) + z = id + kVoxCellBias of the
  // block at (x, y, z), 0 elsewhere (the reference's map key as a linear index, voxel_trace.h).
  // nx planes of 1 MiB; each plane's ny rows of nz codes land at row pitch 1024.
  // Rare (the reference fills its map once, World.cpp:5-18) but stream-ordered like every other
  // upload: the rewrite is queued on the frame's stream s behind every launch, on any stream, that
  // read the old grid (SharedBuffer::before_write: device-side waits), and launches on other
  // streams wait for it -- a frame of another world or renderer in flight is never held up.
  // It writes only the box that holds the new world or anything an earlier one left non-zero.
  int blocks_upload(hipStream_t s) {
    if (!blocks_dirty) return SFRT_OK;
    const size_t n = blocks.size();
    CodeStage& c = stage[stage_next];
    if (c.pending) {  // this pair's previous rewrite (queued by this object, two uploads ago) has run
      HIP_TRY(hipEventSynchronize(c.ev));
      c.pending = false;
    }
    HIP_TRY(shared.before_write(s, slots));
    if (c.cap < n) {  // grows to the largest world seen (the pair is not in use: above)
      size_t cap = 1;
      while (cap < n) cap <<= 1;
      retired_host.add(c.h);  // not hipHostFree: it would wait for the whole device
      c.h = nullptr;
      if (c.d) HIP_TRY(hipFreeAsync(c.d, s));
      c.d = nullptr;
      c.cap = 0;
      HIP_TRY(hipHostMalloc(&c.h, cap, hipHostMallocDefault));
      HIP_TRY(hipMallocAsync((void**)&c.d, cap, s));
      c.cap = cap;
    }
    if (!c.ev) HIP_TRY(hipEventCreateWithFlags(&c.ev, hipEventDisableTiming));
    const size_t bytes = (size_t)nx << 20;
    if (d_cells_cap < bytes) {  // a fresh grid (stream-ordered on s), all zero
      if (d_cells) HIP_TRY(hipFreeAsync(d_cells, s));
      d_cells = nullptr;
      d_cells_cap = 0;
      HIP_TRY(hipMallocAsync((void**)&d_cells, bytes, s));
      d_cells_cap = bytes;
      HIP_TRY(hipMemsetAsync(d_cells, 0, bytes, s));
      box[0] = box[1] = box[2] = 0;
    }
    for (size_t k = 0; k < n; k++)
      c.h[k] = blocks[k] == sfrt::kVoxEmpty ? 0 : (uint8_t)(blocks[k] + sfrt::kVoxCellBias);
    HIP_TRY(hipMemcpyAsync(c.d, c.h, n, hipMemcpyHostToDevice, s));
    // planes past the new nx are outside the kernel's buffer range, but a later, larger world
    // would see them: the box covers them too while they may hold codes
    const int bx = std::max(nx, box[0]), by = std::max(ny, box[1]), bz = std::max(nz, box[2]);
    if (sfrt::launch_voxel_cells(d_cells, c.d, nx, ny, nz, bx, by, bz, s)) return SFRT_E_HIP;
    HIP_TRY(relay.record(s, c.ev));  // s may be a caller's stream
    c.pending = true;
    stage_next ^= 1;
    HIP_TRY(shared.after_write(s));
    box[0] = nx; box[1] = ny; box[2] = nz;
    blocks_dirty = false;
    return SFRT_OK;
  }

  // A texture (textures[slot] or dynTextures[slot], World.h:90-91) uploaded stream-ordered, like the
  // grid: on the object's stream behind every frame that read the old texels (SharedBuffer), a
  // larger one in a new buffer with the old one freed in that order.  Frames queued after the call
  // read the new texels; nothing waits for the device.
  int upload_texture(DevTex& t, const uint8_t* rgba, int w, int h) {
    const size_t n = (size_t)w * h;
    void* staged = nullptr;
    HIP_TRY(tex_stage.fill(rgba, n * 4, &staged));
    HIP_TRY(shared.before_write(stream, slots));
    if (t.cap < n) {
      uint32_t* d = nullptr;
      HIP_TRY(hipMallocAsync((void**)&d, n * 4, stream));
      if (t.d) HIP_TRY(hipFreeAsync(t.d, stream));
      t.d = d;
      t.cap = n;
    }
    HIP_TRY(hipMemcpyAsync(t.d, staged, n * 4, hipMemcpyHostToDevice, stream));
    HIP_TRY(tex_stage.copied(stream));
    HIP_TRY(shared.after_write(stream));
    t.w = w;
    t.h = h;
    return SFRT_OK;
  }

  // The frame record's device pointers: the staged tables at d, the grid (blocks_upload()
  // must have run: the kernel's buffer resource over d_cells has no other guard).
  void fill_frame(sfrt::VoxFrame& f, uint8_t* d, const size_t* off) {
    f.col = (const float*)d;
    f.row = (const float*)(d + off[0]);
    f.cells = d_cells;
    f.cell_bytes = (uint32_t)nx << 20;
    f.dda_qlim = dda_qlim(f.cam, f.maxiter, staged_xmax);
    for (int k = 0; k < sfrt::kVoxSlots; k++) {
      f.tex[k] = {tex[k].d, tex[k].w, tex[k].h};
      f.dyn_tex[k] = {dyn_tex[k].d, dyn_tex[k].w, dyn_tex[k].h};
      f.colors[k] = colors[k];
    }
    f.dyn = (const sfrt::VoxDyn*)(d + off[1]);
    f.ndyn = (int)dyn.size();
    f.lights = (const sfrt::VoxLight*)(d + off[2]);
    f.nlights = (int)lights.size();
    f.status = d_status;
  }

  // The current table slot's event, for the launch that reads it to record (its stop event), and
  // the slot marked busy once that launch is queued on s (the event also covers the launch's
  // read of the grid: SharedBuffer).
  void* launch_event() const { return slots[cur_slot].launch_event(); }
  hipError_t launched(hipStream_t s) { return slots[cur_slot].launched_with(s); }

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
    return (st & 2) ? SFRT_E_TEXEL : SFRT_OK;
  }
};

extern "C" {

int sfrt_voxel_create(int hip_device, sfrt_voxel** out) {
  if (!out) return SFRT_E_INVALID;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || hip_device < 0 || hip_device >= count)
    return SFRT_E_HIP;
  sfrt_voxel* v = new sfrt_voxel();
  v->device = hip_device;
  // Camera defaults (World.h:9-19) and the constructor's fov conversion (World.cpp:55-56).
  v->cam.pos[0] = 15.5f; v->cam.pos[1] = 1.9f; v->cam.pos[2] = 15.5f;
  v->cam.fov_h = 75.0f * (kPI / 180.0f);
  v->cam.fov_v = 47.0f * (kPI / 180.0f);
  sfrt::DeviceGuard g(hip_device);
  if (hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&v->d_status, sizeof(int)) != hipSuccess ||
      hipMemset(v->d_status, 0, sizeof(int)) != hipSuccess) {
    delete v;
    return SFRT_E_HIP;
  }
  *out = v;
  return SFRT_OK;
}

void sfrt_voxel_destroy(sfrt_voxel* v) { delete v; }

int sfrt_voxel_set_size(sfrt_voxel* v, int width, int height) {
  if (!v || width <= 0 || height <= 0) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(v->mu);
  v->width = width;
  v->height = height;
  v->tables_version++;
  return SFRT_OK;
}

int sfrt_voxel_set_camera(sfrt_voxel* v, const sfrt_camera* cam) {
  if (!v || !cam) return SFRT_E_INVALID;
  for (float c : {cam->pos[0], cam->pos[1], cam->pos[2], cam->rotation, cam->hrotation,
                  cam->fov_h, cam->fov_v})
    if (!std::isfinite(c)) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(v->mu);
  v->cam = *cam;
  v->tables_version++;
  return SFRT_OK;
}

int sfrt_voxel_set_view(sfrt_voxel* v, float shadow_distance, float view_distance) {
  if (!v || !std::isfinite(shadow_distance) || !std::isfinite(view_distance) || view_distance < 0)
    return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(v->mu);
  v->shadow_distance = shadow_distance;
  v->view_distance = view_distance;
  return SFRT_OK;
}

int sfrt_voxel_set_blocks(sfrt_voxel* v, const int16_t* texture_ids, int nx, int ny, int nz) {
  // The reference keys blocks by (x << 20) + (y << 10) + z (World.cpp:10); a
  // dense grid is exact for 0 <= x < 2048, 0 <= y, z < 1024.
  if (!v || !texture_ids || nx <= 0 || ny <= 0 || nz <= 0 || nx > sfrt::kVoxMaxX || ny > sfrt::kVoxMaxY || nz > sfrt::kVoxMaxZ)
    return SFRT_E_INVALID;
  const size_t n = (size_t)nx * ny * nz;
  for (size_t k = 0; k < n; k++)
    if (texture_ids[k] != sfrt::kVoxEmpty &&
        (texture_ids[k] >= sfrt::kVoxSlots || texture_ids[k] <= -sfrt::kVoxSlots))
      return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(v->mu);
  v->blocks.assign(texture_ids, texture_ids + n);
  v->nx = nx; v->ny = ny; v->nz = nz;
  v->blocks_dirty = true;
  return SFRT_OK;
}

int sfrt_voxel_load_texture(sfrt_voxel* v, int slot, const uint8_t* rgba, int w, int h) {
  if (!v || !rgba || slot < 0 || slot >= sfrt::kVoxSlots || w <= 0 || h <= 0) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(v->mu);
  sfrt::DeviceGuard g(v->device);
  return v->upload_texture(v->tex[slot], rgba, w, h);
}

int sfrt_voxel_load_dyn_texture(sfrt_voxel* v, int slot, const uint8_t* rgba, int w, int h) {
  if (!v || !rgba || slot < 0 || slot >= sfrt::kVoxSlots || w <= 0 || h <= 0) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(v->mu);
  sfrt::DeviceGuard g(v->device);
  return v->upload_texture(v->dyn_tex[slot], rgba, w, h);
}

int sfrt_voxel_set_colors(sfrt_voxel* v, const uint8_t* rgba, int count) {
  if (!v || !rgba || count < 0 || count > sfrt::kVoxSlots) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(v->mu);
  for (int k = 0; k < count; k++) std::memcpy(&v->colors[k], rgba + 4 * k, 4);
  return SFRT_OK;
}

int sfrt_voxel_set_dynamics(sfrt_voxel* v, const sfrt_dynamic* dyn, int count) {
  if (!v || count < 0 || (count > 0 && !dyn)) return SFRT_E_INVALID;
  for (int k = 0; k < count; k++)
    if (dyn[k].texture_id < 0 || dyn[k].texture_id >= sfrt::kVoxSlots) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(v->mu);
  v->dyn.assign(dyn, dyn + count);
  v->tables_version++;
  return SFRT_OK;
}

float sfrt_voxel_light_dd_pass(float intensity) { return light_dd_pass(intensity); }

int sfrt_voxel_set_lights(sfrt_voxel* v, const sfrt_light* lights, int count) {
  if (!v || count < 0 || (count > 0 && !lights)) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(v->mu);
  v->lights.assign(lights, lights + count);
  v->tables_version++;
  return SFRT_OK;
}

int sfrt_voxel_update_image(sfrt_voxel* v, uint8_t* pixels, int ystart, int yadd, int xstart,
                            int xadd) {
  if (!v || !pixels || ystart < 0 || xstart < 0 || yadd <= 0 || xadd <= 0) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(v->mu);
  const int sub_w = xstart < v->width ? (v->width - xstart + xadd - 1) / xadd : 0;
  const int sub_h = ystart < v->height ? (v->height - ystart + yadd - 1) / yadd : 0;
  if (v->blocks.empty()) return SFRT_E_EMPTY;
  if (sub_w == 0 || sub_h == 0) return SFRT_OK;
  sfrt::DeviceGuard g(v->device);
  const size_t px = (size_t)sub_w * sub_h;
  if (v->d_frame_px < px) {  // the last update_image finished with it (it waits for its copy)
    if (v->d_frame) HIP_TRY(hipFreeAsync(v->d_frame, v->stream));
    v->d_frame = nullptr;
    v->d_frame_px = 0;
    HIP_TRY(hipMallocAsync((void**)&v->d_frame, px * 4, v->stream));
    v->d_frame_px = px;
  }
  sfrt::VoxFrame f;
  int rc = v->prepare(f, v->stream);
  if (rc) return rc;
  f.xstart = xstart; f.xadd = xadd; f.ystart = ystart; f.yadd = yadd;
  f.sub_w = sub_w;
  f.sub_row0 = 0;
  f.sub_rows = sub_h;
  f.out = v->d_frame;
  f.out_pitch = sub_w;
  if (sfrt::launch_voxel(f, v->stream, v->launch_event())) return SFRT_E_HIP;
  HIP_TRY(v->launched(v->stream));
  std::vector<uint32_t> stage(px);
  HIP_TRY(hipMemcpyAsync(stage.data(), v->d_frame, px * 4, hipMemcpyDeviceToHost, v->stream));
  rc = v->read_status(v->stream);
  if (rc) return rc;
  const size_t W = (size_t)v->width;
  for (int b = 0; b < sub_h; b++) {
    const size_t j = (size_t)ystart + (size_t)b * yadd;
    for (int a = 0; a < sub_w; a++)
      std::memcpy(pixels + (j * W + (size_t)xstart + (size_t)a * xadd) * 4, &stage[(size_t)b * sub_w + a], 4);
  }
  return SFRT_OK;
}

int sfrt_voxel_render_band(sfrt_voxel* v, void* dev_pixels, int64_t pitch_bytes, int row0, int rows,
                           void* hip_stream) {
  if (!v || !dev_pixels || row0 < 0 || rows < 0 || pitch_bytes % 4 != 0) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(v->mu);
  if (pitch_bytes < (int64_t)v->width * 4 || row0 + rows > v->height) return SFRT_E_INVALID;
  if (rows == 0) return SFRT_OK;
  sfrt::DeviceGuard g(v->device);
  hipStream_t s = (hipStream_t)hip_stream;
  sfrt::VoxFrame f;
  int rc = v->prepare(f, s);
  if (rc) return rc;
  f.xstart = 0; f.xadd = 1; f.ystart = 0; f.yadd = 1;
  f.sub_w = v->width;
  f.sub_row0 = row0;
  f.sub_rows = rows;
  f.out = (uint32_t*)dev_pixels;
  f.out_pitch = pitch_bytes / 4;
  long long tiles = 0;
  const long long key = v->tile_order_on ? sfrt::voxel_tile_key(f, &tiles) : 0;
  sfrt::TileSchedPtrs p;
  sfrt::TileSched& sched = v->scheds.chain[v->scheds.pick(s)];
  HIP_TRY(sched.begin(key, tiles, s, v->tile_order_on, p));
  f.tile_order = p.tile_order;
  f.tile_cost = p.tile_cost;
  f.prev_cost = p.prev_cost;
  f.next_order = p.next_order;
  f.cost_diff = p.cost_diff ? 1 : 0;
  const bool queued = sfrt::launch_voxel(f, s, v->launch_event()) == 0;
  HIP_TRY(sched.end(p, s, queued));
  if (!queued) return SFRT_E_HIP;
  HIP_TRY(v->launched(s));
  return SFRT_OK;
}

int sfrt_voxel_set_option(sfrt_voxel* v, int option, int value) {
  if (!v) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(v->mu);
  if (option == SFRT_OPT_TILE_ORDER) {
    v->tile_order_on = value == 2 ? 2 : value ? 1 : 0;
    return SFRT_OK;
  }
  return SFRT_E_INVALID;
}

int sfrt_voxel_check(sfrt_voxel* v, void* hip_stream) {
  if (!v) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(v->mu);
  sfrt::DeviceGuard g(v->device);
  return v->read_status((hipStream_t)hip_stream);
}

}  // extern "C"
