// sfrt_glsl.cpp -- host side of the GLSL renderer: the
// shader's uniform state, the `ground` texture with its mip chain, and the
// extern "C" entry points sfrt_glsl_* of include/sfrt.h.
//
// Reference (paths under /root/reference/Raytracing/):
//   uniforms                        rayShader.frag:1-11
//   upload by name                  SphereWorld.cpp:214-238 (UpdateSpheres), Source.cpp:143-146
//   ground: Floor.png, REPEAT, mips SphereWorld.cpp:52-57
//   rt.draw(sp, &world.shader)      Source.cpp:150-153 (one fragment per render-target pixel)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "glsl_trace.h"
#include "sfrt.h"
#include "sfrt_host.h"
#include "sfrt_sched.h"
#include "sfrt_math.h"

#pragma clang fp contract(off)

namespace {

// Uniform values are bounded so that every product in the wall pass stays
// finite (the kernel's step-0 shortcut relies on it).
constexpr float kUniformBound = 1e15f;

bool bounded(float v) { return std::fabs(v) <= kUniformBound; }  // false for NaN

// Largest binary32 s >= 0 with sqrtf(s) <= r (-1 when there is none):
// step(length(rpos), r) == 1  <=>  dot(rpos, rpos) <= s_in (sqrtf is monotone).
float inside_bound(float r) {
  if (!(std::sqrt(0.0f) <= r)) return -1.0f;
  uint32_t lo = 0, hi = 0x7f7fffffu;  // sqrt(lo) <= r holds; find the last such bit pattern
  auto ok = [r](uint32_t b) { return std::sqrt(sfrt_math::u2f(b)) <= r; };
  if (ok(hi)) return sfrt_math::u2f(hi);
  while (hi - lo > 1) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (ok(mid)) lo = mid; else hi = mid;
  }
  return sfrt_math::u2f(lo);
}

// generateMipmap() as DESIGN.md 4b fixes it: 2x2 (2x1, 1x2) box average,
// rounded half up, down to 1x1.  Power-of-two sides.
void build_mips(const uint8_t* rgba, int w, int h, std::vector<uint32_t>& out, int* lw, int* lh,
                int* off, int* levels) {
  std::vector<uint8_t> cur(rgba, rgba + (size_t)w * h * 4);
  out.clear();
  int k = 0;
  for (;;) {
    lw[k] = w;
    lh[k] = h;
    off[k] = (int)out.size();
    for (size_t p = 0; p < (size_t)w * h; p++) {
      uint32_t v;
      std::memcpy(&v, &cur[p * 4], 4);
      out.push_back(v);
    }
    if (w == 1 && h == 1) break;
    const int nw = w > 1 ? w / 2 : 1, nh = h > 1 ? h / 2 : 1;
    const int fx = w > 1 ? 2 : 1, fy = h > 1 ? 2 : 1, n = fx * fy;
    std::vector<uint8_t> nxt((size_t)nw * nh * 4);
    for (int y = 0; y < nh; y++)
      for (int x = 0; x < nw; x++)
        for (int c = 0; c < 4; c++) {
          int sum = 0;
          for (int dy = 0; dy < fy; dy++)
            for (int dx = 0; dx < fx; dx++)
              sum += cur[((size_t)(y * fy + dy) * w + (x * fx + dx)) * 4 + c];
          nxt[((size_t)y * nw + x) * 4 + c] = (uint8_t)((sum + n / 2) / n);
        }
    cur.swap(nxt);
    w = nw;
    h = nh;
    k++;
  }
  *levels = k + 1;
}

bool pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }

}  // namespace

struct sfrt_glsl {
  int device = 0;
  sfrt_glsl_uniforms u{};
  int ground_w = 0, ground_h = 0;
  // SFRT_OPT_TILE_ORDER (sfrt_glsl_draw): on by default since round 4 (1080p -6 %, 4K -1 %, also
  // with the world moving every frame: profiles/ab/r4_ab9); draw_image stays row-major
  int tile_order_on = 1;
  // adaptive tile order (sfrt_sched.h), one chain per stream: draws on two streams share no order
  // or cost buffer, so neither waits on the host for the other (as the sphere world, since round 6)
  sfrt::TileChains scheds;
  // device resources
  hipStream_t stream = nullptr;
  uint32_t* d_mip = nullptr;
  // set_ground is stream-ordered: the new chain goes up on `stream` behind every draw that read
  // the old one (through the table slots' events), and draws on other streams wait for it
  sfrt::SharedBuffer ground;
  sfrt::PinnedStage mip_stage;
  int mip_levels = 0;
  int mip_w[sfrt::kGlslMipLevels] = {}, mip_h[sfrt::kGlslMipLevels] = {},
      mip_off[sfrt::kGlslMipLevels] = {};
  // Per-draw tables (walls | balls | pairs | mats) in a ring of slots, each
  // with a pinned staging copy and the event of the last draw that read it,
  // so draws on different streams never overwrite tables still in use.
  // (sfrt::TableSlot, sfrt_host.h: a reuse on another stream waits for the slot's last user.)
  static constexpr int kSlots = 4;
  sfrt::TableSlot slots[kSlots];
  int next_slot = 0;
  int cur_slot = -1;
  // The tables depend only on the uniform block: every uniform setter bumps u_version, and a
  // draw with the uniforms unchanged since the last staging reuses that slot (no host table
  // build, no copy in front of the kernel).
  uint64_t u_version = 1, staged_version = 0;
  size_t staged_off[3] = {0, 0, 0};  // byte offsets of balls | pairs | mats in the staged slot
  int* d_status = nullptr;
  uint32_t* d_frame = nullptr;
  size_t d_frame_px = 0;
  sfrt::Relay relay;         // events recorded on callers' streams, relayed (sfrt_host.h)
  std::mutex mu;

  sfrt_glsl() {
    for (auto& t : slots) t.relay = &relay;
    ground.relay = &relay;
  }

  ~sfrt_glsl() {
    sfrt::DeviceGuard g(device);
    if (stream) (void)hipStreamSynchronize(stream);
    (void)hipDeviceSynchronize();
    scheds.release();
    (void)hipFree(d_mip);
    mip_stage.release();
    ground.release();
    for (auto& t : slots) t.release();
    relay.release();
    (void)hipFree(d_status);
    (void)hipFree(d_frame);
    if (stream) (void)hipStreamDestroy(stream);
  }

  int validate() const {
    const sfrt_glsl_uniforms& v = u;
    if (v.sphere_count < 0 || v.light_count < 0 || v.all_spheres_count > SFRT_GLSL_MAX_SPHERES ||
        v.sphere_count + v.light_count > v.all_spheres_count)
      return SFRT_E_INVALID;
    for (float c : {v.campos[0], v.campos[1], v.campos[2], v.rotation[0], v.rotation[1], v.fov[0],
                    v.fov[1]})
      if (!bounded(c)) return SFRT_E_INVALID;
    if (!(v.size[0] > 0.0f && v.size[1] > 0.0f && bounded(v.size[0]) && bounded(v.size[1])))
      return SFRT_E_INVALID;
    for (int k = 0; k < v.all_spheres_count; k++)
      for (int c = 0; c < 4; c++)
        if (!bounded(v.spheres[k][c]) || !bounded(v.uvs[k][c]) || !bounded(v.lights[k][c]))
          return SFRT_E_INVALID;
    return SFRT_OK;
  }

  // Frame record + per-draw tables on stream s (stream-ordered reuse).
  int prepare(sfrt::GlslFrame& f, hipStream_t s) {
    if (!d_mip) return SFRT_E_NO_TEXTURE;
    int rc = validate();
    if (rc) return rc;
    HIP_TRY(ground.before_read(s));  // a set_ground queued on another stream lands first
    std::memset(&f, 0, sizeof f);
    const sfrt_glsl_uniforms& v = u;
    const int sc = v.sphere_count, lc = v.light_count, all = v.all_spheres_count;
    // main(), rayShader.frag:165-173 -- VRotateX / VRotateY (:16-25) on unit axes
    auto rot_x = [](const float* a, float amount, float* o) {
      const float s = std::sin(amount), c = std::cos(amount);
      o[0] = a[0];
      o[1] = a[1] * c - a[2] * s;
      o[2] = a[1] * s + a[2] * c;
    };
    auto rot_y = [](const float* a, float amount, float* o) {
      const float s = std::sin(amount), c = std::cos(amount);
      o[0] = a[0] * c + a[2] * s;
      o[1] = a[1];
      o[2] = -a[0] * s + a[2] * c;
    };
    const float ey[3] = {0, 1, 0}, ez[3] = {0, 0, 1}, ex[3] = {1, 0, 0};
    float up0[3], fwd0[3];
    rot_x(ey, -v.rotation[1], up0);
    rot_x(ez, -v.rotation[1], fwd0);
    rot_y(ex, v.rotation[0], f.right);
    rot_y(fwd0, v.rotation[0], f.fwd);
    rot_y(up0, v.rotation[0], f.up);
    for (int c = 0; c < 3; c++) f.campos[c] = v.campos[c];
    f.fov_x = v.fov[0];
    f.fov_y = v.fov[1];
    f.hk = v.fov[0] / v.size[0] * 2.0f;
    f.vk = v.fov[1] / v.size[1] * 2.0f;
    f.sc = sc;
    f.lc = lc;
    f.all = all;
    f.cam_negzero = (std::signbit(v.campos[0]) && v.campos[0] == 0.0f) ||
                    (std::signbit(v.campos[1]) && v.campos[1] == 0.0f) ||
                    (std::signbit(v.campos[2]) && v.campos[2] == 0.0f);
    // tables
    const int nb = all - sc, ns = all - sc - lc;
    std::vector<sfrt::GlslWall> walls(sc > 0 ? sc : 1);
    for (int k = 0; k < sc; k++) {
      const float* S = v.spheres[k];
      walls[k] = {S[0], S[1], S[2], S[3], S[3] * S[3], inside_bound(S[3]), 0.0f, 0.0f};
    }
    // Every lane starts at campos: the wall-pass iterations before the first
    // wall containing campos (same test as the kernel) are no-ops for all of
    // them.  With a -0.0 in campos the kernel's literal update runs from 0.
    f.wall_start = 0;
    if (!f.cam_negzero && sc > 0) {
      int j = 0;
      for (; j < sc; j++) {
        const float rx = v.campos[0] - walls[j].x, ry = v.campos[1] - walls[j].y,
                    rz = v.campos[2] - walls[j].z;
        if ((rx * rx + ry * ry) + rz * rz <= walls[j].s_in) break;
      }
      f.wall_start = j < sc ? j : 3 * sc;  // inside no wall: no lane ever moves
    }
    // The wall cull's margin: every wall-pass position lies inside (or on) some wall reached from
    // campos, so its coordinates are bounded by R = max(|campos|, max_k |c_k| + r_k); the
    // positions' binary32 drift over <= 3 sc moves (an add and a multiply each, each rounding
    // within 2^-24 R) stays below 2 * 3 * sc * 2^-24 R < 2.3e-5 R for sc <= 64
    static_assert(2.0 * 3.0 * 64.0 * 0x1.0p-24 < 1e-3 / 8, "the margin dwarfs the drift");
    f.wall_cull_margin = 0.0f;
    if (!f.cam_negzero && sc > 0 && sc <= 64) {
      double R = std::max({std::fabs((double)v.campos[0]), std::fabs((double)v.campos[1]),
                           std::fabs((double)v.campos[2])});
      for (int k = 0; k < sc; k++)
        for (int c = 0; c < 3; c++)
          R = std::max(R, std::fabs((double)v.spheres[k][c]) + std::fabs((double)v.spheres[k][3]));
      const double m = 1e-3 * R + 1e-4;
      if (std::isfinite(m) && m < 1e30) f.wall_cull_margin = (float)m;
    }
    if (staged_version == u_version && cur_slot >= 0) {  // launched() re-marks the slot
      HIP_TRY(slots[cur_slot].use_on(s));  // staged, or last read, on another stream: wait for it
      fill_tables(f, (uint8_t*)slots[cur_slot].d, staged_off);
      return SFRT_OK;
    }
    std::vector<sfrt::GlslBall> balls(nb > 0 ? nb : 1);
    for (int k = 0; k < nb; k++) {
      const float* S = v.spheres[sc + k];
      // r_skip: r * (1 + 6e-6) rounded up, the dominance test's inflated radius (glsl_trace.hip
      // kThrMul); NaN for r < 0 or NaN, so such a ball is never skipped
      const float rs = S[3] >= 0.0f ? std::nextafter(S[3] * 0x1.000065p+0f, INFINITY) : NAN;
      balls[k] = {S[0], S[1], S[2], S[3], rs, 0.0f, 0.0f, 0.0f};
    }
    std::vector<sfrt::GlslPair> pairs(lc * ns > 0 ? lc * ns : 1);
    for (int li = 0; li < lc; li++)
      for (int k = 0; k < ns; k++) {
        const float* A = v.spheres[sc + li];
        const float* B = v.spheres[sc + lc + k];
        const float qx = A[0] - B[0], qy = A[1] - B[1], qz = A[2] - B[2];
        const float dist = std::sqrt((qx * qx + qy * qy) + qz * qz);    // distance (:140)
        sfrt::GlslPair& P = pairs[li * ns + k];
        P.dist = dist;
        P.sanglet = sfrt_math::atan2f(B[3], dist);                       // :141
        P.ux = (B[0] - A[0]) / dist;                                     // :142
        P.uy = (B[1] - A[1]) / dist;
        P.uz = (B[2] - A[2]) / dist;
        P.bx = B[0];
        P.by = B[1];
        P.bz = B[2];
        // acos(dot) >= sanglet * (1 + 1e-3) + 1e-3 suffices for a factor of 1
        // (DESIGN.md 5c); only for balls near the camera (|pos - ball| < 2000).
        const float cx = v.campos[0] - B[0], cy = v.campos[1] - B[1], cz = v.campos[2] - B[2];
        const float dcam = std::sqrt((cx * cx + cy * cy) + cz * cz);
        P.cos_lit = (P.sanglet > 0.0f && P.sanglet < 1.0f && dcam < 1000.0f)
                        ? std::cos(P.sanglet * 1.001f + 1e-3f) : -2.0f;
      }
    std::vector<sfrt::GlslMat> mats(sfrt::kGlslMax);
    for (int k = 0; k < sfrt::kGlslMax; k++) {
      sfrt::GlslMat& M = mats[k];
      std::memcpy(M.uv, v.uvs[k], sizeof M.uv);
      std::memcpy(M.light, v.lights[k], sizeof M.light);
      M.cx = v.spheres[k][0];
      M.cy = v.spheres[k][1];
      M.cz = v.spheres[k][2];
      M.pad = 0.0f;
    }
    const size_t bw = walls.size() * sizeof walls[0], bb = balls.size() * sizeof balls[0],
                 bp = pairs.size() * sizeof pairs[0], bm = mats.size() * sizeof mats[0];
    const size_t bytes = bw + bb + bp + bm;
    sfrt::TableSlot& t = slots[next_slot];
    HIP_TRY(t.reclaim());
    HIP_TRY(t.grow(bytes, s));  // no wait on other streams (sfrt_host.h)
    uint8_t* blob = (uint8_t*)t.h;
    std::memcpy(blob, walls.data(), bw);
    std::memcpy(blob + bw, balls.data(), bb);
    std::memcpy(blob + bw + bb, pairs.data(), bp);
    std::memcpy(blob + bw + bb + bp, mats.data(), bm);
    HIP_TRY(hipMemcpyAsync(t.d, blob, bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(t.staged(s));
    cur_slot = next_slot;
    next_slot = (next_slot + 1) % kSlots;
    staged_version = u_version;
    staged_off[0] = bw;
    staged_off[1] = bw + bb;
    staged_off[2] = bw + bb + bp;
    fill_tables(f, (uint8_t*)t.d, staged_off);
    return SFRT_OK;
  }

  // The frame record's device pointers: the staged tables at base, the ground's mip chain.
  void fill_tables(sfrt::GlslFrame& f, uint8_t* base, const size_t* off) {
    f.walls = (const sfrt::GlslWall*)base;
    f.balls = (const sfrt::GlslBall*)(base + off[0]);
    f.pairs = (const sfrt::GlslPair*)(base + off[1]);
    f.mats = (const sfrt::GlslMat*)(base + off[2]);
    f.mip = d_mip;
    f.mip_levels = mip_levels;
    for (int k = 0; k < sfrt::kGlslMipLevels; k++) {
      f.mip_w[k] = mip_w[k];
      f.mip_h[k] = mip_h[k];
      f.mip_off[k] = mip_off[k];
    }
    f.status = d_status;
  }

  // The current table slot's event, for the launch that reads it to record (its stop event:
  // sfrt_host.h TableSlot::launch_event), and the slot marked busy once that launch is queued.
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
    return (st & 1) ? SFRT_E_MARCH_LIMIT : SFRT_OK;
  }
};

namespace {

// "spheres[12]" -> ("spheres", 12); plain names -> index -1.
bool parse_name(const char* name, char* base, size_t cap, int* index) {
  const char* br = std::strchr(name, '[');
  size_t n = br ? (size_t)(br - name) : std::strlen(name);
  if (n == 0 || n >= cap) return false;
  std::memcpy(base, name, n);
  base[n] = 0;
  *index = -1;
  if (br) {
    char* end = nullptr;
    const long k = std::strtol(br + 1, &end, 10);
    if (end == br + 1 || *end != ']' || end[1] != 0 || k < 0 || k >= SFRT_GLSL_MAX_SPHERES)
      return false;
    *index = (int)k;
  }
  return true;
}

}  // namespace

extern "C" {

int sfrt_glsl_create(int hip_device, sfrt_glsl** out) {
  if (!out) return SFRT_E_INVALID;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || hip_device < 0 || hip_device >= count)
    return SFRT_E_HIP;
  sfrt_glsl* g = new sfrt_glsl();
  g->device = hip_device;
  sfrt::DeviceGuard dg(hip_device);
  if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&g->d_status, sizeof(int)) != hipSuccess ||
      hipMemset(g->d_status, 0, sizeof(int)) != hipSuccess) {
    delete g;
    return SFRT_E_HIP;
  }
  *out = g;
  return SFRT_OK;
}

void sfrt_glsl_destroy(sfrt_glsl* g) { delete g; }

int sfrt_glsl_set_ground(sfrt_glsl* g, const uint8_t* rgba, int w, int h) {
  if (!g || !rgba || !pow2(w) || !pow2(h) || w > 32768 || h > 32768) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(g->mu);
  std::vector<uint32_t> chain;
  int lw[sfrt::kGlslMipLevels], lh[sfrt::kGlslMipLevels], off[sfrt::kGlslMipLevels], levels = 0;
  build_mips(rgba, w, h, chain, lw, lh, off, &levels);
  sfrt::DeviceGuard dg(g->device);
  // Stream-ordered, no device-wide wait: the new chain goes up on the object's stream behind every
  // draw that read the old one (device-side waits on the table slots' events, sfrt::SharedBuffer)
  // and the old chain is freed in that order; draws on other streams wait for the upload.
  const size_t bytes = chain.size() * 4;
  void* staged = nullptr;
  HIP_TRY(g->mip_stage.fill(chain.data(), bytes, &staged));
  HIP_TRY(g->ground.before_write(g->stream, g->slots));
  uint32_t* chain_d = nullptr;
  HIP_TRY(hipMallocAsync((void**)&chain_d, bytes, g->stream));
  HIP_TRY(hipMemcpyAsync(chain_d, staged, bytes, hipMemcpyHostToDevice, g->stream));
  HIP_TRY(g->mip_stage.copied(g->stream));
  if (g->d_mip) HIP_TRY(hipFreeAsync(g->d_mip, g->stream));
  g->d_mip = chain_d;
  HIP_TRY(g->ground.after_write(g->stream));
  g->mip_levels = levels;
  for (int k = 0; k < sfrt::kGlslMipLevels; k++) {
    g->mip_w[k] = k < levels ? lw[k] : 0;
    g->mip_h[k] = k < levels ? lh[k] : 0;
    g->mip_off[k] = k < levels ? off[k] : 0;
  }
  g->ground_w = w;
  g->ground_h = h;
  return SFRT_OK;
}

int sfrt_glsl_set_uniforms(sfrt_glsl* g, const sfrt_glsl_uniforms* u) {
  if (!g || !u) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(g->mu);
  g->u = *u;
  g->u_version++;
  return SFRT_OK;
}

int sfrt_glsl_get_uniforms(sfrt_glsl* g, sfrt_glsl_uniforms* u) {
  if (!g || !u) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(g->mu);
  *u = g->u;
  return SFRT_OK;
}

int sfrt_glsl_set_uniform(sfrt_glsl* g, const char* name, const float* v, int n) {
  if (!g || !name || !v || n < 1 || n > 4) return SFRT_E_INVALID;
  char base[32];
  int k;
  if (!parse_name(name, base, sizeof base, &k)) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(g->mu);
  sfrt_glsl_uniforms& u = g->u;
  float* dst = nullptr;
  int want = 0;
  if (k < 0) {
    if (!std::strcmp(base, "campos")) dst = u.campos, want = 3;
    else if (!std::strcmp(base, "rotation")) dst = u.rotation, want = 2;
    else if (!std::strcmp(base, "fov")) dst = u.fov, want = 2;
    else if (!std::strcmp(base, "size")) dst = u.size, want = 2;
  } else {
    if (!std::strcmp(base, "spheres")) dst = u.spheres[k], want = 4;
    else if (!std::strcmp(base, "uvs")) dst = u.uvs[k], want = 4;
    else if (!std::strcmp(base, "lights")) dst = u.lights[k], want = 4;
  }
  if (!dst || n != want) return SFRT_E_INVALID;
  std::memcpy(dst, v, sizeof(float) * n);
  g->u_version++;
  return SFRT_OK;
}

int sfrt_glsl_set_uniform_int(sfrt_glsl* g, const char* name, int value) {
  if (!g || !name) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(g->mu);
  if (!std::strcmp(name, "sphereCount")) g->u.sphere_count = value;
  else if (!std::strcmp(name, "allSpheresCount")) g->u.all_spheres_count = value;
  else if (!std::strcmp(name, "lightCount")) g->u.light_count = value;
  else return SFRT_E_INVALID;
  g->u_version++;
  return SFRT_OK;
}

int sfrt_glsl_draw(sfrt_glsl* g, void* dev_pixels, int width, int height, int64_t pitch_bytes,
                   int row0, int rows, void* hip_stream) {
  if (!g || !dev_pixels || width <= 0 || height <= 0 || row0 < 0 || rows < 0 ||
      row0 + rows > height || pitch_bytes < (int64_t)width * 4 || pitch_bytes % 4 != 0 ||
      height >= (1 << 24) || width >= (1 << 24))
    return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(g->mu);
  sfrt::DeviceGuard dg(g->device);
  hipStream_t s = (hipStream_t)hip_stream;
  sfrt::GlslFrame f;
  if (rows == 0) return SFRT_OK;
  const int rc = g->prepare(f, s);
  if (rc) return rc;
  f.width = width;
  f.height = height;
  f.row0 = row0;
  f.rows = rows;
  f.tiles_x = (width + 7) / 8;
  f.out = (uint32_t*)dev_pixels;
  f.out_pitch = pitch_bytes / 4;
  long long tiles = 0;
  const long long key = g->tile_order_on ? sfrt::glsl_tile_key(f, &tiles) : 0;
  sfrt::TileSchedPtrs p;
  sfrt::TileSched& sched = g->scheds.chain[g->scheds.pick(s)];
  HIP_TRY(sched.begin(key, tiles, s, g->tile_order_on, p));
  f.tile_order = p.tile_order;
  f.tile_cost = p.tile_cost;
  f.prev_cost = p.prev_cost;
  f.next_order = p.next_order;
  f.cost_diff = p.cost_diff ? 1 : 0;
  const bool queued = sfrt::launch_glsl(f, s, g->launch_event()) == 0;
  HIP_TRY(sched.end(p, s, queued));
  if (!queued) return SFRT_E_HIP;
  HIP_TRY(g->launched(s));
  return SFRT_OK;
}

int sfrt_glsl_draw_image(sfrt_glsl* g, uint8_t* pixels, int width, int height) {
  if (!g || !pixels || width <= 0 || height <= 0 || height >= (1 << 24) || width >= (1 << 24))
    return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(g->mu);
  sfrt::DeviceGuard dg(g->device);
  const size_t px = (size_t)width * height;
  if (g->d_frame_px < px) {  // stream-ordered behind the last draw_image on the object's stream
    if (g->d_frame) HIP_TRY(hipFreeAsync(g->d_frame, g->stream));
    g->d_frame = nullptr;
    g->d_frame_px = 0;
    HIP_TRY(hipMallocAsync((void**)&g->d_frame, px * 4, g->stream));
    g->d_frame_px = px;
  }
  sfrt::GlslFrame f;
  int rc = g->prepare(f, g->stream);
  if (rc) return rc;
  f.width = width;
  f.height = height;
  f.row0 = 0;
  f.rows = height;
  f.tiles_x = (width + 7) / 8;
  f.out = g->d_frame;
  f.out_pitch = width;
  if (sfrt::launch_glsl(f, g->stream, g->launch_event())) return SFRT_E_HIP;
  HIP_TRY(g->launched(g->stream));
  HIP_TRY(hipMemcpyAsync(pixels, g->d_frame, px * 4, hipMemcpyDeviceToHost, g->stream));
  return g->read_status(g->stream);
}

int sfrt_glsl_set_option(sfrt_glsl* g, int option, int value) {
  if (!g) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(g->mu);
  if (option == SFRT_OPT_TILE_ORDER) {
    g->tile_order_on = value == 2 ? 2 : value ? 1 : 0;
    return SFRT_OK;
  }
  return SFRT_E_INVALID;
}

int sfrt_glsl_check(sfrt_glsl* g, void* hip_stream) {
  if (!g) return SFRT_E_INVALID;
  std::lock_guard<std::mutex> lk(g->mu);
  sfrt::DeviceGuard dg(g->device);
  return g->read_status((hipStream_t)hip_stream);
}

}  // extern "C"
