// sfrt.hpp -- header-only C++ host mirror of the reference's classes over the
// C ABI (include/sfrt.h), for a drop-in at the reference's own call sites.
//
// The reference's renderers are C++ classes whose public state the caller
// mutates and whose frame fill reads it (paths under /root/reference/Raytracing/):
//   sfrt::SphereWorld  <- class SphereWorld (SphereWorld.h:40-78): width,
//                         height, cam, AddSphere, UpdateSpheres, UpdateImage
//   sfrt::MultiSphereWorld <- the same SphereWorld, its frame filled by several
//                         GPUs of the node (row bands gathered on the first one)
//   sfrt::VoxelWorld   <- class World (World.h:58-97): width, height, cam,
//                         shadowDistance, viewDistance, UpdateImage
//   sfrt::Shader       <- sf::Shader running rayShader.frag: setUniform by name,
//                         and rt.draw(sp, &shader) (Source.cpp:143-153)
// Names, argument meaning and the image orientation follow the reference.
// Errors the reference cannot report become sfrt::Error exceptions carrying
// the C ABI code (there is no silent fallback; without a HIP device the
// constructors throw).
#pragma once

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "sfrt.h"

namespace sfrt {

class Error : public std::runtime_error {
 public:
  Error(int code, const std::string& what)
      : std::runtime_error(what + ": " + sfrt_error_string(code)), code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

inline void check(int rc, const char* what) {
  if (rc != SFRT_OK) throw Error(rc, what);
}

struct Vector2f {
  float x = 0, y = 0;
};
struct Vector3f {
  float x = 0, y = 0, z = 0;
};
struct Vec4 {  // sf::Glsl::Vec4
  float x = 0, y = 0, z = 0, w = 0;
};

// struct Camera, the fields the frame fill reads (SphereWorld.h:10-21; World.h:9-19).
struct Camera {
  Vector3f pos;
  float rotation = 0;
  float hrotation = 0;
  float fovH = 0;  // radians, as after the constructors' conversion
  float fovV = 0;
};

// sf::Image::loadFromFile for textures: PNG bytes -> RGBA8 (stb_image's 4-channel rules).
struct Image {
  std::vector<uint8_t> pixels;
  int width = 0, height = 0;
  bool loadFromMemory(const void* data, size_t size) {
    int w = 0, h = 0;
    if (sfrt_png_info(static_cast<const uint8_t*>(data), (int64_t)size, &w, &h) != SFRT_OK)
      return false;
    pixels.resize((size_t)w * h * 4);
    if (sfrt_png_decode(static_cast<const uint8_t*>(data), (int64_t)size, pixels.data(),
                        (int64_t)pixels.size(), &w, &h) != SFRT_OK)
      return false;
    width = w;
    height = h;
    return true;
  }
  bool loadFromFile(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    std::vector<uint8_t> bytes;
    uint8_t buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) bytes.insert(bytes.end(), buf, buf + n);
    std::fclose(f);
    return loadFromMemory(bytes.data(), bytes.size());
  }
};

inline sfrt_camera to_c(const Camera& c) {
  sfrt_camera o{};
  o.pos[0] = c.pos.x;
  o.pos[1] = c.pos.y;
  o.pos[2] = c.pos.z;
  o.rotation = c.rotation;
  o.hrotation = c.hrotation;
  o.fov_h = c.fovH;
  o.fov_v = c.fovV;
  return o;
}

// ---------------------------------------------------------------------------
// SphereWorld (SphereWorld.h:40-78): the sphere-cave frame fill.
class SphereWorld {
 public:
  int width = 320;   // SphereWorld.h:50-51
  int height = 180;
  Camera cam;        // fov 75/47 degrees converted as SphereWorld.cpp:72-73

  explicit SphereWorld(int hip_device = 0) {
    check(sfrt_world_create(hip_device, &w_), "sfrt_world_create");
    sfrt_camera c;
    sfrt_world_get_camera(w_, &c);
    cam.fovH = c.fov_h;
    cam.fovV = c.fov_v;
  }
  ~SphereWorld() { sfrt_world_destroy(w_); }
  SphereWorld(const SphereWorld&) = delete;
  SphereWorld& operator=(const SphereWorld&) = delete;

  // textures[0].loadFromFile("Floor.png") (SphereWorld.cpp:52)
  void LoadTexture(const Image& img) {
    check(sfrt_world_load_texture(w_, 0, img.pixels.data(), img.width, img.height),
          "load_texture");
  }
  // SphereWorld::AddSphere (SphereWorld.cpp:177-190): containment pruning + UpdateSpheres.
  void AddSphere(Vector3f pos, float radius) {
    push_camera();
    check(sfrt_world_add_sphere(w_, pos.x, pos.y, pos.z, radius), "AddSphere");
  }
  // SphereWorld::UpdateSpheres sort (SphereWorld.cpp:199-212), against the current cam.pos.
  void UpdateSpheres() {
    push_camera();
    check(sfrt_world_update_spheres(w_), "UpdateSpheres");
  }
  std::vector<sfrt_sphere> Spheres() const {
    int n = 0;
    check(sfrt_world_get_spheres(w_, nullptr, 0, &n), "get_spheres");
    std::vector<sfrt_sphere> out((size_t)n);
    check(sfrt_world_get_spheres(w_, out.data(), n, &n), "get_spheres");
    return out;
  }
  // SphereWorld::UpdateImage (SphereWorld.cpp:83-112) into a caller-owned sf::Uint8*
  // RGBA8 frame of width*height pixels; only the addressed subset is written.
  void UpdateImage(uint8_t* pixels, short ystart, short yadd, short xstart, short xadd) {
    push_state();
    check(sfrt_world_update_image(w_, pixels, ystart, yadd, xstart, xadd), "UpdateImage");
  }
  // The same into an sf::Image-like object (setPixel(x, y, ColorT(r, g, b, a))), as the
  // reference's signature: world.UpdateImage<sf::Color>(&image, ystart, yadd, xstart, xadd).
  template <class ColorT, class ImageT>
  void UpdateImage(ImageT* v, short ystart, short yadd, short xstart, short xadd) {
    std::vector<uint8_t> frame((size_t)width * height * 4);
    UpdateImage(frame.data(), ystart, yadd, xstart, xadd);
    for (int i = xstart; i < width; i += xadd)
      for (int j = ystart; j < height; j += yadd) {
        const uint8_t* p = &frame[((size_t)j * width + i) * 4];
        v->setPixel((unsigned)i, (unsigned)j, ColorT(p[0], p[1], p[2], p[3]));
      }
  }
  // Device-resident fill of rows [row0, row0+rows) (display / multi-GPU path).
  void RenderBand(void* dev_pixels, int64_t pitch_bytes, int row0, int rows, void* hip_stream) {
    push_state();
    check(sfrt_world_render_band(w_, dev_pixels, pitch_bytes, row0, rows, hip_stream),
          "render_band");
  }
  void Check(void* hip_stream = nullptr) { check(sfrt_world_check(w_, hip_stream), "check"); }
  sfrt_world* handle() { return w_; }

 private:
  void push_camera() {
    const sfrt_camera c = to_c(cam);
    check(sfrt_world_set_camera(w_, &c), "set_camera");
  }
  void push_state() {
    check(sfrt_world_set_size(w_, width, height), "set_size");
    push_camera();
  }
  sfrt_world* w_ = nullptr;
};

// ---------------------------------------------------------------------------
// MultiSphereWorld: SphereWorld's state and frame fill over the GPUs `devices`
// (sfrt_multi_*: row bands with global row indices, gathered on devices[0] by
// RCCL or peer copies).  UpdateImage fills the whole frame, as the reference's
// eight RenderThreads together do once per full cycle (Source.cpp:17-28).
class MultiSphereWorld {
 public:
  int width = 320;
  int height = 180;
  Camera cam;

  explicit MultiSphereWorld(const std::vector<int>& devices, int transport = SFRT_MULTI_AUTO) {
    check(sfrt_multi_create(devices.data(), (int)devices.size(), transport, &m_),
          "sfrt_multi_create");
    sfrt_world* w0 = nullptr;
    sfrt_multi_world(m_, 0, &w0);
    sfrt_camera c;
    sfrt_world_get_camera(w0, &c);
    cam.fovH = c.fov_h;
    cam.fovV = c.fov_v;
  }
  ~MultiSphereWorld() { sfrt_multi_destroy(m_); }
  MultiSphereWorld(const MultiSphereWorld&) = delete;
  MultiSphereWorld& operator=(const MultiSphereWorld&) = delete;

  void LoadTexture(const Image& img) {
    check(sfrt_multi_load_texture(m_, 0, img.pixels.data(), img.width, img.height),
          "multi_load_texture");
  }
  void AddSphere(Vector3f pos, float radius) {
    push_camera();
    check(sfrt_multi_add_sphere(m_, pos.x, pos.y, pos.z, radius), "AddSphere");
  }
  void UpdateSpheres() {
    push_camera();
    check(sfrt_multi_update_spheres(m_), "UpdateSpheres");
  }
  void SetSpheres(const std::vector<sfrt_sphere>& s) {
    check(sfrt_multi_set_spheres(m_, s.data(), (int)s.size()), "set_spheres");
  }
  // Rows per GPU (rank 0 first; empty = equal bands).
  void SetBands(const std::vector<int>& rows) {
    check(sfrt_multi_set_bands(m_, rows.empty() ? nullptr : rows.data(), (int)rows.size()),
          "set_bands");
  }
  // Cost-weighted bands from the last frame's per-row march work (sfrt_multi_balance):
  // rank 0 (no link) gets root_factor shares of the work, every other GPU one share.
  void Balance(float root_factor = 1.0f) { check(sfrt_multi_balance(m_, root_factor), "balance"); }
  // Band transfer format: SFRT_TRANSFER_AUTO (default: packed RGB + alpha bit when every
  // texel's alpha is 0 or 255), SFRT_TRANSFER_RGBA or SFRT_TRANSFER_PACKED.
  void SetTransfer(int format) { check(sfrt_multi_set_transfer(m_, format), "set_transfer"); }
  // The whole frame into a caller-owned sf::Uint8* RGBA8 buffer (width*height*4).
  void UpdateImage(uint8_t* pixels) {
    push_state();
    check(sfrt_multi_update_image(m_, pixels), "UpdateImage");
  }
  // The whole frame into device memory on devices[0] (pitch width*4), queued after
  // hip_stream's work; complete when hip_stream passes this point.
  void Render(void* dev_frame, void* hip_stream) {
    push_state();
    check(sfrt_multi_render(m_, dev_frame, (int64_t)width * 4, hip_stream), "render");
  }
  void Check() { check(sfrt_multi_check(m_), "check"); }
  sfrt_multi* handle() { return m_; }

 private:
  void push_camera() {
    const sfrt_camera c = to_c(cam);
    check(sfrt_multi_set_camera(m_, &c), "set_camera");
  }
  void push_state() {
    check(sfrt_multi_set_size(m_, width, height), "set_size");
    push_camera();
  }
  sfrt_multi* m_ = nullptr;
};

// ---------------------------------------------------------------------------
// VoxelWorld (World.h:58-97): the voxel frame fill over a World snapshot.
class VoxelWorld {
 public:
  int width = 320;               // World.h:67-68
  int height = 180;
  Camera cam;                    // World.h:9-19 defaults, fov converted as World.cpp:55-56
  float shadowDistance = 16.0f;  // World.h:70
  float viewDistance = 24.0f;    // World.h:71

  explicit VoxelWorld(int hip_device = 0) {
    check(sfrt_voxel_create(hip_device, &v_), "sfrt_voxel_create");
    cam.pos = {15.5f, 1.9f, 15.5f};
    cam.fovH = 75.0f * (3.1415926535f / 180.0f);
    cam.fovV = 47.0f * (3.1415926535f / 180.0f);
  }
  ~VoxelWorld() { sfrt_voxel_destroy(v_); }
  VoxelWorld(const VoxelWorld&) = delete;
  VoxelWorld& operator=(const VoxelWorld&) = delete;

  void SetBlocks(const std::vector<int16_t>& ids, int nx, int ny, int nz) {
    check(sfrt_voxel_set_blocks(v_, ids.data(), nx, ny, nz), "set_blocks");
  }
  void LoadTexture(int slot, const Image& img) {
    check(sfrt_voxel_load_texture(v_, slot, img.pixels.data(), img.width, img.height),
          "load_texture");
  }
  void LoadDynTexture(int slot, const Image& img) {
    check(sfrt_voxel_load_dyn_texture(v_, slot, img.pixels.data(), img.width, img.height),
          "load_dyn_texture");
  }
  void SetColors(const std::vector<uint8_t>& rgba) {
    check(sfrt_voxel_set_colors(v_, rgba.data(), (int)(rgba.size() / 4)), "set_colors");
  }
  void SetDynamics(const std::vector<sfrt_dynamic>& dyn) {
    check(sfrt_voxel_set_dynamics(v_, dyn.data(), (int)dyn.size()), "set_dynamics");
  }
  void SetLights(const std::vector<sfrt_light>& lights) {
    check(sfrt_voxel_set_lights(v_, lights.data(), (int)lights.size()), "set_lights");
  }
  // World::UpdateImage (World.cpp:62-87) into a caller-owned RGBA8 frame.
  void UpdateImage(uint8_t* pixels, short ystart, short yadd, short xstart, short xadd) {
    push_state();
    check(sfrt_voxel_update_image(v_, pixels, ystart, yadd, xstart, xadd), "UpdateImage");
  }
  void RenderBand(void* dev_pixels, int64_t pitch_bytes, int row0, int rows, void* hip_stream) {
    push_state();
    check(sfrt_voxel_render_band(v_, dev_pixels, pitch_bytes, row0, rows, hip_stream),
          "render_band");
  }
  void Check(void* hip_stream = nullptr) { check(sfrt_voxel_check(v_, hip_stream), "check"); }

 private:
  void push_state() {
    check(sfrt_voxel_set_size(v_, width, height), "set_size");
    const sfrt_camera c = to_c(cam);
    check(sfrt_voxel_set_camera(v_, &c), "set_camera");
    check(sfrt_voxel_set_view(v_, shadowDistance, viewDistance), "set_view");
  }
  sfrt_voxel* v_ = nullptr;
};

// ---------------------------------------------------------------------------
// Shader: sf::Shader with rayShader.frag loaded (SphereWorld.cpp:47), its
// setUniform calls (SphereWorld.cpp:214-238, Source.cpp:143-146) and the draw
// of a width x height render target (Source.cpp:150-153).
class Shader {
 public:
  explicit Shader(int hip_device = 0) { check(sfrt_glsl_create(hip_device, &g_), "sfrt_glsl_create"); }
  ~Shader() { sfrt_glsl_destroy(g_); }
  Shader(const Shader&) = delete;
  Shader& operator=(const Shader&) = delete;

  // setUniform("ground", texture) with setRepeated(true) + generateMipmap()
  void setGround(const Image& img) {
    check(sfrt_glsl_set_ground(g_, img.pixels.data(), img.width, img.height), "set_ground");
  }
  void setUniform(const std::string& name, float x) { set(name, &x, 1); }
  void setUniform(const std::string& name, Vector2f v) {
    const float f[2] = {v.x, v.y};
    set(name, f, 2);
  }
  void setUniform(const std::string& name, Vector3f v) {
    const float f[3] = {v.x, v.y, v.z};
    set(name, f, 3);
  }
  void setUniform(const std::string& name, Vec4 v) {
    const float f[4] = {v.x, v.y, v.z, v.w};
    set(name, f, 4);
  }
  void setUniform(const std::string& name, int v) {
    check(sfrt_glsl_set_uniform_int(g_, name.c_str(), v), name.c_str());
  }
  // rt.draw(sp, &shader) into device memory, rows [row0, row0+rows) of the target.
  void draw(void* dev_pixels, int width, int height, int64_t pitch_bytes, int row0, int rows,
            void* hip_stream) {
    check(sfrt_glsl_draw(g_, dev_pixels, width, height, pitch_bytes, row0, rows, hip_stream),
          "draw");
  }
  // rt.draw + rt.getTexture().copyToImage() into a host RGBA8 frame.
  void drawImage(uint8_t* pixels, int width, int height) {
    check(sfrt_glsl_draw_image(g_, pixels, width, height), "draw_image");
  }
  sfrt_glsl* handle() { return g_; }

 private:
  void set(const std::string& name, const float* v, int n) {
    check(sfrt_glsl_set_uniform(g_, name.c_str(), v, n), name.c_str());
  }
  sfrt_glsl* g_ = nullptr;
};

}  // namespace sfrt
