/*
 * sfrt.h -- C ABI of the MI355X sphere-cave tracer (libsfrt.so).
 *
 * Drop-in for the reference's CPU frame fill
 *   void SphereWorld::UpdateImage(sf::Image* v, short ystart, short yadd,
 *                                 short xstart, short xadd)
 *   (/root/reference/Raytracing/SphereWorld.h:43, SphereWorld.cpp:83-112)
 * and the scene state it reads (SphereWorld.h:50-57,74).  `sf::Uint8` is
 * `unsigned char`, so an SFML caller passes its own RGBA8 buffer (the bytes
 * it would give to sf::Texture::update / sf::Image::create); see
 * INTEGRATION.md.  Plain C types only: no HIP, torch or SFML types cross this
 * boundary.  All functions return 0 (SFRT_OK) or a negative SFRT_E_* code.
 * A world is safe to call from several host threads (calls serialise on an
 * internal mutex); distinct worlds are independent.
 */
#ifndef SFRT_H
#define SFRT_H

#include <stdint.h>

#if defined(__GNUC__)
#define SFRT_API __attribute__((visibility("default")))
#else
#define SFRT_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define SFRT_OK 0
#define SFRT_E_INVALID -1      /* bad argument (null, size <= 0, non-finite value, radius <= 0) */
#define SFRT_E_EMPTY -2        /* no spheres: the reference throws std::out_of_range (SphereWorld.cpp:373) */
#define SFRT_E_NO_TEXTURE -3   /* textures[0] not loaded (SphereWorld.cpp:52) */
#define SFRT_E_TOO_MANY -4     /* more than SFRT_MAX_SPHERES spheres */
#define SFRT_E_HIP -5          /* HIP runtime error (no device, launch or copy failure) */
#define SFRT_E_MARCH_LIMIT -6  /* a ray exceeded SFRT_MAX_ITERATIONS march steps */
#define SFRT_E_TEXEL -7        /* a texel index fell outside the texture (reference: out-of-bounds read) */

#define SFRT_MAX_SPHERES 1024
#define SFRT_MAX_ITERATIONS (1 << 20)
#define SFRT_TEXTURE_SLOTS 10  /* sf::Image* textures = new sf::Image[10] (SphereWorld.h:74) */

/* sf::Vector3f pos + float radius of struct Sphere (SphereWorld.h:23-29). */
typedef struct {
  float x, y, z, radius;
} sfrt_sphere;

/* The fields of struct Camera (SphereWorld.h:10-21) that the frame fill reads.
 * fov_h / fov_v are in radians, i.e. after `cam.fovH *= PI / 180.0f`
 * (SphereWorld.cpp:72-73); sfrt_deg_to_rad reproduces that conversion. */
typedef struct {
  float pos[3];
  float rotation;
  float hrotation;
  float fov_h;
  float fov_v;
} sfrt_camera;

/* Float intermediates of one pixel (parity/debug): final march position,
 * drawSphere, march iterations, xcoord/ycoord/brightness of
 * SphereWorld.cpp:373-375, texel coordinates and the RGBA8 result. */
typedef struct {
  float pos[3];
  int32_t draw;
  int32_t iters;
  float xcoord, ycoord, brightness;
  uint32_t texel[2];
  uint32_t rgba;
} sfrt_pixel_dump;

typedef struct sfrt_world sfrt_world;

/* ---- world lifetime (SphereWorld::SphereWorld / ~SphereWorld, SphereWorld.cpp:43-81) ----
 * A new world has width 320, height 180, camera at the origin with
 * fov 75/47 degrees converted to radians, no spheres and no textures. */
SFRT_API int sfrt_world_create(int hip_device, sfrt_world** out);
SFRT_API void sfrt_world_destroy(sfrt_world* w);

/* ---- scene state ---- */
SFRT_API int sfrt_world_set_size(sfrt_world* w, int width, int height);          /* SphereWorld::width/height */
SFRT_API int sfrt_world_get_size(const sfrt_world* w, int* width, int* height);
SFRT_API int sfrt_world_set_camera(sfrt_world* w, const sfrt_camera* cam);       /* SphereWorld::cam */
SFRT_API int sfrt_world_get_camera(const sfrt_world* w, sfrt_camera* cam);
/* textures[slot].loadFromFile(...) (SphereWorld.cpp:52): RGBA8 rows, w*h*4 bytes. Slot 0 is sampled. */
SFRT_API int sfrt_world_load_texture(sfrt_world* w, int slot, const uint8_t* rgba, int tex_w, int tex_h);
/* AddSphere (SphereWorld.cpp:177-190): append, drop contained spheres, re-sort. */
SFRT_API int sfrt_world_add_sphere(sfrt_world* w, float x, float y, float z, float radius);
/* Replace the sphere list verbatim (caller order = the order the march visits). */
SFRT_API int sfrt_world_set_spheres(sfrt_world* w, const sfrt_sphere* spheres, int count);
SFRT_API int sfrt_world_get_spheres(const sfrt_world* w, sfrt_sphere* out, int capacity, int* count);
/* UpdateSpheres sort part (SphereWorld.cpp:199-212): stable by |c - cam.pos| + r. */
SFRT_API int sfrt_world_update_spheres(sfrt_world* w);

/* ---- the frame fill ----
 * SphereWorld::UpdateImage(v, ystart, yadd, xstart, xadd): renders pixels
 * {i = xstart + k*xadd < width} x {j = ystart + l*yadd < height} into the
 * caller's host buffer `pixels` (width*height*4 bytes, RGBA8 row-major,
 * pitch 4*width) and writes no other byte.  Returns when the bytes are in
 * `pixels`. */
SFRT_API int sfrt_world_update_image(sfrt_world* w, uint8_t* pixels, int ystart, int yadd, int xstart,
                            int xadd);

/* Device-resident frame fill for the display / multi-GPU path: rows
 * [row0, row0 + rows) of the width x height frame into `dev_pixels` (device
 * memory on this world's device; row r of the band at dev_pixels +
 * (r - row0) * pitch_bytes).  Rays use the GLOBAL row index, so row bands
 * rendered on different GPUs tile the single-GPU frame byte for byte.
 * Asynchronous on `hip_stream` (a hipStream_t; NULL = the HIP null stream);
 * call sfrt_world_check(w, hip_stream) to synchronise and read the
 * march-limit / texel status of the launches since the last check. */
SFRT_API int sfrt_world_render_band(sfrt_world* w, void* dev_pixels, int64_t pitch_bytes, int row0,
                           int rows, void* hip_stream);
SFRT_API int sfrt_world_check(sfrt_world* w, void* hip_stream);

/* Pipelined frame fill for the display path: renders the
 * whole width x height frame of the world's current state into `pixels`
 * (width*height*4 bytes) without blocking, then copies it back while the
 * caller submits the next frame (two frames in flight).  `pixels` should come
 * from sfrt_host_alloc (pinned: the copy overlaps compute and runs at PCIe
 * rate); it must stay valid until sfrt_world_wait_frame(ticket) returns, and
 * then holds the same bytes sfrt_world_update_image(w, pixels, 0, 1, 0, 1)
 * would have written.  The scene/camera are snapshotted at submit time. */
SFRT_API int sfrt_world_submit_frame(sfrt_world* w, uint8_t* pixels, int64_t* ticket);
SFRT_API int sfrt_world_wait_frame(sfrt_world* w, int64_t ticket);
SFRT_API int sfrt_host_alloc(void** ptr, int64_t bytes);
SFRT_API int sfrt_host_free(void* ptr);

/* Float intermediates for `count` pixels (ij = i0, j0, i1, j1, ...), synchronous. */
SFRT_API int sfrt_world_trace_points(sfrt_world* w, const int32_t* ij, int count, sfrt_pixel_dump* out);

/* Options: SFRT_OPT_CULL (1 = per-wave sphere culling, default; 0 = visit
 * every sphere -- same bytes, slower; used by A/B parity tests).
 * SFRT_OPT_VARIANT: kernel tuning variant for A/B timing (0 = default build;
 * every variant produces the same bytes). */
#define SFRT_OPT_CULL 1
#define SFRT_OPT_VARIANT 2
SFRT_API int sfrt_world_set_option(sfrt_world* w, int option, int value);

/* ---- stateless helpers ---- */
/* UpdateSpheres ordering of an array in place (SphereWorld.cpp:199-212). */
SFRT_API int sfrt_sort_spheres(sfrt_sphere* spheres, int count, const float cam_pos[3]);
/* deg * (PI / 180.0f) in binary32 (SphereWorld.cpp:72-73). */
SFRT_API float sfrt_deg_to_rad(float deg);
/* Exact pass threshold: for every binary32 s >= 0,
 * (radius - sqrtf(s) > 0.01f)  <=>  (s < sfrt_pass_threshold(radius)). */
SFRT_API float sfrt_pass_threshold(float radius);
SFRT_API const char* sfrt_error_string(int code);
SFRT_API int sfrt_version(void);

#ifdef __cplusplus
}
#endif
#endif /* SFRT_H */
