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
/* textures[slot].loadFromFile(...) (SphereWorld.cpp:52): RGBA8 rows, w*h*4 bytes. Slot 0 is sampled.
   Stream-ordered, no device-wide wait: frames queued before the call read the old texels, frames
   queued after it (on any stream) the new ones. */
SFRT_API int sfrt_world_load_texture(sfrt_world* w, int slot, const uint8_t* rgba, int tex_w, int tex_h);
/* AddSphere (SphereWorld.cpp:177-190): append, drop contained spheres, re-sort. */
SFRT_API int sfrt_world_add_sphere(sfrt_world* w, float x, float y, float z, float radius);
/* Replace the sphere list verbatim (caller order = the order the march visits). */
SFRT_API int sfrt_world_set_spheres(sfrt_world* w, const sfrt_sphere* spheres, int count);
SFRT_API int sfrt_world_get_spheres(const sfrt_world* w, sfrt_sphere* out, int capacity, int* count);
/* Extension ("all textures"): a texture slot per sphere, in the
 * current sphere order (count == number of spheres); slots travel with their spheres
 * through AddSphere / UpdateSpheres.  Default 0 = textures[0] everywhere = the
 * reference (SphereWorld.cpp:376-377 samples textures[0] only). */
SFRT_API int sfrt_world_set_sphere_textures(sfrt_world* w, const int32_t* slots, int count);
SFRT_API int sfrt_world_get_sphere_textures(sfrt_world* w, int32_t* out, int capacity, int* count);
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
/* Estimated work per pixel row of the world's last frame fill that ran in the adaptive
 * tile order (sfrt_world_render_band, sfrt_world_submit_frame; SFRT_OPT_TILE_ORDER on):
 * *row0, *rows = the global rows it covered, costs[i] (i < *rows <= capacity) = the
 * ray-steps of row *row0 + i, from the per-tile march-step classes that launch recorded
 * (each pixel costs its tile's class steps plus ~4 for shading).  For cost-weighted row
 * bands (sfrt_multi_cost_bands).  Synchronises with that fill; SFRT_E_INVALID if no
 * such fill exists (or capacity is short). */
SFRT_API int sfrt_world_row_costs(sfrt_world* w, float* costs, int capacity, int* row0, int* rows);

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
/* hipHostFree underneath: it returns only once the whole device is idle (profiles/r6u_hip_alloc_calls.txt),
   so free pinned frames at shutdown or between bursts, not between frames. */
SFRT_API int sfrt_host_free(void* ptr);

/* Float intermediates for `count` pixels (ij = i0, j0, i1, j1, ...), synchronous: the
 * march position, drawSphere and loop trips of SphereWorld.cpp:362-372, xcoord, ycoord,
 * brightness and the texel of :373-377, and the RGBA8 pixel, read out of the frame-fill
 * kernel itself (its DUMP instantiation renders the whole frame with the world's options:
 * tile shape, culling, and -- SFRT_OPT_TILE_ORDER on -- three launches in the adaptive
 * order).  A pixel may be listed more than once. */
SFRT_API int sfrt_world_trace_points(sfrt_world* w, const int32_t* ij, int count, sfrt_pixel_dump* out);

/* Options: SFRT_OPT_CULL (1 = per-wave sphere culling, default; 0 = visit
 * every sphere -- same bytes, slower; used by A/B parity tests).
 * SFRT_OPT_RAYS_PER_LANE (0 = default): pixels per lane R of the frame-fill
 * kernel, i.e. its (8R)x8 tile width; 1-4 force that shape (parity tests run
 * every shipped tile shape; same bytes), 0 lets the kernel table choose
 * (sphere_trace.hip trace_rays).
 * SFRT_OPT_TILE_ORDER (1 = default): sfrt_world_render_band dispatches the tiles
 * of a frame longest-first by the march steps an earlier render_band of the same
 * geometry recorded (two frames back; the sort runs inside the next launch);
 * 0 = row-major order.  Scheduling only: same bytes either way. */
#define SFRT_OPT_CULL 1
#define SFRT_OPT_RAYS_PER_LANE 2
#define SFRT_OPT_TILE_ORDER 3
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
/* "release" for the shipped build; "diagnostic" for a -DSFRT_EXP timing/counter build
 * (writes wrong bytes by design) and "ab" for a build with extra flags (build-flag A/B).
 * bench.py refuses anything but "release". */
SFRT_API const char* sfrt_build_flavour(void);

/* ======================================================================
 * Band transfer packing (the exchange step of SURVEY 8e).  A frame
 * pixel's alpha is its texel's (SphereWorld.cpp:376-381, :109), and the
 * reference's textures hold alpha 0 or 255 only, so a band whose alphas are all
 * 0 or 255 packs losslessly into RGB plus one alpha bit: 3.125 bytes per pixel
 * on the wire instead of 4.  Format: B = ceil(pixels / 256), B * 800 bytes in two
 * planes: [0, 768*B) the RGB plane, pixel p's R, G, B at bytes 3p..3p+2 (zero past
 * the last pixel), then [768*B, 800*B) the alpha plane, the little-endian bit string
 * whose bit p is set when pixel p's alpha is 255 (zero past the last pixel).
 * Asynchronous on `hip_stream` of the device
 * current to the calling thread, which holds both buffers; dev_rgba 4-byte
 * and dev_packed 8-byte aligned.  Pixels whose alpha is neither 0 nor 255
 * unpack with alpha 0 -- pack only bands of a world whose
 * sfrt_world_alpha_binary is 1.
 * ====================================================================== */
SFRT_API int64_t sfrt_band_packed_bytes(int64_t pixels);  /* < 0: invalid */
SFRT_API int sfrt_band_pack(const void* dev_rgba, int64_t pixels, void* dev_packed, void* hip_stream);
SFRT_API int sfrt_band_unpack(const void* dev_packed, int64_t pixels, void* dev_rgba, void* hip_stream);
/* 1 when at least one texture is loaded and every texel of every loaded texture has
 * alpha 0 or 255 (so every pixel the world renders does), else 0. */
SFRT_API int sfrt_world_alpha_binary(const sfrt_world* w, int* binary);

/* ======================================================================
 * One frame over several GPUs of this node (BASELINE configs 4-5):
 * the reference caller is ONE C++ process (Source.cpp:17-28,47-52) that fills
 * one sf::Image; here it fills it on n GPUs.  The frame is split into
 * contiguous row bands, rank r = devices[r] renders rows [row0_r, row0_r +
 * rows_r) with the global row index (so the gathered frame is byte-identical
 * to a one-GPU render), and the bands travel to devices[0]:
 *   SFRT_MULTI_RCCL -- RCCL (librccl, loaded at create): one ncclGather for
 *                      equal bands, grouped ncclSend/ncclRecv otherwise;
 *   SFRT_MULTI_PEER -- hipMemcpyPeerAsync over xGMI (also serves a device
 *                      listed twice, which RCCL refuses);
 *   SFRT_MULTI_AUTO -- RCCL when the devices are distinct, else PEER.
 * Band transfers run on per-rank copy streams, so frame k's transfer overlaps
 * frame k+1's render (two band buffers per rank).  The scene setters below
 * apply to every rank's world; sfrt_multi_world gives a rank's world for
 * anything else (options).
 * ====================================================================== */
typedef struct sfrt_multi sfrt_multi;

#define SFRT_MULTI_AUTO 0
#define SFRT_MULTI_RCCL 1
#define SFRT_MULTI_PEER 2

SFRT_API int sfrt_multi_create(const int* hip_devices, int n, int transport, sfrt_multi** out);
/* The library behind SFRT_MULTI_RCCL: "" until the process's first RCCL context, then
 * "librccl.so.1" (or "librccl.so"), or "test:<path>" for a test transport; " (not loaded)"
 * is appended when it did not resolve.  SFRT_E_INVALID if it does not fit in `size`. */
SFRT_API int sfrt_multi_transport_library(char* buf, int size);
/* TEST ONLY: the RCCL C API from `library_path` instead of librccl (the tests' loopback
 * transport, tests/native/rccl_loopback.cpp, which accepts a device listed twice, so the
 * RCCL branch runs with n > 1 on one GPU).  Only before the process's first RCCL context
 * (else SFRT_E_INVALID); nothing in the environment selects it; reported by
 * sfrt_multi_transport_library. */
SFRT_API int sfrt_multi_use_test_transport(const char* library_path);
SFRT_API void sfrt_multi_destroy(sfrt_multi* m);
SFRT_API int sfrt_multi_count(const sfrt_multi* m, int* n, int* transport);
SFRT_API int sfrt_multi_world(sfrt_multi* m, int rank, sfrt_world** out);
SFRT_API int sfrt_multi_set_size(sfrt_multi* m, int width, int height);
SFRT_API int sfrt_multi_set_camera(sfrt_multi* m, const sfrt_camera* cam);
SFRT_API int sfrt_multi_load_texture(sfrt_multi* m, int slot, const uint8_t* rgba, int tex_w, int tex_h);
SFRT_API int sfrt_multi_set_spheres(sfrt_multi* m, const sfrt_sphere* spheres, int count);
SFRT_API int sfrt_multi_add_sphere(sfrt_multi* m, float x, float y, float z, float radius);
SFRT_API int sfrt_multi_update_spheres(sfrt_multi* m);
SFRT_API int sfrt_multi_set_sphere_textures(sfrt_multi* m, const int32_t* slots, int count);
SFRT_API int sfrt_multi_set_option(sfrt_multi* m, int option, int value);
/* Transfer format of the bands that cross a link (see "Band transfer packing"):
 * SFRT_TRANSFER_AUTO (default) packs when every rank's world is alpha-binary
 * (sfrt_world_alpha_binary), SFRT_TRANSFER_RGBA never packs, SFRT_TRANSFER_PACKED
 * always does (sfrt_multi_render fails with SFRT_E_INVALID on a world that is not
 * alpha-binary).  Packed bands travel by point-to-point transfers (RCCL) or peer
 * copies and are unpacked into the frame on devices[0]; the frame's bytes are the
 * same either way.  sfrt_multi_get_transfer: the setting and whether the last
 * render packed. */
#define SFRT_TRANSFER_AUTO 0
#define SFRT_TRANSFER_RGBA 1
#define SFRT_TRANSFER_PACKED 2
SFRT_API int sfrt_multi_set_transfer(sfrt_multi* m, int format);
SFRT_API int sfrt_multi_get_transfer(sfrt_multi* m, int* format, int* last_packed);
/* Band heights: rows[r] for rank r (rank 0 first, sum = height at render time);
 * rows == NULL restores the default equal split (sfrt_multi_bands, factor 1). */
SFRT_API int sfrt_multi_set_bands(sfrt_multi* m, const int* rows, int n);
/* The partition helper (stateless, no device): row0/rows of n ranks for a frame
 * of `height` rows where rank 0 -- whose band never crosses a link -- gets about
 * `root_factor` times the rows of every other rank (their bands equal and
 * multiples of the 8-row tile); root_factor 1 = equal split
 * [r*H/n, (r+1)*H/n). */
SFRT_API int sfrt_multi_bands(int height, int n, float root_factor, int* row0, int* rows);
/* Cost-weighted partition (SURVEY 8e "Balance"; stateless, no device): rank 0 gets
 * `root_factor` shares of the frame's march cost sum(row_cost[0..height)), every
 * other rank one share; band edges on 8-row tile boundaries (or the last row).
 * row_cost: per-row work, e.g. from sfrt_world_row_costs / sfrt_multi_row_costs.
 * Invalid or all-zero costs give sfrt_multi_bands' partition. */
SFRT_API int sfrt_multi_cost_bands(const float* row_cost, int height, int n, float root_factor,
                                   int* row0, int* rows);
/* Per-row march cost of the whole frame from every rank's last band render
 * (sfrt_world_row_costs of each rank's world; costs[height]).  Synchronises. */
SFRT_API int sfrt_multi_row_costs(sfrt_multi* m, float* costs, int height);
/* Re-partition from the last frame's row costs: sfrt_multi_row_costs +
 * sfrt_multi_cost_bands + sfrt_multi_set_bands.  Call after a frame was rendered. */
SFRT_API int sfrt_multi_balance(sfrt_multi* m, float root_factor);
/* Render the whole width x height frame into `dev_frame` (device memory on
 * devices[0], pitch exactly width*4), asynchronously: every rank starts after
 * the work already queued on `hip_stream` (a stream of devices[0]; NULL = null
 * stream), and the frame is complete when `hip_stream` reaches the point after
 * this call.  sfrt_multi_check synchronises and reads every rank's status. */
SFRT_API int sfrt_multi_render(sfrt_multi* m, void* dev_frame, int64_t pitch_bytes, void* hip_stream);
SFRT_API int sfrt_multi_check(sfrt_multi* m);
/* UpdateImage(v, 0, 1, 0, 1) on n GPUs: the whole frame into the caller's host
 * RGBA8 buffer (width*height*4 bytes, pitch 4*width).  Synchronous. */
SFRT_API int sfrt_multi_update_image(sfrt_multi* m, uint8_t* pixels);

/* ======================================================================
 * Voxel World frame fill: drop-in for
 *   void World::UpdateImage(sf::Image* v, short ystart, short yadd,
 *                           short xstart, short xadd)
 *   (/root/reference/Raytracing/World.h:60, World.cpp:62-87; Raycast and
 *   LRaycast World.cpp:302-491) over a snapshot of the World state.
 * ====================================================================== */

/* struct Dynamic (World.h:25-38): the fields Raycast reads. */
typedef struct {
  float pos[3];
  float size[2];
  float r, g, b;
  float dist_to_camera;
  int32_t texture_id; /* dynTextures slot */
} sfrt_dynamic;

/* struct Light (World.h:40-47). */
typedef struct {
  float pos[3];
  float intensity, r, g, b;
  int32_t shadows;
} sfrt_light;

typedef struct sfrt_voxel sfrt_voxel;

#define SFRT_VOXEL_EMPTY (-32768)

/* A new voxel world: 320x180, Camera defaults of World.h:9-19 (pos 15.5, 1.9,
 * 15.5; fov 75/47 degrees converted like World.cpp:55-56), shadowDistance 16,
 * viewDistance 24 (World.h:70-71), no blocks/textures/objects/lights. */
SFRT_API int sfrt_voxel_create(int hip_device, sfrt_voxel** out);
SFRT_API void sfrt_voxel_destroy(sfrt_voxel* v);
SFRT_API int sfrt_voxel_set_size(sfrt_voxel* v, int width, int height);
SFRT_API int sfrt_voxel_set_camera(sfrt_voxel* v, const sfrt_camera* cam);
SFRT_API int sfrt_voxel_set_view(sfrt_voxel* v, float shadow_distance, float view_distance);
/* `blocks` (World.h:75) as a dense grid: texture_ids[(x*ny + y)*nz + z] is
 * Block::textureID (>= 0: textures[id]; < 0: colors[-id]) or SFRT_VOXEL_EMPTY;
 * lookups keep the map's (x<<20)+(y<<10)+z key semantics.  1 <= nx <= 2048, 1 <= ny, nz
 * <= 1024; the device copy is the key space itself, nx MiB of bytes (100 MiB for a
 * 100-wide world; 2 GiB for nx = 2048 whatever ny and nz are), rewritten by the first
 * frame after each call, stream-ordered on that frame's stream (no device-wide sync: it
 * waits on the device for the launches that read the old grid).  The call itself touches
 * no device memory: a grid the device cannot allocate fails that first frame call with
 * SFRT_E_HIP. */
SFRT_API int sfrt_voxel_set_blocks(sfrt_voxel* v, const int16_t* texture_ids, int nx, int ny, int nz);
SFRT_API int sfrt_voxel_load_texture(sfrt_voxel* v, int slot, const uint8_t* rgba, int w, int h);
SFRT_API int sfrt_voxel_load_dyn_texture(sfrt_voxel* v, int slot, const uint8_t* rgba, int w, int h);
SFRT_API int sfrt_voxel_set_colors(sfrt_voxel* v, const uint8_t* rgba, int count); /* colors[] */
/* `dyn` in list order (World.h:93) and `alights` in list order (World.h:95). */
SFRT_API int sfrt_voxel_set_dynamics(sfrt_voxel* v, const sfrt_dynamic* dyn, int count);
SFRT_API int sfrt_voxel_set_lights(sfrt_voxel* v, const sfrt_light* lights, int count);
/* The smallest squared distance dd >= 0 at which a light of this intensity adds nothing,
 * `intensity / dd - dd * 0.002f <= 0` in binary32 (World.cpp:425-426); 0 when no dd passes.
 * The kernel skips a light for a wave none of whose hit points is that close. */
SFRT_API float sfrt_voxel_light_dd_pass(float intensity);
/* World::UpdateImage into the caller's host RGBA8 frame; only addressed pixels written. */
SFRT_API int sfrt_voxel_update_image(sfrt_voxel* v, uint8_t* pixels, int ystart, int yadd, int xstart,
                                     int xadd);
/* Device row band [row0, row0+rows), asynchronous on hip_stream (NULL = null stream). */
SFRT_API int sfrt_voxel_render_band(sfrt_voxel* v, void* dev_pixels, int64_t pitch_bytes, int row0,
                                    int rows, void* hip_stream);
SFRT_API int sfrt_voxel_check(sfrt_voxel* v, void* hip_stream);
/* SFRT_OPT_TILE_ORDER as for sfrt_world, but off (0) by default here: render_band with 1
 * dispatches 8x8 tiles longest-first by the DDA + shadow steps of two frames back (same
 * bytes; measured 1-6% slower on the voxel worlds). */
SFRT_API int sfrt_voxel_set_option(sfrt_voxel* v, int option, int value);

/* ======================================================================
 * GLSL renderer: drop-in for the live GPU path
 *   world.shader.setUniform(...)                (SphereWorld.cpp:214-238,
 *                                                Source.cpp:143-146)
 *   rt.draw(sp, &world.shader)                  (Source.cpp:150-153)
 * i.e. rayShader.frag (/root/reference/Raytracing/rayShader.frag:1-179) run
 * once per pixel of a width x height render target.  Semantics the shader
 * leaves to the driver are fixed in DESIGN.md section 4b.
 * ====================================================================== */

#define SFRT_GLSL_MAX_SPHERES 100 /* uniform vec4 spheres[100] (rayShader.frag:6-8) */

/* The shader's uniforms (rayShader.frag:1-11); `ground` is set separately. */
typedef struct {
  float campos[3];
  float rotation[2]; /* (cam.rotation, cam.hrotation) */
  float fov[2];      /* (fovH, fovV) in radians */
  float size[2];     /* render-target size */
  int32_t sphere_count, all_spheres_count, light_count;
  float spheres[SFRT_GLSL_MAX_SPHERES][4]; /* xyz, radius: walls, lights, ospheres */
  float uvs[SFRT_GLSL_MAX_SPHERES][4];
  float lights[SFRT_GLSL_MAX_SPHERES][4];
} sfrt_glsl_uniforms;

typedef struct sfrt_glsl sfrt_glsl;

/* A new shader instance: all uniforms zero (GLSL's initial uniform values),
 * no ground texture. */
SFRT_API int sfrt_glsl_create(int hip_device, sfrt_glsl** out);
SFRT_API void sfrt_glsl_destroy(sfrt_glsl* g);
/* setUniform("ground", t) with t.setRepeated(true), t.generateMipmap()
 * (SphereWorld.cpp:52-57): RGBA8 rows, power-of-two sides. */
SFRT_API int sfrt_glsl_set_ground(sfrt_glsl* g, const uint8_t* rgba, int w, int h);
SFRT_API int sfrt_glsl_set_uniforms(sfrt_glsl* g, const sfrt_glsl_uniforms* u);
SFRT_API int sfrt_glsl_get_uniforms(sfrt_glsl* g, sfrt_glsl_uniforms* u);
/* sf::Shader::setUniform by name: "campos" (3 floats), "rotation", "fov",
 * "size" (2), "spheres[k]", "uvs[k]", "lights[k]" (4); ints "sphereCount",
 * "allSpheresCount", "lightCount".  Unknown names -> SFRT_E_INVALID. */
SFRT_API int sfrt_glsl_set_uniform(sfrt_glsl* g, const char* name, const float* v, int n);
SFRT_API int sfrt_glsl_set_uniform_int(sfrt_glsl* g, const char* name, int value);
/* rt.draw: rows [row0, row0+rows) of a width x height target into device
 * memory (row 0 = top of the image, as rt.getTexture().copyToImage()),
 * asynchronous on hip_stream (NULL = null stream). */
SFRT_API int sfrt_glsl_draw(sfrt_glsl* g, void* dev_pixels, int width, int height,
                            int64_t pitch_bytes, int row0, int rows, void* hip_stream);
/* rt.draw + rt.getTexture().copyToImage() into a host RGBA8 buffer (synchronous). */
SFRT_API int sfrt_glsl_draw_image(sfrt_glsl* g, uint8_t* pixels, int width, int height);
SFRT_API int sfrt_glsl_check(sfrt_glsl* g, void* hip_stream);
/* SFRT_OPT_TILE_ORDER as for sfrt_world, on (1) by default: sfrt_glsl_draw dispatches 8x8
 * tiles longest-first by the metaball-march steps of two frames back (same bytes; 1-6 % faster
 * on the round-4 kernel); 0 = row-major.  sfrt_glsl_draw_image is row-major. */
SFRT_API int sfrt_glsl_set_option(sfrt_glsl* g, int option, int value);

/* ======================================================================
 * Asset pipeline: PNG -> RGBA8 as sf::Image::loadFromFile
 * (SFML 2.4.2 / stb_image, 4 channels) decodes the reference's textures
 * (SphereWorld.cpp:52-53, World.cpp:40-45).  Host-only; no device needed.
 * ====================================================================== */
SFRT_API int sfrt_png_info(const uint8_t* data, int64_t len, int* width, int* height);
/* rgba: capacity bytes >= width*height*4 (query with sfrt_png_info). */
SFRT_API int sfrt_png_decode(const uint8_t* data, int64_t len, uint8_t* rgba, int64_t capacity,
                             int* width, int* height);

#ifdef __cplusplus
}
#endif
#endif /* SFRT_H */
