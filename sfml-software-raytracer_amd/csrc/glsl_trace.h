// glsl_trace.h -- launch record shared by the GLSL-mode host mirror
// (sfrt_glsl.cpp) and its gfx950 kernel (glsl_trace.hip).  SURVEY 8f row f1.
//
// rayShader.frag (/root/reference/Raytracing/rayShader.frag) recomputes per
// fragment several terms that depend only on the uniforms; the host evaluates
// them once per draw with the same expressions:
//  * the camera basis of main() (:165-169, sin/cos) and fov.x / size.x * 2;
//  * per wall sphere the exact squared-length bound of the containment test
//    `step(length(rpos), r)` (:74), so the wall pass needs no sqrt to decide;
//  * per (light, shadow ball) pair distance(light, ball), atan(r, distance)
//    and the unit light->ball direction (:140-142).
#pragma once

#include <stdint.h>

namespace sfrt {

constexpr int kGlslMax = 100;          // uniform vec4 spheres[100] (rayShader.frag:6-8)
constexpr int kGlslMipLevels = 16;
constexpr int kGlslMarchCap = 1 << 20; // the shader has no cap; the status reports hitting it

struct GlslWall {                      // spheres[0 .. sphereCount)
  float x, y, z, r;
  float rr;                            // r*r (:77)
  float s_in;                          // step(sqrt(s), r) == 1  <=>  s <= s_in
  float pad0, pad1;
};

struct GlslBall {                      // spheres[sphereCount .. allSpheresCount)
  float x, y, z, r;
  float r_skip;                        // RU(r * (1+6e-6)) when r >= 0 (the march's dominance test), else NaN
  float pad0, pad1, pad2;
};

struct GlslPair {                      // light i, shadow ball j (:140-142)
  float dist;                          // distance(spheres[i], spheres[j])
  float sanglet;                       // atan(spheres[j].w, dist)
  float ux, uy, uz;                    // (spheres[j] - spheres[i]) / dist
  float bx, by, bz;                    // spheres[j].xyz
  float cos_lit;                       // dot(-tolightnorm, u) <= cos_lit => factor 1 (or -2)
};

struct GlslMat {                       // per uniform index: uvs[k], lights[k], spheres[k].xyz
  float uv[4];
  float light[4];
  float cx, cy, cz, pad;
};

struct GlslFrame {
  float campos[3];
  float fwd[3], right[3], up[3];
  float fov_x, fov_y, hk, vk;          // hk = fov.x / size.x * 2 (:172), vk likewise
  int32_t sc, lc, all;
  int32_t cam_negzero;                 // a campos component is -0.0 (wall pass, below)
  int32_t wall_start;                  // first wall-pass iteration that can change a lane
  // The per-wave wall cull's distance margin (glsl_trace.hip wall_mask): 1e-3 of the largest
  // coordinate the wall pass can reach, + 1e-4; 0 disables the cull (a -0.0 in campos, more than
  // 64 walls, non-finite bounds)
  float wall_cull_margin;
  int32_t width, height, row0, rows, tiles_x;
  const GlslWall* walls;
  const GlslBall* balls;               // all - sc entries (lights, then ospheres)
  const GlslPair* pairs;               // [light][shadow ball], lc x (all - sc - lc)
  const GlslMat* mats;                 // kGlslMax entries
  const uint32_t* mip;                 // RGBA8 levels back to back
  int32_t mip_levels;
  int32_t mip_w[kGlslMipLevels], mip_h[kGlslMipLevels], mip_off[kGlslMipLevels];
  long long out_pitch;                 // in pixels
  uint32_t* out;
  int* status;                         // bit 0: march cap reached
  // Adaptive tile order (sfrt_sched.h): 8x8 tiles, one per one-wave
  // workgroup, slot -> tile_order; cost = the tile's longest metaball march.
  const uint32_t* tile_order;
  uint8_t* tile_cost;
  const uint8_t* prev_cost;
  uint32_t* next_order;
  // tile_order's classes are the ones in tile_cost: store only changed classes (sfrt_device.h
  // store_cost, sfrt_sched.h TileSchedPtrs::cost_diff)
  int32_t cost_diff;
};

// Tile grid of the ordered GLSL kernel for f: key (> 0) and tile count.
long long glsl_tile_key(const GlslFrame& f, long long* tiles);
// done_event (hipEvent_t, may be null): recorded by the launch's own completion (its stop event).
int launch_glsl(const GlslFrame& f, void* stream, void* done_event = nullptr);

}  // namespace sfrt
