// sfrt_trace.h -- per-frame launch record shared by the host mirror
// (sfrt_world.cpp) and the gfx950 kernels (sphere_trace.hip).
//
// Everything that the reference recomputes per pixel but is uniform over the
// frame is computed once on the host with the reference's own expressions
// (camera basis SphereWorld.cpp:100-104, ray-angle steps :85-89, the first
// march iteration from cam.pos, per-sphere atan2f(c.z, c.x) of :326) and
// shipped here, so the kernel only does per-pixel work.
#pragma once

#include <stdint.h>

namespace sfrt {

constexpr int kInlineSpheres = 64;    // spheres carried in the kernel-argument segment
constexpr int kMaxSpheres = 1024;     // 16 culling words of 64 spheres, compacted per wave
constexpr int kTile = 8;              // tile rows; a wave's tile is (8R) x 8 pixels
constexpr int kMaxIterations = 1 << 20;  // march guard; the reference has none
// Per-wave culling is proven safe while every lane of the wave has made at
// most this many march steps (the accumulated binary32 error of the march
// positions stays below the culling margin, see cull_margin); a wave that
// goes further switches to the full sphere list for the rest of its march.
constexpr int kCullSafeIterations = 1024;
constexpr int kPairMinSpheres = 16;  // above this, n <= 64 frames use 16x8 tiles (2 px per lane)
#ifndef SFRT_SLOTS
#define SFRT_SLOTS 2
#endif
constexpr int kSlots = SFRT_SLOTS;  // culled spheres held in SGPRs per wave (2: best of 0-4, 6; profiles/ab/r2_ab32)

// One sphere as the kernel reads it: 32 B, one s_load_dwordx8.
struct SphereRec {
  float cx, cy, cz, r;
  float s_pass;    // exact pass threshold: r - sqrtf(s) > 0.01f  <=>  s < s_pass
  float atan_c;    // atan2f(cz, cx), the centre term of VAngleXZ (SphereWorld.cpp:326)
  uint32_t tex_off;  // this sphere's texture (textures[0], or its extension slot) in the atlas
  uint32_t tex_wh;   // its width | height << 16
};

struct FrameRec {
  float cam[3];
  float fwd[3], right[3], up[3];   // basis after VRotateX/VRotateY (SphereWorld.cpp:100-104)
  float h_start, h_inc, v_start, v_inc;  // SphereWorld.cpp:85-89
  float first_l;                    // largestDist of the first march iteration (pos == cam)
  int first_draw;                   // drawSphere after the first iteration
  int n;                            // sphere count
  int width, height;                // global frame (bounds for the subset walk)
  int xstart, xadd, ystart, yadd;   // UpdateImage pixel subset (SphereWorld.cpp:94,97)
  int sub_w;                        // columns in the subset
  int sub_row0, sub_rows;           // subset rows rendered by this launch
  int tiles_x;                      // ceil(sub_w / 8)
  int cull;                         // 1: per-wave cone culling (default), 0: every sphere
  float cull_margin;                // absolute inflation of every sphere in the cone test
  int rays;                         // SFRT_OPT_RAYS_PER_LANE: 0 = the kernel table's choice, 1-4 forced
  long long out_pitch;              // output pitch in pixels
  uint32_t* out;                    // pixel (a, b) -> out[(b - sub_row0) * out_pitch + a]
  const uint32_t* tex;              // RGBA8 texture atlas (every loaded slot, back to back)
  const SphereRec* spheres;         // device copy (used when n > kInlineSpheres)
  int* status;                      // device word: bit 0 = march guard hit, bit 1 = bad texel
  // Adaptive tile order ("Tile order"), one-wave-per-workgroup
  // kernels only; all null = row-major order, nothing recorded.  Launch k of a
  // chain (stream-ordered launches with one tile grid) dispatches tile slot s on
  // tile tile_order[s] (longest tiles of launch k-2 first) and records each
  // tile's march-step class (tile_bucket) in tile_cost.  With prev_cost set the
  // grid has one extra workgroup, 0, dispatched first: it sorts launch k-1's
  // classes into next_order for launch k+1 (stable counting sort in its LDS, no
  // atomics) and renders nothing; tile slot s is then workgroup s + 1.
  const uint32_t* tile_order;
  uint8_t* tile_cost;
  const uint8_t* prev_cost;
  uint32_t* next_order;
  // The camera moved since the launch whose classes the sorter ranks: rank each
  // tile by the longest of it and its row neighbours (sfrt_device.h sort_tiles).
  int order_dilate;
  // tile_order's classes are the ones in tile_cost: store only changed classes (sfrt_device.h
  // store_cost, sfrt_sched.h TileSchedPtrs::cost_diff)
  int32_t cost_diff;
};

// Kernel argument for n <= kInlineSpheres: frame + spheres in the kernarg segment.
struct InlineArgs {
  FrameRec f;
  SphereRec s[kInlineSpheres];
};

struct PixelDump {
  float pos[3];
  int draw;
  int iters;  // loop trips of SphereWorld.cpp:362 (the host's first one included)
  float xcoord, ycoord, brightness;
  uint32_t texel[2];
  uint32_t rgba;
};

// Float intermediates out of the frame-fill kernels themselves (sfrt_world_trace_points):
// the DUMP instantiation of the same march and shading, plus an epilogue that writes
// pixel (a, b)'s record to out[q] when pix[q] == (b - sub_row0) * sub_w + a (binary search
// of the sorted, distinct listed pixels: O(listed pixels) memory whatever the frame size).
// The DUMP kernels store no frame pixel (each record carries its rgba).
struct DumpArgs {
  const int64_t* pix;  // ascending, distinct
  int npix;
  PixelDump* out;      // npix records
};

// sphere_trace.hip.  dump != nullptr: the DUMP instantiation of the kernel the table picks.
// done_event (hipEvent_t, may be null): recorded by the list kernel's own completion (its stop
// event; the inline kernel, which reads no device records, takes none).
int launch_trace(const FrameRec& f, const SphereRec* host_spheres, void* stream,
                 const DumpArgs* dump = nullptr, void* done_event = nullptr);
// "release" for the shipped build; "diagnostic" (-DSFRT_EXP: wrong bytes by design) or
// "ab" (EXTRA build flags, tools/ab_libs.py) otherwise.
const char* trace_build_flavour();
// Tile grid of the kernel launch_trace picks for f when that kernel takes part in
// the adaptive tile order: a key naming the grid (> 0) and its tile count; else 0.
long long trace_tile_key(const FrameRec& f, long long* tiles);

}  // namespace sfrt
