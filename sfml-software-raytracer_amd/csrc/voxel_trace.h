// voxel_trace.h -- launch records shared by the voxel World host mirror
// (sfrt_voxel.cpp) and its gfx950 kernel (voxel_trace.hip).  SURVEY 8f f2.
//
// Per-frame terms the reference recomputes per pixel with libm are computed
// once on the host with the same expressions (World.cpp:62-87): per column
// i the ray's x/z direction (sinf, cosf, the edge-distortion divide) and
// atan2f(dir.z, dir.x) of VAngleXZ; per row j dir.y and r->yscale; per
// dynamic object its VNormalizeXZ'd direction's atan2f.  The kernel needs no
// transcendental.
#pragma once

#include <stdint.h>

namespace sfrt {

constexpr int kVoxSlots = 10;              // textures / dynTextures / colors (World.h:90-92)
constexpr int16_t kVoxEmpty = -32768;
// Block grid limits (sfrt_voxel_set_blocks refuses larger grids): the reference's map key
// (x << 20) + (y << 10) + z (World.cpp:385) addresses x < 2048, y, z < 1024 without overlap.
constexpr int kVoxMaxX = 2048, kVoxMaxY = 1024, kVoxMaxZ = 1024;
// On the device the world is the key-indexed byte array of cell_hit (voxel_trace.hip): byte
// (x << 20) + (y << 10) + z holds id + kVoxCellBias for a block (ids are in (-kVoxSlots,
// kVoxSlots)), 0 for no block; nx << 20 bytes, at most 2 GiB, so the buffer range fits an int.
constexpr int kVoxCellBias = 10;
static_assert(kVoxMaxY == 1024 && kVoxMaxZ == 1024, "the key's y and z fields are 10 bits");
static_assert((long long)kVoxMaxX << 20 <= (1ll << 31), "byte offsets and the range fit 31 bits");
static_assert(2 * (kVoxSlots - 1) + 1 <= 255, "a code fits a byte");

struct VoxDyn {                             // struct Dynamic fields Raycast reads (World.h:25-38)
  float px, py, pz;
  float sx, sy;                             // size
  float r, g, b;
  float dist;                               // distToCamera
  float atan_b;                             // atan2f of VNormalizeXZ(pos - cam.pos) (World.cpp:361)
  int32_t tex;
  int32_t pad;
};

struct VoxLight {                           // struct Light (World.h:40-47)
  float px, py, pz;
  // Squared distances dd >= dd_pass have intensity / dd - dd * 0.002f <= 0 in binary32
  // (World.cpp:425-426: the light adds nothing there): dd_pass is the smallest such float, found
  // on the host by bisection over the bit patterns (the test is monotone in dd; 0 when no dd
  // passes).  The kernel's per-wave skip tests the fma-evaluated squared distance, within
  // 6 ulp (relative 2^-20) of the reference's, against dd_skip = RU(dd_pass / (1 - 2^-20)):
  // ddf >= dd_skip implies dd >= dd_pass.  Beside the position, so that the skip test's four
  // dwords are one scalar load.
  float dd_skip;
  float intensity, r, g, b;
  int32_t shadows;
};

struct VoxTex {
  const uint32_t* texels;                   // RGBA8
  int32_t w, h;
};

struct VoxFrame {
  float cam[3];
  float view_distance, shadow_distance;
  uint32_t maxiter;                         // (unsigned)(viewDistance * 1.5f), World.cpp:322
  int32_t xstart, xadd, ystart, yadd;
  int32_t sub_w, sub_row0, sub_rows;
  const float* col;                         // per column i: dir.x, dir.z, atan2f(dir.z, dir.x)
  const float* row;                         // per row j: dir.y, yscale
  const uint8_t* cells;                     // key-indexed codes (cell_hit), nx << 20 bytes
  uint32_t cell_bytes;                      // nx << 20: the buffer range
  // The fast primary DDA's bound (sfrt_voxel.cpp dda_qlim): a ray whose direction
  // has max|d_k| <= dda_qlim * min|d_k| keeps every DDA position below 2^30 in magnitude, where
  // a plain v_cvt_i32_f32 equals to_i32; 0 sends every wave to the guarded DDA
  float dda_qlim;
  VoxTex tex[kVoxSlots];
  VoxTex dyn_tex[kVoxSlots];
  uint32_t colors[kVoxSlots];               // RGBA8 packed
  const VoxDyn* dyn;
  int32_t ndyn;
  const VoxLight* lights;
  int32_t nlights;
  long long out_pitch;
  uint32_t* out;
  int* status;                              // bit 1: out-of-range texel read
  // Adaptive tile order (sfrt_sched.h): one 8x8 tile per one-wave
  // workgroup, slot -> tile_order; cost = the tile's DDA + shadow-ray steps.
  const uint32_t* tile_order;
  uint8_t* tile_cost;
  const uint8_t* prev_cost;
  uint32_t* next_order;
  // tile_order's classes are the ones in tile_cost: store only changed classes (sfrt_device.h
  // store_cost, sfrt_sched.h TileSchedPtrs::cost_diff)
  int32_t cost_diff;
};

// Tile grid of launch_voxel for f (8x8 tiles): key (> 0) and tile count.
long long voxel_tile_key(const VoxFrame& f, long long* tiles);
// done_event (hipEvent_t, may be null): recorded by the launch's own completion (its stop event).
int launch_voxel(const VoxFrame& f, void* stream, void* done_event = nullptr);

// Rewrites the key-indexed grid `cells` for a world of nx x ny x nz codes (`codes`, device,
// x-major then y then z, as set_blocks takes them): every byte of planes x < bx, rows y < by,
// columns z < bz gets its code inside the world and 0 outside it.  (bx, by, bz) covers the world
// and every byte an earlier world may have left non-zero, so the grid is the new world's alone.
int launch_voxel_cells(uint8_t* cells, const uint8_t* codes, int nx, int ny, int nz, int bx, int by,
                       int bz, void* stream);

}  // namespace sfrt
