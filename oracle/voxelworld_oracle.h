/* voxelworld_oracle.h -- TEST INFRASTRUCTURE ONLY (see voxelworld_oracle.c). */
#ifndef VOXELWORLD_ORACLE_H
#define VOXELWORLD_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OVOX_EMPTY (-32768) /* no block in this cell */
#define OVOX_SLOTS 10

typedef struct {
  float pos[3];
  float size[2];
  float r, g, b;
  float dist_to_camera;
  int32_t texture_id;
} ovox_dynamic; /* struct Dynamic (World.h:25-38), the fields Raycast reads */

typedef struct {
  float pos[3];
  float intensity, r, g, b;
  int32_t shadows;
} ovox_light; /* struct Light (World.h:40-47) */

typedef struct {
  const uint8_t* rgba; /* RGBA8 rows */
  int32_t w, h;
} ovox_texture;

typedef struct {
  int32_t width, height;
  float cam_pos[3];
  float cam_rotation, cam_hrotation;
  float fov_h, fov_v; /* radians (World.cpp:55-56 applied) */
  float shadow_distance, view_distance;
  const int16_t* blocks; /* dense grid, index (x*ny + y)*nz + z; textureID or OVOX_EMPTY */
  int32_t nx, ny, nz;
  ovox_texture textures[OVOX_SLOTS];
  ovox_texture dyn_textures[OVOX_SLOTS];
  uint8_t colors[OVOX_SLOTS][4];
  const ovox_dynamic* dyn; /* `dyn`, in list order */
  int32_t ndyn;
  const ovox_light* lights; /* `alights`, in list order */
  int32_t nlights;
} ovox_scene;

void ovox_update_image(const ovox_scene* sc, uint8_t* rgba, int ystart, int yadd, int xstart,
                       int xadd);
void ovox_render_threaded(const ovox_scene* sc, uint8_t* rgba, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
