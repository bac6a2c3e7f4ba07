/* sphereworld_oracle.h -- TEST INFRASTRUCTURE ONLY (see sphereworld_oracle.c). */
#ifndef SPHEREWORLD_ORACLE_H
#define SPHEREWORLD_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  float x, y, z, radius;
} oracle_sphere;

typedef struct {
  int width, height;
  float cam_pos[3];
  float cam_rotation, cam_hrotation;
  float fov_h, fov_v;            /* radians, as UpdateImage sees them */
  const oracle_sphere* spheres;  /* in UpdateSpheres order */
  int sphere_count;
  const uint8_t* texture;        /* RGBA8, tex_w * tex_h * 4 */
  int tex_w, tex_h;
  /* Extension ("all textures"): a texture slot per sphere,
   * in sphere order; NULL = slot 0 (`texture`) for every sphere, which is the
   * reference.  Slots 1..9 are textures[k] with tex_ws[k] x tex_hs[k] texels. */
  const int32_t* sphere_tex;
  const uint8_t* textures[10];
  int tex_ws[10], tex_hs[10];
} oracle_scene;

typedef struct {
  float pos[3];
  int draw;
  int iters;
  float xcoord, ycoord, brightness;
  unsigned texel[2];
  uint8_t rgba[4];
} oracle_pixel_dump;

int oracle_scene_valid(const oracle_scene* sc);
void oracle_update_image(const oracle_scene* sc, uint8_t* rgba, int ystart, int yadd,
                         int xstart, int xadd);
void oracle_render_band(const oracle_scene* sc, uint8_t* band, int row0, int rows);
void oracle_render_threaded(const oracle_scene* sc, uint8_t* rgba, int nthreads);
void oracle_iteration_map(const oracle_scene* sc, int32_t* iters, int nthreads);
void oracle_trace_dump(const oracle_scene* sc, int i, int j, oracle_pixel_dump* out);
void oracle_sort_spheres(oracle_sphere* s, int n, const float cam_pos[3]);
int oracle_add_sphere(oracle_sphere* s, int n, oracle_sphere add, const float cam_pos[3]);
float oracle_deg2rad(float deg);
uint64_t oracle_fnv1a64(const uint8_t* p, size_t n);

#ifdef __cplusplus
}
#endif
#endif
