/* glsl_oracle.h -- TEST INFRASTRUCTURE ONLY (see glsl_oracle.c). */
#ifndef GLSL_ORACLE_H
#define GLSL_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OGLSL_MAX 100 /* uniform vec4 spheres[100] (rayShader.frag:6-8) */

/* The shader's uniform block (rayShader.frag:1-11) as main() and
 * UpdateSpheres upload it (Source.cpp:143-146, SphereWorld.cpp:214-238). */
typedef struct {
  float campos[3];
  float rotation[2]; /* (cam.rotation, cam.hrotation) */
  float fov[2];      /* radians */
  float size[2];     /* render-target size */
  int32_t sphere_count, all_spheres_count, light_count;
  float spheres[OGLSL_MAX][4];
  float uvs[OGLSL_MAX][4];
  float lights[OGLSL_MAX][4];
} oglsl_uniforms;

/* Per-pixel intermediates for diagnostics and tests. */
typedef struct {
  float dir[3];
  float wall_pos[3];
  float wall_dist;
  int32_t wall_sphere;
  int32_t march_steps;
  float ball_dist, smooth_dist;
  int32_t checkstep, draw_sphere;
  float total_dist, xcoord, ycoord, brightness;
  float color[4]; /* before the framebuffer conversion */
} oglsl_dump;

/* Target rows [row0, row0+rows) of a width x height render target, written
 * top-down (the row order of rt.getTexture().copyToImage()), RGBA8, pitch
 * width*4.  ground: RGBA8 rows, power-of-two sides (setRepeated(true) +
 * generateMipmap(), SphereWorld.cpp:52-57).  Returns the number of pixels
 * whose march hit the iteration cap (0 for every scene in the tests). */
long oglsl_render(const oglsl_uniforms* u, const uint8_t* ground, int gw, int gh, int width,
                  int height, int row0, int rows, uint8_t* out);
long oglsl_render_threaded(const oglsl_uniforms* u, const uint8_t* ground, int gw, int gh,
                           int width, int height, uint8_t* out, int nthreads);
void oglsl_pixel(const oglsl_uniforms* u, const uint8_t* ground, int gw, int gh, int width,
                 int height, int i, int row, oglsl_dump* d);
/* March-step histogram support: steps[row*width + i] for the whole target. */
void oglsl_march_steps(const oglsl_uniforms* u, int width, int height, int32_t* steps,
                       int nthreads);

#ifdef __cplusplus
}
#endif
#endif
