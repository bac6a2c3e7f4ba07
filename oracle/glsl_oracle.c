/*
 * glsl_oracle.c -- CPU restatement of the reference's GLSL renderer
 * rayShader.frag.
 *
 *   TEST INFRASTRUCTURE ONLY: the parity checker for libsfrt.so's GLSL-mode
 *   kernel.  The product never links, calls or falls back to it.
 *
 * Restates (paths relative to /root/reference/Raytracing/):
 *   main()                rayShader.frag:163-179  (oglsl_pixel)
 *   Raycast(pos, dir, 1)  rayShader.frag:63-161   (raycast)
 *   polsmin               rayShader.frag:57-61
 *   VRotateX / VRotateY   rayShader.frag:16-25
 * and the pipeline state the shader depends on: `ground` = Floor.png with
 * setRepeated(true) + generateMipmap() (SphereWorld.cpp:52-57); the draw into
 * a width x height RenderTexture (Source.cpp:146-153).
 *
 * GLSL leaves what follows to the driver; this restatement fixes it, and the
 * GPU kernel is held to it bit for bit:
 *  - float is IEEE binary32, round to nearest, no contraction; `/`, sqrt are
 *    correctly rounded; length(v) = sqrt(dot(v, v)), dot left to right,
 *    normalize(v) = v / length(v), distance(a, b) = length(a - b);
 *  - min/max/clamp/step/mod/smoothstep/sign are the GLSL spec's formulas
 *    (min(x, y) = y < x ? y : x, max(x, y) = x < y ? y : x, mod = x - y*floor(x/y));
 *  - sin, cos (per frame), atan(y, x) and acos are glibc 2.35's sinf, cosf,
 *    atan2f and acosf;
 *  - NVIDIA-lenient implicit int<->float conversions (:47, :76, :105, :114,
 *    :117-120, :130) are exact conversions; float -> int truncates;
 *  - gl_FragCoord = (i + 0.5, height - 1 - row + 0.5): row 0 is the top of
 *    the image, i.e. the last row of the OpenGL framebuffer (SFML flips
 *    RenderTexture contents for display);
 *  - textureLod: GL_NEAREST magnification for lod <= 0 (and NaN), otherwise
 *    GL_NEAREST_MIPMAP_LINEAR (SFML's min filter with mipmaps and smooth off):
 *    nearest texel of levels floor(lod) and floor(lod)+1, blended
 *    (1 - f) * t1 + f * t2 with f = lod - floor(lod); level q (the 1x1 level)
 *    alone for lod >= q.  Texel = byte / 255.0f; REPEAT wrap; a non-finite
 *    or |u| >= 2^24 coordinate reads texel 0 of its axis.  Mip level k+1 is
 *    the 2x2 (or 2x1) box average of level k, rounded half up in 8 bits;
 *  - framebuffer conversion: NaN -> 0, else clamp to [0, 1] and
 *    floor(v * 255 + 0.5).
 *
 * Pinning: no OpenGL context can run here (no EGL/OSMesa/Xvfb),
 * so this row is UNPINNED against the reference's own output; the scene
 * fixture (glsl_scenes.py) is pinned by reproducing the survey's srand(0)
 * default10 wall list.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "glsl_oracle.h"

#define MARCH_CAP (1L << 20) /* the shader has no cap; counts, never hit in tests */

typedef struct { float x, y, z; } v3;
static v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 scale(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static v3 fscale(float s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }
static v3 divs(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
static float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static float length(v3 a) { return sqrtf(dot(a, a)); }
static v3 normalize(v3 a) { return divs(a, length(a)); }
static float distance(v3 a, v3 b) { return length(sub(a, b)); }
static v3 ball(const oglsl_uniforms* u, int k) {
  return mk(u->spheres[k][0], u->spheres[k][1], u->spheres[k][2]);
}

static float g_min(float x, float y) { return y < x ? y : x; }
static float g_max(float x, float y) { return x < y ? y : x; }
static float g_clamp(float x, float lo, float hi) { return g_min(g_max(x, lo), hi); }
static float g_step(float edge, float x) { return x < edge ? 0.0f : 1.0f; }
static float g_mod(float x, float y) { return x - y * floorf(x / y); }
static float g_smoothstep(float e0, float e1, float x) {
  const float t = g_clamp((x - e0) / (e1 - e0), 0.0f, 1.0f);
  return t * t * (3.0f - 2.0f * t);
}
static int g_sign_i(int x) { return x > 0 ? 1 : (x < 0 ? -1 : 0); }

/* rayShader.frag:16-25 */
static v3 rotate_x(v3 v, float amount) {
  const float s = sinf(amount), c = cosf(amount);
  return mk(v.x, v.y * c - v.z * s, v.y * s + v.z * c);
}
static v3 rotate_y(v3 v, float amount) {
  const float s = sinf(amount), c = cosf(amount);
  return mk(v.x * c + v.z * s, v.y, -v.x * s + v.z * c);
}
/* rayShader.frag:57-61 */
static float polsmin(float a, float b, float k) {
  const float h = g_max(k - fabsf(a - b), 0.0f) / k;
  return g_min(a, b) - h * h * k * (1.0f / 4.0f);
}

/* ---- ground texture: REPEAT + generateMipmap ---- */
#define MAX_LEVELS 16
typedef struct {
  int levels;
  int w[MAX_LEVELS], h[MAX_LEVELS];
  uint8_t* px[MAX_LEVELS];
} mip_chain;

static void mip_build(mip_chain* m, const uint8_t* ground, int gw, int gh) {
  memset(m, 0, sizeof *m);
  m->w[0] = gw;
  m->h[0] = gh;
  m->px[0] = (uint8_t*)malloc((size_t)gw * gh * 4);
  memcpy(m->px[0], ground, (size_t)gw * gh * 4);
  int k = 0;
  while (m->w[k] > 1 || m->h[k] > 1) {
    const int w = m->w[k], h = m->h[k];
    const int nw = w > 1 ? w / 2 : 1, nh = h > 1 ? h / 2 : 1;
    const int fx = w > 1 ? 2 : 1, fy = h > 1 ? 2 : 1, n = fx * fy;
    uint8_t* dst = (uint8_t*)malloc((size_t)nw * nh * 4);
    for (int y = 0; y < nh; y++)
      for (int x = 0; x < nw; x++)
        for (int c = 0; c < 4; c++) {
          int sum = 0;
          for (int dy = 0; dy < fy; dy++)
            for (int dx = 0; dx < fx; dx++)
              sum += m->px[k][((size_t)(y * fy + dy) * w + (x * fx + dx)) * 4 + c];
          dst[((size_t)y * nw + x) * 4 + c] = (uint8_t)((sum + n / 2) / n);
        }
    k++;
    m->w[k] = nw;
    m->h[k] = nh;
    m->px[k] = dst;
  }
  m->levels = k + 1;
}

static void mip_free(mip_chain* m) {
  for (int k = 0; k < m->levels; k++) free(m->px[k]);
}

static int wrap(float coord, int n) {
  const float u = floorf(coord * (float)n);
  if (!(fabsf(u) < 16777216.0f)) return 0;
  int i = (int)u % n;
  return i < 0 ? i + n : i;
}

static void texel(const mip_chain* m, int level, float s, float t, float out[4]) {
  const int i = wrap(s, m->w[level]), j = wrap(t, m->h[level]);
  const uint8_t* p = m->px[level] + ((size_t)j * m->w[level] + i) * 4;
  for (int c = 0; c < 4; c++) out[c] = (float)p[c] / 255.0f;
}

static void texture_lod(const mip_chain* m, float s, float t, float lod, float out[4]) {
  const int q = m->levels - 1;
  if (!(lod > 0.0f)) {
    texel(m, 0, s, t, out);
  } else if (lod >= (float)q) {
    texel(m, q, s, t, out);
  } else {
    const float fl = floorf(lod);
    const int d1 = (int)fl;
    const float f = lod - fl;
    float t1[4], t2[4];
    texel(m, d1, s, t, t1);
    texel(m, d1 + 1, s, t, t2);
    for (int c = 0; c < 4; c++) out[c] = (1.0f - f) * t1[c] + f * t2[c];
  }
}

static uint8_t unorm8(float v) {
  if (v != v) return 0;
  if (!(v > 0.0f)) return 0;
  if (!(v < 1.0f)) return 255;
  return (uint8_t)(int)floorf(v * 255.0f + 0.5f);
}

/* ---- rayShader.frag:63-161 ---- */
static void raycast(const oglsl_uniforms* u, const mip_chain* m, v3 pos, v3 dir, int lit,
                    float c_out[4], oglsl_dump* d, long* capped) {
  const int sc = u->sphere_count, all = u->all_spheres_count, lc = u->light_count;
  const v3 campos = mk(u->campos[0], u->campos[1], u->campos[2]);
  dir = normalize(dir);
  int drawSphere = 0;
  float totalDist = 0.0f;
  float normalsign = -1.0f;

  for (int j = 0; j < sc * 3; j++) {                       /* :71-85 */
    const int i = j % sc;
    const v3 rpos = sub(pos, ball(u, i));
    const int checkstep = (int)g_step(length(rpos), u->spheres[i][3]);
    const float b = (float)checkstep * 2.0f * dot(rpos, dir);
    const float c = (float)checkstep * dot(rpos, rpos) - u->spheres[i][3] * u->spheres[i][3];
    const float tosurf = (float)checkstep * (-b + fabsf(sqrtf(b * b - 4.0f * c))) * 0.5f;
    drawSphere = checkstep * i + (1 - checkstep) * drawSphere;
    pos = add(pos, scale(dir, tosurf));
    totalDist += tosurf;
  }
  if (d) {
    d->dir[0] = dir.x; d->dir[1] = dir.y; d->dir[2] = dir.z;
    d->wall_pos[0] = pos.x; d->wall_pos[1] = pos.y; d->wall_pos[2] = pos.z;
    d->wall_dist = totalDist;
    d->wall_sphere = drawSphere;
  }

  float ballDist = 0.0f;
  float shortest = 999999999.0f;
  int closest = 0;
  float smoothDist = 999999999.0f;
  const float minstep = 0.01f;
  v3 smoothNormal = mk(0, 0, 0);
  long steps = 0;
  while (ballDist < totalDist && smoothDist > minstep) {  /* :94-112 */
    if (++steps > MARCH_CAP) {
      (*capped)++;
      break;
    }
    const v3 testPos = add(campos, scale(dir, ballDist));
    smoothDist = 999999999.0f;
    closest = 0;
    shortest = 9999999.0f;
    smoothNormal = mk(0, 0, 0);
    for (int j = sc; j < all; j++) {
      const v3 tos = sub(ball(u, j), testPos);
      const float otherDist = length(tos) - u->spheres[j][3];
      smoothDist = polsmin(smoothDist, otherDist, 0.5f);
      closest = (int)(g_step(shortest, otherDist) * (float)closest +
                      (1.0f - g_step(shortest, otherDist)) * (float)j);
      shortest = g_min(shortest, otherDist);
      const float normalFactor = g_clamp(otherDist, 0.0f, 0.5f) * 2.0f;
      smoothNormal = sub(fscale(normalFactor, smoothNormal), fscale(1.0f - normalFactor, tos));
    }
    ballDist += smoothDist + minstep;
  }

  const int checkstep = (int)g_step(minstep, smoothDist);  /* :114-120 */
  totalDist = (float)checkstep * totalDist + (float)(1 - checkstep) * ballDist;
  drawSphere = checkstep * drawSphere + (1 - checkstep) * closest;
  pos = add(fscale((float)checkstep, pos),
            fscale((float)(1 - checkstep), add(campos, scale(dir, ballDist))));
  normalsign = (float)checkstep * normalsign + (float)(1 - checkstep);

  /* :123-126 */
  const v3 rpos = add(scale(smoothNormal, 1.0f - (float)checkstep),
                      fscale((float)checkstep, sub(pos, ball(u, drawSphere))));
  const float* uv = u->uvs[drawSphere];
  const float ycoord =
      g_mod(rpos.y / (0.8f + 0.2f * (fabsf(rpos.x) + fabsf(rpos.z))), uv[0]) + uv[3];
  const float xcoord = g_mod(g_min(fabsf(rpos.z), fabsf(rpos.x)), uv[0]) + uv[2];
  float c[4];
  texture_lod(m, xcoord, ycoord, totalDist * 0.05f, c);

  float brightness = (float)lit * 1.0f / g_max(totalDist, 1.0f);       /* :128 */
  const float lightc = g_step((float)sc, (float)drawSphere) *          /* :130 */
                       g_step((float)drawSphere, (float)(sc + lc - 1));

  for (int i = sc; i < sc + lc; i++) {                                  /* :132-151 */
    const v3 tolight = sub(ball(u, i), pos);
    const float tolightlen = length(tolight);
    const v3 tolightnorm = divs(tolight, tolightlen);
    const float normalMult = length(add(normalize(scale(rpos, normalsign)), tolightnorm)) - 1.0f;
    float shadow = 1.0f;
    for (int j = sc + lc; j < all && drawSphere < j; j++) {
      const float lightshadowdist = distance(ball(u, i), ball(u, j));
      const float sanglet = atan2f(u->spheres[j][3], lightshadowdist);
      float sangle = acosf(dot(mk(-tolightnorm.x, -tolightnorm.y, -tolightnorm.z),
                               divs(sub(ball(u, j), ball(u, i)), lightshadowdist)));
      const float pointshadowdist = 1.5f / (0.8f + 0.2f * distance(pos, ball(u, j)));
      sangle = sangle * pointshadowdist - (pointshadowdist - 1.0f) * sanglet;
      shadow *= g_clamp(sangle / sanglet + 1.0f -
                            g_step(lightshadowdist, tolightlen) * g_smoothstep(0.0f, 0.5f, normalMult),
                        1.0f - (float)abs(g_sign_i(j - drawSphere)), 1.0f);
    }
    brightness += 10.0f / tolightlen / tolightlen * g_max(0.5f + 0.5f * normalMult, 0.0f) * shadow;
  }

  brightness = lightc * 2.0f + (1.0f - lightc) * brightness;          /* :153-158 */
  const float* L = u->lights[drawSphere];
  for (int k = 0; k < 3; k++) c[k] = L[3] * L[k] * 0.5f + (1.0f - L[3]) * c[k];
  const float viewDist = 50.0f;
  const float f = g_clamp(brightness, 0.0f, 3.0f) + g_min(-totalDist + viewDist * 0.66f, 0.0f);
  for (int k = 0; k < 3; k++) c[k] *= f;
  c[3] = 1.0f;
  memcpy(c_out, c, sizeof c);
  if (d) {
    d->march_steps = (int32_t)steps;
    d->ball_dist = ballDist;
    d->smooth_dist = smoothDist;
    d->checkstep = checkstep;
    d->draw_sphere = drawSphere;
    d->total_dist = totalDist;
    d->xcoord = xcoord;
    d->ycoord = ycoord;
    d->brightness = brightness;
    memcpy(d->color, c, sizeof c);
  }
}

/* rayShader.frag:163-179 for the fragment at target pixel (i, row). */
static void shade_pixel(const oglsl_uniforms* u, const mip_chain* m, int height, int i, int row,
                        uint8_t* px, oglsl_dump* d, long* capped) {
  v3 up = rotate_x(mk(0, 1, 0), -u->rotation[1]);
  v3 forward = rotate_x(mk(0, 0, 1), -u->rotation[1]);
  const v3 right = rotate_y(mk(1, 0, 0), u->rotation[0]);
  forward = rotate_y(forward, u->rotation[0]);
  up = rotate_y(up, u->rotation[0]);
  const float fx = (float)i + 0.5f, fy = (float)(height - 1 - row) + 0.5f;
  const float ax = -u->fov[0] + u->fov[0] / u->size[0] * 2.0f * fx;
  const float ay = -u->fov[1] + u->fov[1] / u->size[1] * 2.0f * fy;
  const v3 dir = add(add(forward, scale(right, ax)), scale(up, ay));
  float c[4];
  raycast(u, m, mk(u->campos[0], u->campos[1], u->campos[2]), dir, 1, c, d, capped);
  if (px)
    for (int k = 0; k < 4; k++) px[k] = unorm8(c[k]);
}

long oglsl_render(const oglsl_uniforms* u, const uint8_t* ground, int gw, int gh, int width,
                  int height, int row0, int rows, uint8_t* out) {
  mip_chain m;
  mip_build(&m, ground, gw, gh);
  long capped = 0;
  for (int r = 0; r < rows; r++)
    for (int i = 0; i < width; i++)
      shade_pixel(u, &m, height, i, row0 + r, out + ((size_t)r * width + i) * 4, NULL, &capped);
  mip_free(&m);
  return capped;
}

typedef struct {
  const oglsl_uniforms* u;
  const mip_chain* m;
  int width, height, t, nt;
  uint8_t* out;
  int32_t* steps;
  long capped;
} job;

static void* worker(void* p) {
  job* jb = (job*)p;
  for (int r = jb->t; r < jb->height; r += jb->nt)
    for (int i = 0; i < jb->width; i++) {
      if (jb->out) {
        shade_pixel(jb->u, jb->m, jb->height, i, r, jb->out + ((size_t)r * jb->width + i) * 4, NULL,
                    &jb->capped);
      } else {
        oglsl_dump d;
        shade_pixel(jb->u, jb->m, jb->height, i, r, NULL, &d, &jb->capped);
        jb->steps[(size_t)r * jb->width + i] = d.march_steps;
      }
    }
  return NULL;
}

static long run_threads(const oglsl_uniforms* u, const mip_chain* m, int width, int height,
                        uint8_t* out, int32_t* steps, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  job jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (job){u, m, width, height, t, nthreads, out, steps, 0};
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  long capped = 0;
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    capped += jobs[t].capped;
  }
  return capped;
}

long oglsl_render_threaded(const oglsl_uniforms* u, const uint8_t* ground, int gw, int gh,
                           int width, int height, uint8_t* out, int nthreads) {
  mip_chain m;
  mip_build(&m, ground, gw, gh);
  const long capped = run_threads(u, &m, width, height, out, NULL, nthreads);
  mip_free(&m);
  return capped;
}

void oglsl_march_steps(const oglsl_uniforms* u, int width, int height, int32_t* steps,
                       int nthreads) {
  static const uint8_t one_texel[4] = {0, 0, 0, 255};
  mip_chain m;
  mip_build(&m, one_texel, 1, 1);
  run_threads(u, &m, width, height, NULL, steps, nthreads);
  mip_free(&m);
}

void oglsl_pixel(const oglsl_uniforms* u, const uint8_t* ground, int gw, int gh, int width,
                 int height, int i, int row, oglsl_dump* d) {
  (void)width;
  mip_chain m;
  mip_build(&m, ground, gw, gh);
  long capped = 0;
  memset(d, 0, sizeof *d);
  shade_pixel(u, &m, height, i, row, NULL, d, &capped);
  mip_free(&m);
}
