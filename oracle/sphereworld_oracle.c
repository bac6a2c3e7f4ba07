/*
 * sphereworld_oracle.c -- CPU restatement of the reference's sphere-cave
 * trace-and-shade path.
 *
 *   TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the timed
 *   CPU baseline ("cpu_baseline.kind = port").  Only tests/, bench.py's
 *   cpu_baseline leg and __graft_entry__.smoke() may load it.  The product
 *   (libsfrt.so) never links, calls or falls back to it.
 *
 * What it restates (paths relative to /root/reference/Raytracing/):
 *   SphereWorld::UpdateImage   SphereWorld.cpp:83-112   (oracle_update_image)
 *   SphereWorld::Raycast       SphereWorld.cpp:355-382  (trace_pixel)
 *   VRotateX / VRotateY        SphereWorld.cpp:27-36
 *   VAngleXZ                   SphereWorld.cpp:324-328
 *   VNormalize / VLength       SphereWorld.cpp:330-343
 *   UpdateSpheres (sort part)  SphereWorld.cpp:199-212  (oracle_sort_spheres)
 *   AddSphere (prune + sort)   SphereWorld.cpp:177-190  (oracle_add_sphere)
 *   RenderThread interleave    Source.cpp:17-28         (oracle_render_threaded)
 *
 * Arithmetic is written expression-for-expression in the reference's order,
 * in IEEE binary32, and MUST be compiled with -ffp-contract=off and without
 * -ffast-math (oracle/Makefile).  Transcendentals are the host libm's
 * (glibc 2.35 here and on the GPU box: sinf, cosf, atan2f, asinf), exactly
 * what the reference calls through std::sin / std::atan2 / std::asinf.
 *
 * PARITY UNPINNED.  The reference itself cannot be built in this image: it
 * needs SFML 2.4.2 (SphereWorld.h:3 includes <SFML/Graphics.hpp>), which is
 * absent, and stand-in headers are not allowed.  It ships no tests, fixtures or
 * golden data.  So nothing here pins this restatement to the reference's own
 * output.  What exists is a sanity check: the survey's per-pixel march
 * iteration statistics from a stub-SFML build, which
 * tests/test_oracle_golden.py reproduces.  The survey's FNV-1a-64 frame hashes
 * from that stub build do NOT reproduce (the stub's Image/Color semantics are
 * unrecorded).  tests/golden/ holds hashes generated from THIS file.  See
 * DESIGN.md section 3.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "sphereworld_oracle.h"

/* SphereWorld.h:6-8 */
#define O_PI 3.1415926535f
#define O_PI2 6.28318530718f

typedef struct { float x, y, z; } v3;

static v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 vadd(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 vsub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 vmul(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static v3 vdiv(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }

/* SphereWorld.cpp:340-343 */
static float vlength(v3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }
/* SphereWorld.cpp:330-333 */
static v3 vnormalize(v3 v) { return vdiv(v, vlength(v)); }

/* SphereWorld.cpp:27-31 */
static v3 rot_x(v3 v, float amount) {
  float s = sinf(amount);
  float c = cosf(amount);
  return mk(v.x, v.y * c - v.z * s, v.y * s + v.z * c);
}
/* SphereWorld.cpp:32-36 */
static v3 rot_y(v3 v, float amount) {
  float s = sinf(amount);
  float c = cosf(amount);
  return mk(v.x * c + v.z * s, v.y, -v.x * s + v.z * c);
}

/* SphereWorld.cpp:324-328; a = hit point, b = sphere centre (both world space) */
static float angle_xz(v3 a, v3 b) {
  float ang = atan2f(b.z, b.x) - atan2f(a.z, a.x);
  return ang > O_PI ? ang - O_PI2 : ang < -O_PI ? ang + O_PI2 : ang;
}

static v3 sphere_pos(const oracle_sphere* s) { return mk(s->x, s->y, s->z); }

/* SphereWorld::Raycast, SphereWorld.cpp:355-382.  dir is the un-normalised
 * primary direction; the RGBA result is packed little-endian (r in byte 0). */
static uint32_t trace_pixel(const oracle_scene* sc, v3 dir, oracle_pixel_dump* dump) {
  const oracle_sphere* sp = sc->spheres;
  const int n = sc->sphere_count;
  v3 cam = mk(sc->cam_pos[0], sc->cam_pos[1], sc->cam_pos[2]);
  v3 pos = cam;                         /* :357 */
  dir = vnormalize(dir);                /* :358 */
  float largest = 1.0f;                 /* :359 */
  int draw = 0;                         /* :360 */
  int iters = 0;
  while (largest > 0) {                 /* :362 */
    largest = 0;
    for (int i = 0; i < n; i++) {       /* :364 */
      float dist = vlength(vsub(pos, sphere_pos(&sp[i])));
      if (sp[i].radius - dist > 0.01f) {               /* :366 */
        float t = sp[i].radius - dist;
        largest = largest < t ? t : largest;           /* std::max :367 */
        draw = i;                                      /* :368 */
      }
    }
    pos = vadd(pos, vmul(dir, largest));               /* :371 */
    iters++;
  }
  const oracle_sphere* d = &sp[draw];
  v3 dc = sphere_pos(d);
  float xcoord = angle_xz(pos, dc) / O_PI2 + 1.0f;                  /* :373 */
  float ycoord = (asinf(vnormalize(vsub(pos, dc)).y) / O_PI + 0.5f); /* :374 */
  float len = vlength(vsub(pos, cam));
  float brightness = 3.0f / (len < 3.0f ? 3.0f : len);              /* :375 */
  /* :376-377: getPixel((unsigned)(fmodf(..)*texsize.x), (unsigned)(..)); the
   * texture is textures[0] unless the per-sphere extension names another slot */
  const int slot = sc->sphere_tex ? sc->sphere_tex[draw] : 0;
  const uint8_t* tex = slot ? sc->textures[slot] : sc->texture;
  const int tw = slot ? sc->tex_ws[slot] : sc->tex_w, th = slot ? sc->tex_hs[slot] : sc->tex_h;
  float fx = fmodf(xcoord * 4 * d->radius, 1.0f) * (float)(unsigned)tw;
  float fy = fmodf(ycoord * 2 * d->radius, 1.0f) * (float)(unsigned)th;
  unsigned tx = (unsigned)(int64_t)fx; /* x86-64 g++: cvttss2si to 64-bit, low 32 bits */
  unsigned ty = (unsigned)(int64_t)fy;
  const uint8_t* px = tex + ((size_t)(tx + ty * (unsigned)tw)) * 4;
  uint8_t r = px[0], g = px[1], b = px[2], a = px[3];
  r = (uint8_t)(int)(r * brightness);                                 /* :378 */
  g = (uint8_t)(int)(g * brightness);                                 /* :379 */
  b = (uint8_t)(int)(b * brightness);                                 /* :380 */
  if (dump) {
    dump->pos[0] = pos.x; dump->pos[1] = pos.y; dump->pos[2] = pos.z;
    dump->draw = draw;
    dump->iters = iters;
    dump->xcoord = xcoord;
    dump->ycoord = ycoord;
    dump->brightness = brightness;
    dump->texel[0] = tx; dump->texel[1] = ty;
  }
  return (uint32_t)r | ((uint32_t)g << 8) | ((uint32_t)b << 16) | ((uint32_t)a << 24);
}

/* Primary direction of pixel (i, j): SphereWorld.cpp:85-106, basis rebuilt
 * per pixel exactly as the reference does. */
static v3 primary_dir(const oracle_scene* sc, int i, int j) {
  float vStart = -sc->fov_v;                              /* :85 */
  float vIncreaseBy = sc->fov_v / sc->height * 2;         /* :86 */
  float hStart = -sc->fov_h;                              /* :88 */
  float hIncreaseBy = sc->fov_h / sc->width * 2;          /* :89 */
  float hray = (hStart + hIncreaseBy * i);                /* :95 */
  float vray = (vStart + j * vIncreaseBy);                /* :98 */
  v3 up = rot_x(mk(0, -1, 0), -sc->cam_hrotation);        /* :100 */
  v3 forward = rot_x(mk(0, 0, 1), -sc->cam_hrotation);    /* :101 */
  v3 right = rot_y(mk(1, 0, 0), sc->cam_rotation);        /* :102 */
  forward = rot_y(forward, sc->cam_rotation);             /* :103 */
  up = rot_y(up, sc->cam_rotation);                       /* :104 */
  return vadd(vadd(forward, vmul(right, hray)), vmul(up, vray)); /* :106 */
}

int oracle_scene_valid(const oracle_scene* sc) {
  if (!sc || sc->width <= 0 || sc->height <= 0) return 0;
  if (sc->sphere_count <= 0 || !sc->spheres) return 0;  /* spheres.at(0) throws */
  if (!sc->texture || sc->tex_w <= 0 || sc->tex_h <= 0) return 0;
  if (sc->sphere_tex)
    for (int i = 0; i < sc->sphere_count; i++) {
      const int k = sc->sphere_tex[i];
      if (k < 0 || k >= 10 || (k && (!sc->textures[k] || sc->tex_ws[k] <= 0 || sc->tex_hs[k] <= 0)))
        return 0;
    }
  return 1;
}

/* SphereWorld::UpdateImage(v, ystart, yadd, xstart, xadd), SphereWorld.cpp:83-112.
 * rgba is the full width*height*4 frame; only the addressed pixels are written. */
void oracle_update_image(const oracle_scene* sc, uint8_t* rgba, int ystart, int yadd,
                         int xstart, int xadd) {
  for (int i = xstart; i < sc->width; i += xadd) {       /* :94 */
    for (int j = ystart; j < sc->height; j += yadd) {    /* :97 */
      uint32_t c = trace_pixel(sc, primary_dir(sc, i, j), NULL);
      memcpy(rgba + ((size_t)j * sc->width + i) * 4, &c, 4); /* setPixel :109 */
    }
  }
}

/* Per-pixel march iteration counts (reference loop trips of :362), row-major;
 * rows == t (mod nthreads) per thread. */
typedef struct {
  const oracle_scene* sc;
  int32_t* iters;
  int t, T;
} iter_arg;

static void* iteration_thread(void* p) {
  iter_arg* a = (iter_arg*)p;
  oracle_pixel_dump d;
  for (int j = a->t; j < a->sc->height; j += a->T)
    for (int i = 0; i < a->sc->width; i++) {
      trace_pixel(a->sc, primary_dir(a->sc, i, j), &d);
      a->iters[(size_t)j * a->sc->width + i] = d.iters;
    }
  return NULL;
}

void oracle_iteration_map(const oracle_scene* sc, int32_t* iters, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  iter_arg* args = (iter_arg*)malloc(sizeof(iter_arg) * nthreads);
  for (int t = 0; t < nthreads; t++) {
    args[t].sc = sc; args[t].iters = iters; args[t].t = t; args[t].T = nthreads;
    pthread_create(&th[t], NULL, iteration_thread, &args[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  free(args);
}

void oracle_trace_dump(const oracle_scene* sc, int i, int j, oracle_pixel_dump* out) {
  uint32_t c = trace_pixel(sc, primary_dir(sc, i, j), out);
  memcpy(out->rgba, &c, 4);
}

/* Rows [row0, row0+rows) of the frame into a band buffer (row0 is a global row). */
void oracle_render_band(const oracle_scene* sc, uint8_t* band, int row0, int rows) {
  for (int j = row0; j < row0 + rows && j < sc->height; j++)
    for (int i = 0; i < sc->width; i++) {
      uint32_t c = trace_pixel(sc, primary_dir(sc, i, j), NULL);
      memcpy(band + ((size_t)(j - row0) * sc->width + i) * 4, &c, 4);
    }
}

typedef struct {
  const oracle_scene* sc;
  uint8_t* rgba;
  int t, T;
} thread_arg;

static void* render_thread(void* p) {
  thread_arg* a = (thread_arg*)p;
  /* Source.cpp:21 -- world.UpdateImage(&gameImage, num, threadCount, cycle, fullCycles),
   * here with one full column cycle: rows == t (mod T), every column. */
  oracle_update_image(a->sc, a->rgba, a->t, a->T, 0, 1);
  return NULL;
}

void oracle_render_threaded(const oracle_scene* sc, uint8_t* rgba, int nthreads) {
  if (nthreads <= 1) {
    oracle_update_image(sc, rgba, 0, 1, 0, 1);
    return;
  }
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  thread_arg* args = (thread_arg*)malloc(sizeof(thread_arg) * nthreads);
  for (int t = 0; t < nthreads; t++) {
    args[t].sc = sc; args[t].rgba = rgba; args[t].t = t; args[t].T = nthreads;
    pthread_create(&th[t], NULL, render_thread, &args[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  free(args);
}

/* UpdateSpheres sort part, SphereWorld.cpp:199-212: stable insertion by
 * |c - cam| + r, inserted after equal keys. */
void oracle_sort_spheres(oracle_sphere* s, int n, const float cam_pos[3]) {
  v3 cam = mk(cam_pos[0], cam_pos[1], cam_pos[2]);
  oracle_sphere* tmp = (oracle_sphere*)malloc(sizeof(oracle_sphere) * (n > 0 ? n : 1));
  memcpy(tmp, s, sizeof(oracle_sphere) * n);
  int count = 0;
  for (int i = 0; i < n; i++) {
    float dist = vlength(vsub(sphere_pos(&tmp[i]), cam)) + tmp[i].radius;
    int ins = 0;
    for (int j = 0; j < count; j++) {
      if (dist < vlength(vsub(sphere_pos(&s[j]), cam)) + s[j].radius) break;
      ins++;
    }
    memmove(&s[ins + 1], &s[ins], sizeof(oracle_sphere) * (count - ins));
    s[ins] = tmp[i];
    count++;
  }
  free(tmp);
}

/* AddSphere, SphereWorld.cpp:177-190: push, drop every sphere contained in
 * another one, then re-sort.  Returns the new count (capacity must be >= n+1). */
int oracle_add_sphere(oracle_sphere* s, int n, oracle_sphere add, const float cam_pos[3]) {
  s[n++] = add;
  for (int i = 0; i < n; i++) {
    for (int j = 0; j < n; j++) {
      if (i != j &&
          vlength(vsub(sphere_pos(&s[i]), sphere_pos(&s[j]))) + s[i].radius <= s[j].radius) {
        memmove(&s[i], &s[i + 1], sizeof(oracle_sphere) * (n - i - 1));
        n--;
        i--;
        break;
      }
    }
  }
  oracle_sort_spheres(s, n, cam_pos);
  return n;
}

/* cam.fovH *= PI / 180.0f  (SphereWorld.cpp:72-73) */
float oracle_deg2rad(float deg) { return deg * (O_PI / 180.0f); }

uint64_t oracle_fnv1a64(const uint8_t* p, size_t n) {
  uint64_t h = 0xcbf29ce484222325ULL;
  for (size_t k = 0; k < n; k++) {
    h ^= p[k];
    h *= 0x100000001b3ULL;
  }
  return h;
}
