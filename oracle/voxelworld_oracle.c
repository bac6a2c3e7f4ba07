/*
 * voxelworld_oracle.c -- CPU restatement of the reference's voxel World
 * frame fill.
 *
 *   TEST INFRASTRUCTURE ONLY: the parity checker for libsfrt.so's voxel
 *   kernel.  The product never links, calls or falls back to it.
 *
 * Restates (paths relative to /root/reference/Raytracing/):
 *   World::UpdateImage   World.cpp:62-87    (ovox_update_image)
 *   World::Raycast       World.cpp:302-453  (raycast)
 *   World::LRaycast      World.cpp:455-491  (lraycast)
 *   World::VAngleXZ      World.cpp:271-275, VNormalizeXZ :282-285, VLength* :287-300
 * Arithmetic is binary32 in the reference's expression order, compiled with
 * -ffp-contract=off; sinf/cosf/atan2f are the host libm's, as the reference's
 * std::sin/std::cos/std::atan2 calls.  The scene is a snapshot: the dense
 * block grid stands for the `blocks` unordered_map (World.cpp:6-32) with the
 * same key semantics, `dyn` and `alights` are passed in list order.
 *
 * Pinning: World.cpp needs SFML (absent) and stand-in headers are not allowed,
 * so it is not built here; it ships no tests.  The survey's single World hash
 * (8a3a61d6af69ddca, its own stub and unrecorded world state) cannot be
 * reproduced.  Parity for this row is therefore UNPINNED against the
 * original build: the GPU kernel is held bit-exact to this restatement.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "voxelworld_oracle.h"

#define O_PI 3.1415926535f   /* World.h:5 */
#define O_PI2 6.28318530718f /* World.h:6 */

typedef struct { float x, y, z; } v3;
static v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }

/* float -> sf::Uint8 as x86-64 g++ converts (cvttss2si to int, low byte). */
static uint8_t to_u8(float f) {
  if (!(f > -2147483648.0f && f < 2147483648.0f)) return 0; /* x86: 0x80000000 -> low byte 0 */
  return (uint8_t)(int32_t)f;
}
/* float -> int (x86 cvttss2si; out of range and NaN give INT_MIN). */
static int32_t to_i32(float f) {
  if (!(f > -2147483648.0f && f < 2147483648.0f)) return INT32_MIN;
  return (int32_t)f;
}
/* float -> unsigned (x86-64: cvttss2si to 64 bits, low 32). */
static uint32_t to_u32(float f) {
  if (!(f > -9.2233720368547758e18f && f < 9.2233720368547758e18f)) return 0;
  return (uint32_t)(int64_t)f;
}

/* blocks.contains((x << 20) + (y << 10) + z) (World.cpp:246,337): the map's
 * keys are those of occupied grid cells, so a key is present iff it is
 * non-negative and decodes to an occupied cell. */
static int block_at(const ovox_scene* sc, int32_t x, int32_t y, int32_t z, int16_t* id) {
  const int32_t key = (int32_t)(((uint32_t)x << 20) + ((uint32_t)y << 10) + (uint32_t)z);
  if (key < 0) return 0;
  const int32_t cx = key >> 20, cy = (key >> 10) & 1023, cz = key & 1023;
  if (cx >= sc->nx || cy >= sc->ny || cz >= sc->nz) return 0;
  const int16_t v = sc->blocks[((size_t)cx * sc->ny + cy) * sc->nz + cz];
  if (v == OVOX_EMPTY) return 0;
  if (id) *id = v;
  return 1;
}

static long bad_texel_reads = 0;

static const uint8_t* texel(const ovox_texture* t, uint32_t x, uint32_t y) {
  const uint32_t idx = x + y * (uint32_t)t->w;
  if (!t->rgba || idx >= (uint32_t)(t->w * t->h)) {
    __atomic_add_fetch(&bad_texel_reads, 1, __ATOMIC_RELAXED); /* reference: UB read */
    static const uint8_t magenta[4] = {255, 0, 255, 255};
    return magenta;
  }
  return t->rgba + (size_t)idx * 4;
}

long ovox_bad_texel_reads(void) { return bad_texel_reads; }

/* World::VAngleXZ, World.cpp:271-275 */
static float angle_xz(v3 a, v3 b) {
  float ang = atan2f(b.z, b.x) - atan2f(a.z, a.x);
  return ang > O_PI ? ang - O_PI2 : ang < -O_PI ? ang + O_PI2 : ang;
}

/* World::LRaycast, World.cpp:455-491: free path from pos to the light? */
static int lraycast(const ovox_scene* sc, v3 pos, v3 dir, float maxDist) {
  float dist = 0;
  int32_t pix = to_i32(pos.x), piy = to_i32(pos.y), piz = to_i32(pos.z);
  const float dirxadd = dir.x > 0 ? 1.0f : 0, diryadd = dir.y > 0 ? 1.0f : 0,
              dirzadd = dir.z > 0 ? 1.0f : 0;
  const int dirxsign = dir.x > 0 ? -1 : 1, dirysign = dir.y > 0 ? -1 : 1,
            dirzsign = dir.z > 0 ? -1 : 1;
  const float dirxlen = fabsf(dir.x), dirylen = fabsf(dir.y), dirzlen = fabsf(dir.z);
  const float m2 = maxDist * 2;
  const uint32_t maxIter = to_u32(m2 < 20.0f ? 20.0f : m2);         /* :473 */
  for (uint32_t i = 0; i < maxIter && dist < maxDist; i++) {         /* :475 */
    if (block_at(sc, pix, piy, piz, NULL)) return 0;                 /* :476-478 */
    const float a = (dirxadd + (float)dirxsign * (pos.x - (float)pix)) / dirxlen;
    const float b = (diryadd + (float)dirysign * (pos.y - (float)piy)) / dirylen;
    const float c = (dirzadd + (float)dirzsign * (pos.z - (float)piz)) / dirzlen;
    float raySpeed = a; /* std::min({a, b, c}) :479-481 */
    if (b < raySpeed) raySpeed = b;
    if (c < raySpeed) raySpeed = c;
    raySpeed += 0.002f;                                               /* :482 */
    dist += raySpeed;
    pos = mk(pos.x + dir.x * raySpeed, pos.y + dir.y * raySpeed, pos.z + dir.z * raySpeed);
    pix = to_i32(pos.x); piy = to_i32(pos.y); piz = to_i32(pos.z);
  }
  return dist >= maxDist;                                             /* :490 */
}

/* std::min(v, 255.0f) == (255.0f < v) ? 255.0f : v  (NaN stays NaN) */
static float min255(float v) { return 255.0f < v ? 255.0f : v; }

static uint32_t pack(uint8_t r, uint8_t g, uint8_t b, uint8_t a) {
  return (uint32_t)r | ((uint32_t)g << 8) | ((uint32_t)b << 16) | ((uint32_t)a << 24);
}

/* World::Raycast, World.cpp:302-453, for primary direction dir and r->yscale. */
static uint32_t raycast(const ovox_scene* sc, v3 dir, float yscale) {
  const v3 cam = mk(sc->cam_pos[0], sc->cam_pos[1], sc->cam_pos[2]);
  float dist = 0;
  v3 pos = cam;
  int32_t pix = to_i32(pos.x), piy = to_i32(pos.y), piz = to_i32(pos.z);
  v3 tryPos = pos;
  const float dirxadd = dir.x > 0 ? 1.0f : 0, diryadd = dir.y > 0 ? 1.0f : 0,
              dirzadd = dir.z > 0 ? 1.0f : 0;
  int dirxsign = dir.x > 0 ? -1 : 1, dirysign = dir.y > 0 ? -1 : 1,
      dirzsign = dir.z > 0 ? -1 : 1;
  const float dirxlen = fabsf(dir.x), dirylen = fabsf(dir.y), dirzlen = fabsf(dir.z);
  uint32_t DI = 0;
  float raySpeed = 0;
  int colRay = 0;
  uint32_t i = 0;
  const uint32_t maxiter = to_u32(sc->view_distance * 1.5f);         /* :322 */

  while (dist < sc->view_distance && i < maxiter) {                   /* :324 */
    const float xray = (dirxadd + (float)dirxsign * (pos.x - (float)pix)) / dirxlen;
    const float yray = (diryadd + (float)dirysign * (pos.y - (float)piy)) / dirylen;
    const float zray = (dirzadd + (float)dirzsign * (pos.z - (float)piz)) / dirzlen;
    if (xray <= yray && xray <= zray) {                               /* :329 */
      raySpeed = xray;
      tryPos.x += dir.x * (raySpeed + 0.002f);
      tryPos.y += dir.y * raySpeed;
      tryPos.z += dir.z * raySpeed;
      colRay = 1;
    } else if (yray <= xray && yray <= zray) {                        /* :336 */
      raySpeed = yray;
      tryPos.x += dir.x * raySpeed;
      tryPos.y += dir.y * (raySpeed + 0.002f);
      tryPos.z += dir.z * raySpeed;
      colRay = 2;
    } else {                                                          /* :343 */
      raySpeed = zray;
      tryPos.x += dir.x * raySpeed;
      tryPos.y += dir.y * raySpeed;
      tryPos.z += dir.z * (raySpeed + 0.002f);
      colRay = 3;
    }
    const float tryDist = dist + raySpeed;                            /* :351 */

    /* dynamic billboards before the next block, :353-378 */
    while (DI < (uint32_t)sc->ndyn && tryDist >= sc->dyn[DI].dist_to_camera) {
      const ovox_dynamic* d = &sc->dyn[DI];
      raySpeed = d->dist_to_camera - dist;
      dist = d->dist_to_camera;
      pos = mk(pos.x + dir.x * raySpeed, pos.y + dir.y * raySpeed, pos.z + dir.z * raySpeed);
      const float to = d->pos[1] - pos.y;
      const float sizey = d->size[1] * yscale;
      if (fabsf(to) < sizey) {
        const v3 dd = mk(d->pos[0] - cam.x, d->pos[1] - cam.y, d->pos[2] - cam.z);
        const float lxz = sqrtf(dd.x * dd.x + dd.z * dd.z);          /* VNormalizeXZ */
        const v3 bn = mk(dd.x / lxz, dd.y / lxz, dd.z / lxz);
        const float ang = angle_xz(dir, bn) * dist;
        const ovox_texture* tex = &sc->dyn_textures[d->texture_id];
        const float xf = (0.5f + ang / O_PI * 0.5f / d->size[0]);
        if (xf > 0 && xf < 1) {
          int32_t x = to_i32(xf * (float)(uint32_t)tex->w);
          int32_t y = to_i32((sizey + to) / sizey / 2 * (float)(uint32_t)tex->h);
          x = x < 0 ? 0 : x;
          y = y < 0 ? 0 : y;
          const uint8_t* c = texel(tex, (uint32_t)x, (uint32_t)y);
          if (c[3] > 127) {
            float fr = c[0] * d->r, fg = c[1] * d->g, fb = c[2] * d->b;
            return pack(to_u8(min255(fr)), to_u8(min255(fg)), to_u8(min255(fb)), c[3]);
          }
        }
      }
      DI++;
    }

    dist = tryDist;                                                   /* :380 */
    pos = tryPos;
    pix = to_i32(pos.x); piy = to_i32(pos.y); piz = to_i32(pos.z);
    int16_t id;
    if (block_at(sc, pix, piy, piz, &id)) {                           /* :385 */
      uint8_t c[4];
      if (id < 0) {
        memcpy(c, sc->colors[-id], 4);
      } else {
        const ovox_texture* tex = &sc->textures[id];
        const float tw = (float)(uint32_t)tex->w, th = (float)(uint32_t)tex->h;
        if (colRay == 1) {
          memcpy(c, texel(tex, to_u32(tw * (pos.z - (float)piz)), to_u32(th * (pos.y - (float)piy))), 4);
          pos.x += (float)dirxsign * 0.01f;
          dirysign = 0;
          dirzsign = 0;
        } else if (colRay == 2) {
          memcpy(c, texel(tex, to_u32(tw * (pos.x - (float)pix)), to_u32(th * (pos.z - (float)piz))), 4);
          pos.y += (float)dirysign * 0.01f;
          dirxsign = 0;
          dirzsign = 0;
        } else {
          memcpy(c, texel(tex, to_u32(tw * (pos.x - (float)pix)), to_u32(th * (pos.y - (float)piy))), 4);
          pos.z += (float)dirzsign * 0.01f;
          dirxsign = 0;
          dirysign = 0;
        }
      }
      const float l0 = 0.05f / dist - dist * 0.0001f;                 /* :414 */
      float litr = l0 < 0.0f ? 0.0f : l0;
      float litg = litr, litb = litr;
      for (int j = 0; j < sc->nlights; j++) {                         /* :418 */
        const ovox_light* L = &sc->lights[j];
        const v3 dl = mk(pos.x - L->pos[0], pos.y - L->pos[1], pos.z - L->pos[2]);
        float dd = dl.x * dl.x + dl.y * dl.y + dl.z * dl.z;           /* VLengthS */
        float add = (L->intensity / dd - dd * 0.002f);
        if (add > 0) {
          v3 nd = mk(L->pos[0] - pos.x, L->pos[1] - pos.y, L->pos[2] - pos.z);
          add *= ((nd.x * (float)dirxsign + nd.y * (float)dirysign + nd.z * (float)dirzsign) * 0.7f + 0.3f);
          if (add > 0) {
            if (L->shadows && tryDist < sc->shadow_distance) {        /* :425 */
              dd = sqrtf(nd.x * nd.x + nd.y * nd.y + nd.z * nd.z);   /* VLength */
              nd = mk(nd.x / dd, nd.y / dd, nd.z / dd);
              if (lraycast(sc, pos, nd, dd)) {
                litr += add * L->r;
                litg += add * L->g;
                litb += add * L->b;
              }
            } else {
              litr += add * L->r;
              litg += add * L->g;
              litb += add * L->b;
            }
          }
        }
      }
      const float fr = c[0] * litr, fg = c[1] * litg, fb = c[2] * litb; /* :446 */
      return pack(to_u8(min255(fr)), to_u8(min255(fg)), to_u8(min255(fb)), c[3]);
    }
    i += 1;
  }
  return pack(0, 0, 0, 255); /* sf::Color::Black, :452 */
}

/* World::UpdateImage, World.cpp:62-87 */
void ovox_update_image(const ovox_scene* sc, uint8_t* rgba, int ystart, int yadd, int xstart,
                       int xadd) {
  const float vStart = sc->fov_v / 2;
  const float vIncreaseBy = sc->fov_v / sc->height;
  const float vOff = sinf(sc->cam_hrotation);
  const float hStart = sc->cam_rotation - sc->fov_h / 2;
  const float hIncreaseBy = sc->fov_h / sc->width;
  v3 dir = mk(0, 0, 0);
  for (int i = xstart; i < sc->width; i += xadd) {
    const float hray = (hStart + hIncreaseBy * i);
    dir.x = sinf(hray);
    dir.z = cosf(hray);
    const float fix = cosf(sc->cam_rotation - hray); /* "Fix distortion on edges" :77 */
    dir = mk(dir.x / fix, dir.y / fix, dir.z / fix);
    for (int j = ystart; j < sc->height; j += yadd) {
      const float vray = (vStart - j * vIncreaseBy);
      const float yscale = cosf(sc->cam_hrotation + vray);
      dir.y = (vOff + sinf(vray));
      const uint32_t c = raycast(sc, dir, yscale);
      memcpy(rgba + ((size_t)j * sc->width + i) * 4, &c, 4);
    }
  }
}

typedef struct {
  const ovox_scene* sc;
  uint8_t* rgba;
  int t, T;
} thread_arg;

static void* render_thread(void* p) {
  thread_arg* a = (thread_arg*)p;
  ovox_update_image(a->sc, a->rgba, a->t, a->T, 0, 1);
  return NULL;
}

void ovox_render_threaded(const ovox_scene* sc, uint8_t* rgba, int nthreads) {
  if (nthreads <= 1) {
    ovox_update_image(sc, rgba, 0, 1, 0, 1);
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
