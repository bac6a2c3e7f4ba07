"""Uniform snapshots for the GLSL renderer.

rayShader.frag reads nothing but its uniforms and the `ground` texture.  The
reference uploads them from SphereWorld::UpdateSpheres (every AddSphere /
AddLight call and every frame, /root/reference/Raytracing/SphereWorld.cpp:
199-238) and from main() (campos, rotation, fov, size; Source.cpp:143-146).
The upload is history dependent: `uvs[k]` and `lights[k]` keep whatever an
earlier UpdateSpheres call wrote when the current lists no longer cover k
(e.g. the light's `uvs` slot still holds osphere 0's (0.5, 1, 0.5, 0) from
before the light was added).  ``ShaderWorld`` replays that sequence:

* the constructor (SphereWorld.cpp:43-70) with glibc's ``rand`` after
  ``srand(seed)`` -- the survey's default10 scene is seed 0, and the replay
  reproduces it (``rand()`` arguments evaluate right to left, as g++ does);
* ``update_world`` -- the osphere part of SphereWorld::UpdateWorld
  (SphereWorld.cpp:119-146), so animated frames follow the same stream;
  camera physics (Move, :241-306) is not replayed: the camera stays put;
* ``uniforms`` -- the block main() completes before ``rt.draw``.

All arithmetic that feeds the uniforms is binary32 (numpy float32) in the
reference's expression order.  No compute happens here.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from scenes import FOV_H, FOV_V, vlength

F = np.float32
MAX_SPHERES = 100  # uniform vec4 spheres[100] (rayShader.frag:6-8)

# sfrt_glsl_uniforms (include/sfrt.h), field for field.
UNIFORM_DTYPE = np.dtype([
    ("campos", "<f4", 3), ("rotation", "<f4", 2), ("fov", "<f4", 2), ("size", "<f4", 2),
    ("sphere_count", "<i4"), ("all_spheres_count", "<i4"), ("light_count", "<i4"),
    ("spheres", "<f4", (MAX_SPHERES, 4)), ("uvs", "<f4", (MAX_SPHERES, 4)),
    ("lights", "<f4", (MAX_SPHERES, 4)),
])


class GlibcRand:
    """glibc ``random()`` TYPE_3 (x^31 + x^3 + 1 additive feedback), as ``rand()``."""

    def __init__(self, seed: int = 0):
        r = [0] * 34
        r[0] = seed & 0xFFFFFFFF or 1
        if r[0] >= 1 << 31:
            r[0] -= 1 << 32
        for i in range(1, 31):
            hi, lo = divmod(r[i - 1], 127773) if r[i - 1] >= 0 else (
                -((-r[i - 1]) // 127773), -((-r[i - 1]) % 127773))
            w = 16807 * lo - 2836 * hi
            if w < 0:
                w += 2147483647
            r[i] = w
        for i in range(31, 34):
            r[i] = r[i - 31]
        r = [v & 0xFFFFFFFF for v in r]
        for i in range(34, 344):
            r.append((r[i - 31] + r[i - 3]) & 0xFFFFFFFF)
        self._r = r[-34:]

    def __call__(self) -> int:
        r = self._r
        v = (r[-31] + r[-3]) & 0xFFFFFFFF
        r.append(v)
        del r[0]
        return v >> 1


@dataclass
class Ball:
    """struct Sphere (SphereWorld.h:23-29)."""
    pos: np.ndarray
    radius: np.float32
    light: np.ndarray = field(default_factory=lambda: np.zeros(4, F))
    move: np.ndarray = field(default_factory=lambda: np.zeros(3, F))
    move_target: np.ndarray = field(default_factory=lambda: np.zeros(3, F))


def _v3(x, y, z) -> np.ndarray:
    return np.array([x, y, z], dtype=F)


def _normalize(v: np.ndarray) -> np.ndarray:
    """SphereWorld::VNormalize (SphereWorld.cpp:330-333)."""
    l = vlength(v)
    return np.array([F(v[0] / l), F(v[1] / l), F(v[2] / l)], dtype=F)


class ShaderWorld:
    """The part of SphereWorld that feeds rayShader.frag."""

    def __init__(self, seed: int = 0, cam_pos=(0.0, 0.0, 0.0)):
        self.rand = GlibcRand(seed)
        self.cam_pos = _v3(*cam_pos)
        self.spheres: list[Ball] = []
        self.ospheres: list[Ball] = []
        self.lights: list[Ball] = []
        self.u = np.zeros((), dtype=UNIFORM_DTYPE)
        rand = self.rand
        # SphereWorld.cpp:59-70
        self.add_sphere(_v3(0, 0, 0), F(4))
        for _ in range(10):
            r = F(rand() % 6 + 2)          # arguments evaluate right to left
            z = F(rand() % 20 - 10)
            y = F(rand() % 10 - 5)
            x = F(rand() % 20 - 10)
            self.add_sphere(_v3(x, y, z), r)
        for i in range(10):
            r = F(F(rand() % 2 + 1) * F(0.3))
            self.add_light(_v3(F(F(i) * F(1.2)), 1, 1), r, np.array([0.5, 1, 1, 1], F), True)
        self.add_light(_v3(0, -1, 1), F(0.2), np.array([1, 1, 1, 1], F), False)

    # --- SphereWorld.cpp:177-197 ---
    def add_sphere(self, pos, radius) -> None:
        self.spheres.append(Ball(pos.astype(F), F(radius)))
        i = 0
        while i < len(self.spheres):
            for j in range(len(self.spheres)):
                si, sj = self.spheres[i], self.spheres[j]
                if i != j and F(vlength(si.pos - sj.pos) + si.radius) <= sj.radius:
                    del self.spheres[i]
                    i -= 1
                    break
            i += 1
        self.update_spheres()

    def add_light(self, pos, radius, color, notlight: bool) -> None:
        (self.ospheres if notlight else self.lights).append(
            Ball(pos.astype(F), F(radius), np.asarray(color, F).copy()))
        self.update_spheres()

    # --- SphereWorld.cpp:199-238 ---
    def update_spheres(self, onlyo: bool = False) -> None:
        out: list[Ball] = []
        keys: list = []
        for s in self.spheres:
            key = F(vlength(s.pos - self.cam_pos) + s.radius)
            ins = 0
            for k in keys:
                if key < k:
                    break
                ins += 1
            out.insert(ins, s)
            keys.insert(ins, key)
        self.spheres = out
        u = self.u
        ns, nl = len(self.spheres), len(self.lights)
        if not onlyo:
            for i, s in enumerate(self.spheres):
                u["spheres"][i] = (*s.pos, s.radius)
                u["lights"][i] = 0
                u["uvs"][i] = (0.5, 0.0, 0.0, 0.0)
            for i, L in enumerate(self.lights):
                u["spheres"][i + ns] = (*L.pos, L.radius)
                u["lights"][i + ns] = (*L.light[:3], 1.0)
        for i, o in enumerate(self.ospheres):
            u["spheres"][i + ns + nl] = (*o.pos, o.radius)
            u["lights"][i + ns + nl] = o.light
            u["uvs"][i + ns + nl] = (0.5, 1.0, 0.5, 0.0)
        u["light_count"] = nl
        u["sphere_count"] = ns
        u["all_spheres_count"] = nl + ns + len(self.ospheres)

    # --- SphereWorld.cpp:119-146 (osphere motion; the camera is not moved) ---
    def update_world(self) -> None:
        rand = self.rand
        for o in self.ospheres:
            o.pos = (o.pos + o.move * F(0.01)).astype(F)
            o.move = (F(0.99) * o.move + F(0.01) * o.move_target).astype(F)
            if rand() % 100 == 0:
                z = F(rand() % 3 - 1)
                y = F(rand() % 3 - 1)
                x = F(rand() % 3 - 1)
                o.move_target = _v3(x, y, z)
            isinside = False
            smallest = F(9999)
            index = 0
            for j, s in enumerate(self.spheres):
                dist = F(vlength(o.pos - s.pos) + o.radius)
                if dist < s.radius:
                    isinside = True
                    break
                elif F(s.radius - dist) < smallest:
                    smallest = F(s.radius - dist)
                    index = j
            if not isinside:
                z = F(rand() % 3 - 1)
                y = F(rand() % 3 - 1)
                x = F(rand() % 3 - 1)
                o.move = (o.move + ((self.spheres[index].pos - o.pos) + _v3(x, y, z) * F(0.5))).astype(F)
                o.move = _normalize(o.move)
        self.update_spheres()

    # --- Source.cpp:143-146 ---
    def uniforms(self, width: int = 1920, height: int = 1080, rotation=0.0, hrotation=0.0,
                 fov_h=None, fov_v=None) -> np.ndarray:
        u = self.u.copy()
        u["campos"] = self.cam_pos
        u["rotation"] = (F(rotation), F(hrotation))
        u["fov"] = (FOV_H if fov_h is None else F(fov_h), FOV_V if fov_v is None else F(fov_v))
        u["size"] = (F(width), F(height))
        return u


def default_uniforms(width=1920, height=1080, rotation=0.0, hrotation=0.0, frames=0, seed=0):
    """The constructor's world (srand(seed)) after `frames` UpdateWorld calls."""
    w = ShaderWorld(seed)
    for _ in range(frames):
        w.update_world()
    return w.uniforms(width, height, rotation, hrotation)


def random_uniforms(seed: int, n_walls: int, n_lights: int, n_balls: int, width=320, height=180):
    """Stress block: random walls around the origin, lights and balls inside,
    none of them containing the camera."""
    rng = np.random.default_rng(seed)
    u = np.zeros((), dtype=UNIFORM_DTYPE)
    cam = rng.uniform(-1, 1, 3)

    def place(lo, hi, rlo, rhi):
        while True:
            c, r = rng.uniform(lo, hi, 3), rng.uniform(rlo, rhi)
            if np.linalg.norm(c - cam) > r + 0.3:
                return c, r

    walls = [(0.0, 0.0, 0.0, 6.0)] + [
        (*rng.uniform(-6, 6, 3), rng.uniform(2, 7)) for _ in range(n_walls - 1)]
    k = 0
    for s in walls:
        u["spheres"][k] = s
        u["uvs"][k] = (0.5, 0, 0, 0)
        k += 1
    for _ in range(n_lights):
        c, r = place(-2, 2, 0.1, 0.4)
        u["spheres"][k] = (*c, r)
        u["lights"][k] = (*rng.uniform(0.3, 1, 3), 1.0)
        u["uvs"][k] = (0.5, 1.0, 0.5, 0.0)
        k += 1
    for _ in range(n_balls):
        c, r = place(-3, 3, 0.2, 0.8)
        u["spheres"][k] = (*c, r)
        u["lights"][k] = (*rng.uniform(0, 1, 3), rng.uniform(0, 1))
        u["uvs"][k] = (0.5, 1.0, 0.5, 0.0)
        k += 1
    u["sphere_count"], u["light_count"], u["all_spheres_count"] = n_walls, n_lights, k
    u["campos"] = cam
    u["rotation"] = (rng.uniform(0, 6.28), rng.uniform(-0.6, 0.6))
    u["fov"] = (FOV_H, FOV_V)
    u["size"] = (width, height)
    return u
