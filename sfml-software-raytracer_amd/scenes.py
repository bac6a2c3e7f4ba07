"""Pinned scene fixtures for the sphere-cave path (host side, no compute).

The reference builds its scene from ``srand(time(NULL))`` + ``rand()``
(/root/reference/Raytracing/SphereWorld.cpp:45,59-62), so it is not
reproducible; SURVEY.md section 8(d) pins explicit scenes instead and this
module states them:

* ``one_sphere``  -- config 1: one sphere {0,0,0,r=4} (SphereWorld.cpp:59).
* ``default10``   -- config 2: the 10 spheres the survey's glibc ``srand(0)``
  run produced, already in ``UpdateSpheres`` order.
* ``lcg64``       -- config 3: {0,0,0,4} + 63 spheres from an MSVC-style LCG
  (seed 12345, fields x, y, z, radius in that order, no containment pruning),
  then the ``UpdateSpheres`` sort (SphereWorld.cpp:199-212).

All arithmetic that feeds the renderer is IEEE binary32 (numpy float32), in
the reference's expression order.
"""
from __future__ import annotations

from dataclasses import dataclass, field
import os

import numpy as np

F = np.float32
PI = F(3.1415926535)  # SphereWorld.h:6

HERE = os.path.dirname(os.path.abspath(__file__))
FLOOR_PATH = os.path.join(HERE, "assets", "floor_128x128.rgba")


def deg2rad(deg: float) -> np.float32:
    """``cam.fovH *= PI / 180.0f`` (SphereWorld.cpp:72-73), in float32."""
    return F(F(deg) * F(PI / F(180.0)))


FOV_H = deg2rad(75.0)  # Camera::fovH default, SphereWorld.h:14
FOV_V = deg2rad(47.0)  # Camera::fovV default, SphereWorld.h:15


@dataclass
class Scene:
    name: str
    spheres: np.ndarray  # (n, 4) float32: x, y, z, radius in UpdateSpheres order
    cam_pos: tuple = (0.0, 0.0, 0.0)
    rotation: float = 0.0
    hrotation: float = 0.0
    fov_h: np.float32 = field(default_factory=lambda: FOV_H)
    fov_v: np.float32 = field(default_factory=lambda: FOV_V)

    def posed(self, rotation: float, hrotation: float) -> "Scene":
        return Scene(self.name, self.spheres, self.cam_pos, float(F(rotation)),
                     float(F(hrotation)), self.fov_h, self.fov_v)


def vlength(v: np.ndarray) -> np.float32:
    """``sqrtf(x*x + y*y + z*z)`` left to right (SphereWorld.cpp:340-343)."""
    x, y, z = (F(c) for c in v)
    return F(np.sqrt(F(F(F(x * x) + F(y * y)) + F(z * z))))


def sort_spheres(spheres: np.ndarray, cam_pos=(0.0, 0.0, 0.0)) -> np.ndarray:
    """Stable insertion sort by |c - cam| + r (SphereWorld.cpp:199-212)."""
    cam = np.asarray(cam_pos, dtype=F)
    out: list = []
    keys: list = []
    for s in np.asarray(spheres, dtype=F):
        key = F(vlength(s[:3] - cam) + s[3])
        ins = 0
        for k in keys:
            if key < k:
                break
            ins += 1
        out.insert(ins, s.copy())
        keys.insert(ins, key)
    return np.array(out, dtype=F).reshape(-1, 4)


def one_sphere() -> Scene:
    return Scene("one_sphere", np.array([[0, 0, 0, 4]], dtype=F))


# SURVEY.md section 8(d), config 2 (post-sort order, camera at the origin).
_DEFAULT10 = [
    (5, 2, -4, 3), (6, -3, -4, 2), (-1, 2, -2, 7), (-3, 4, 8, 2), (-7, -3, 0, 4),
    (2, 1, 5, 7), (-8, 4, 5, 3), (-8, -4, 6, 3), (-4, -2, 9, 4), (-3, -3, -9, 5),
]


def default10() -> Scene:
    return Scene("default10", np.array(_DEFAULT10, dtype=F))


def msvc_rand(state: int) -> tuple[int, int]:
    """MSVC ``rand()``: s = s*214013 + 2531011 (mod 2^32); r = (s >> 16) & 0x7fff."""
    state = (state * 214013 + 2531011) & 0xFFFFFFFF
    return state, (state >> 16) & 0x7FFF


def lcg_spheres(count: int = 63, seed: int = 12345) -> np.ndarray:
    s = seed
    rows = [(0.0, 0.0, 0.0, 4.0)]
    for _ in range(count):
        s, r = msvc_rand(s); x = r % 40 - 20
        s, r = msvc_rand(s); y = r % 10 - 5
        s, r = msvc_rand(s); z = r % 40 - 20
        s, r = msvc_rand(s); rad = r % 6 + 2
        rows.append((x, y, z, rad))
    return np.array(rows, dtype=F)


def lcg64() -> Scene:
    return Scene("lcg64", sort_spheres(lcg_spheres()))


def lcg256() -> Scene:
    """Beyond the reference's scenes (11 spheres, SphereWorld.cpp:59-62; AddSphere grows the
    list, :177-190): {0,0,0,4} + 255 spheres of the same LCG stream as lcg64 (its first 63
    are lcg64's), sorted.  Exercises the n > 64 kernel."""
    return Scene("lcg256", sort_spheres(lcg_spheres(count=255)))


SCENES = {"one_sphere": one_sphere, "default10": default10, "lcg64": lcg64, "lcg256": lcg256}


def load_floor() -> tuple[np.ndarray, int, int]:
    """Floor.png (textures[0], SphereWorld.cpp:52) decoded to RGBA8 by tools/make_assets.py."""
    data = np.fromfile(FLOOR_PATH, dtype=np.uint8)
    if data.size != 128 * 128 * 4:
        raise RuntimeError(f"{FLOOR_PATH}: expected 65536 bytes, got {data.size}")
    return data, 128, 128


# SURVEY 8d config 3, "all textures": every texture the reference ships, one slot each
# (slot 0 = Floor.png = textures[0]); the extension samples slot (i % 6) for the
# sphere at sorted position i.  Decoded RGBA8 assets (tools/make_assets.py).
ALL_TEXTURES = ["floor_128x128", "Wall", "Ceiling", "Block", "dynamic", "Projectile"]


def load_all_textures() -> list:
    out = []
    for name in ALL_TEXTURES:
        if name == "floor_128x128":
            out.append(load_floor())
            continue
        path = os.path.join(HERE, "assets", f"{name}.rgba")
        with open(path + ".shape") as f:
            w, h = (int(v) for v in f.read().split())
        data = np.fromfile(path, dtype=np.uint8)
        if data.size != w * h * 4:
            raise RuntimeError(f"{path}: expected {w * h * 4} bytes, got {data.size}")
        out.append((data, w, h))
    return out


def all_texture_slots(n: int) -> np.ndarray:
    return (np.arange(n) % len(ALL_TEXTURES)).astype(np.int32)


# Workloads named by BASELINE.json's configs; (width, height, scene, poses).
CONFIGS = {
    "c1_320x240_one_sphere": (320, 240, "one_sphere", [(0.0, 0.0)]),
    "c2_1920x1080_default10": (1920, 1080, "default10", [(0.0, 0.0), (0.7, 0.3)]),
    "c3_3840x2160_lcg64": (3840, 2160, "lcg64", [(0.0, 0.0), (1.1, -0.2)]),
    "c3_3840x2160_default10": (3840, 2160, "default10", [(0.0, 0.0)]),
    "c4_7680x4320_default10": (7680, 4320, "default10", [(0.0, 0.0)]),
    "c4_7680x4320_lcg64": (7680, 4320, "lcg64", [(0.0, 0.0)]),
    "c5_16384x16384_default10": (16384, 16384, "default10", [(0.0, 0.0)]),
    "c5_16384x16384_lcg64": (16384, 16384, "lcg64", [(0.0, 0.0)]),
    # bench.py --gpus N's weak-scaling frame (3840 x 2160*N, 64 spheres) at N = 2, 4, 8: the
    # gathered headline frames of the driver's SCALE run, pinned like the configs above
    "w2_3840x4320_lcg64": (3840, 4320, "lcg64", [(0.0, 0.0)]),
    "w4_3840x8640_lcg64": (3840, 8640, "lcg64", [(0.0, 0.0)]),
    "w8_3840x17280_lcg64": (3840, 17280, "lcg64", [(0.0, 0.0)]),
    # beyond the reference's scene sizes: the n > 64 kernel's bench line (bench.py also)
    "x_3840x2160_lcg256": (3840, 2160, "lcg256", [(0.0, 0.0)]),
}


def golden_key(width: int, height: int, scene: str, pose=(0.0, 0.0)):
    """The tests/golden/golden.json "frames" key of a (frame size, scene, pose), or None."""
    for cfg, (w, h, s, poses) in CONFIGS.items():
        if (w, h, s) == (width, height, scene) and tuple(pose) in poses:
            return f"{cfg}@{pose[0]:g},{pose[1]:g}"
    return None

# FNV-1a-64 frame hashes the survey recorded from the unmodified reference TU
# (BASELINE.md).  Key: (config, pose).
SURVEY_HASHES = {
    ("c1_320x240_one_sphere", (0.0, 0.0)): "ae94525773d7b353",
    ("c2_1920x1080_default10", (0.0, 0.0)): "9b2bc61650210880",
    ("c3_3840x2160_default10", (0.0, 0.0)): "ef7c2dc3d58a86fc",
    ("c3_3840x2160_lcg64", (0.0, 0.0)): "709972509f1cfd7c",
    ("c3_3840x2160_lcg64", (1.1, -0.2)): "514f78106d360502",
    ("c4_7680x4320_default10", (0.0, 0.0)): "a527cedb73ea6066",
    ("c4_7680x4320_lcg64", (0.0, 0.0)): "2156280e786afa03",
    ("c5_16384x16384_default10", (0.0, 0.0)): "75df2beff065426b",
}


def fnv1a64(buf) -> str:
    """FNV-1a-64 over bytes (numpy-vectorised over 8-way interleaved lanes is
    not equivalent, so this is the plain serial definition on a uint8 view)."""
    b = np.ascontiguousarray(np.asarray(buf, dtype=np.uint8)).ravel()
    h = 0xCBF29CE484222325
    for v in b.tobytes():
        h = ((h ^ v) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"
