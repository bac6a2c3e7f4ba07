"""Pinned voxel-world snapshots for the World renderer.

The reference's voxel world (/root/reference/Raytracing/World.cpp) builds a
100x10x100 block map in its constructor (:6-32), 128 lamps (a Light + an unlit
Dynamic each) and 5 sprite Dynamics with rand() directions (:47-53), then
changes light positions, sprite lighting, the `dyn` order and the active light
list `alights` every frame in UpdateDyn (:180-241).  The frame fill reads only
a snapshot of that state, so this module builds one deterministically: the
constructor's layout, sprites standing still (dir = 0 instead of rand()), and
two UpdateDyn passes (the first puts the lamps' lights at their lamps and
selects `alights`, the second lights the sprites from them), in binary32 with
the host libm's sinf/cosf/atan2f/sqrtf, as the reference does.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import os
from dataclasses import dataclass

import numpy as np

F = np.float32
EMPTY = -32768
PI = F(3.1415926535)   # World.h:5
PI2 = F(6.28318530718)  # World.h:6
HERE = os.path.dirname(os.path.abspath(__file__))
ASSETS = os.path.join(HERE, "assets")

_libm = ctypes.CDLL(ctypes.util.find_library("m"))
for _n in ("sinf", "cosf", "sqrtf"):
    getattr(_libm, _n).argtypes = [ctypes.c_float]
    getattr(_libm, _n).restype = ctypes.c_float
_libm.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
_libm.atan2f.restype = ctypes.c_float


def sinf(x):
    return F(_libm.sinf(float(x)))


def cosf(x):
    return F(_libm.cosf(float(x)))


def sqrtf(x):
    return F(_libm.sqrtf(float(x)))


def atan2f(y, x):
    return F(_libm.atan2f(float(y), float(x)))


def deg2rad(deg):
    return F(F(deg) * F(PI / F(180.0)))


@dataclass
class VoxelScene:
    blocks: np.ndarray        # int16 [nx, ny, nz], textureID or EMPTY
    dyn: np.ndarray           # structured, list order (Dynamic fields Raycast reads)
    lights: np.ndarray        # structured, `alights` order
    cam_pos: tuple
    rotation: float = 0.0
    hrotation: float = 0.0
    fov_h: np.float32 = deg2rad(75)    # Camera::fovH (World.h:13) after World.cpp:55
    fov_v: np.float32 = deg2rad(47)
    shadow_distance: float = 16.0      # World.h:70
    view_distance: float = 24.0        # World.h:71


DYN_DTYPE = np.dtype([("pos", "<f4", 3), ("size", "<f4", 2), ("r", "<f4"), ("g", "<f4"),
                      ("b", "<f4"), ("dist_to_camera", "<f4"), ("texture_id", "<i4")])
LIGHT_DTYPE = np.dtype([("pos", "<f4", 3), ("intensity", "<f4"), ("r", "<f4"), ("g", "<f4"),
                        ("b", "<f4"), ("shadows", "<i4")])


def default_blocks() -> np.ndarray:
    """Block map of World::World (World.cpp:6-32)."""
    b = np.full((100, 10, 100), EMPTY, dtype=np.int16)
    x = np.arange(100)[:, None, None]
    y = np.arange(10)[None, :, None]
    z = np.arange(100)[None, None, :]
    floor = np.broadcast_to(y == 0, b.shape)
    wall = np.broadcast_to(((x == 0) | (x == 99) | (z == 0) | (z == 99)) | ((x % 9 == 0) & (z % 5 == 0)), b.shape)
    block = np.broadcast_to((y == 4) & (x % 3 != 0) & (z % 4 != 0), b.shape)
    ceiling = np.broadcast_to(y == 9, b.shape)
    # the constructor's if/else chain gives floor > wall > block > ceiling; later
    # assignments here win, so apply them in reverse precedence
    b[ceiling] = 2
    b[block] = 3
    b[wall] = 0
    b[floor] = 1
    return b


def _lamps():
    """Lamp cells of World::World (World.cpp:17-29), in construction order."""
    out = []
    for x in range(100):
        for y in range(10):
            for z in range(100):
                if y == 0:
                    continue
                if (x == 0 or x == 99 or z == 0 or z == 99) or (x % 9 == 0 and z % 5 == 0):
                    continue
                if y == 4 and x % 3 != 0 and z % 4 != 0:
                    continue
                if y == 9:
                    continue
                if (y == 2 or y == 6) and (x % 11 == 0 and z % 11 == 0):
                    out.append((x, y, z))
    return out


def _vangle_xz(a, b):
    ang = F(atan2f(b[2], b[0]) - atan2f(a[2], a[0]))
    return F(ang - PI2) if ang > PI else (F(ang + PI2) if ang < -PI else ang)


def _normalize_xz(v):
    l = sqrtf(F(F(v[0] * v[0]) + F(v[2] * v[2])))
    return np.array([F(v[0] / l), F(v[1] / l), F(v[2] / l)], dtype=F)


def default_world(cam_pos=(15.5, 1.9, 15.5), rotation=0.0, hrotation=0.0) -> VoxelScene:
    """World::World + two UpdateDyn passes, sprites at rest."""
    cam = np.array(cam_pos, dtype=F)
    rotation, hrotation = F(rotation), F(hrotation)
    view_distance = F(24.0)
    lights = []   # dicts: pos, intensity, r, g, b, shadows
    dyn = []      # dicts: pos, size, r, g, b, dist, tex, unlit, dlight
    for (x, y, z) in _lamps():
        lights.append({"pos": np.array([17.5, 2.0, 17.5], F), "intensity": F(2), "r": F(1),
                       "g": F(1), "b": F(1), "shadows": 1})           # Light defaults, World.h:40-47
        dyn.append({"pos": np.array([F(x) + F(0.5), F(y) + F(0.5), F(z) + F(0.5)], F),
                    "size": np.array([0.01, 0.03], F), "r": F(1), "g": F(1), "b": F(1),
                    "dist": F(1000), "tex": 1, "unlit": True, "dlight": len(lights) - 1})
    for i in range(5):                                                  # World.cpp:47-53
        dyn.append({"pos": np.array([F(12.5) + F(F(i) * F(0.2)), 1.45, 18.5], F),
                    "size": np.array([0.15, 0.45], F), "r": F(1), "g": F(1), "b": F(1),
                    "dist": F(1000), "tex": 0, "unlit": False, "dlight": -1})
    alights = []
    for _ in range(2):                                                  # UpdateDyn, World.cpp:180-241
        for d in dyn:
            if d["dlight"] >= 0:
                lights[d["dlight"]]["pos"] = d["pos"].copy()
        for i, d in enumerate(dyn):
            if not d["unlit"]:
                d["r"] = d["g"] = d["b"] = F(0)
                for L in alights:
                    if L["intensity"] > 0:
                        v = d["pos"] - L["pos"]
                        dist = F(F(F(v[0] * v[0]) + F(v[1] * v[1])) + F(v[2] * v[2]))
                        dist = dist if not (dist < F(1)) else F(1)
                        add = F(F(L["intensity"] / dist) - F(dist * F(0.001)))
                        if add > 0:
                            d["r"] = F(d["r"] + F(add * L["r"]))
                            d["g"] = F(d["g"] + F(add * L["g"]))
                            d["b"] = F(d["b"] + F(add * L["b"]))
            to = d["pos"] - cam
            d["dist"] = sqrtf(F(F(to[0] * to[0]) + F(to[2] * to[2])))
            if i > 0 and d["dist"] < dyn[i - 1]["dist"]:
                dyn[i], dyn[i - 1] = dyn[i - 1], dyn[i]
        alights = []
        fwd = np.array([sinf(rotation), 0, cosf(rotation)], F)
        for L in lights:
            ad = F(F(view_distance * view_distance) * F(1.5))
            ang = abs(_vangle_xz(_normalize_xz(L["pos"] - cam), fwd))
            v = L["pos"] - cam
            ls = F(F(F(v[0] * v[0]) + F(v[1] * v[1])) + F(v[2] * v[2]))
            if ls < F(ad - F(F(F(ang / PI) * ad) * F(0.7))):
                alights.append(L)
    dyn_arr = np.zeros(len(dyn), dtype=DYN_DTYPE)
    for k, d in enumerate(dyn):
        dyn_arr[k] = (d["pos"], d["size"], d["r"], d["g"], d["b"], d["dist"], d["tex"])
    light_arr = np.zeros(len(alights), dtype=LIGHT_DTYPE)
    for k, L in enumerate(alights):
        light_arr[k] = (L["pos"], L["intensity"], L["r"], L["g"], L["b"], L["shadows"])
    return VoxelScene(default_blocks(), dyn_arr, light_arr, tuple(float(c) for c in cam),
                      float(rotation), float(hrotation))


def random_world(seed: int) -> tuple[VoxelScene, int, int]:
    """Stress snapshot (tests only): a random block grid of random size (textures 0-3 and colours
    -1..-5, some with floor and border walls), the camera in an empty cell with random turn and
    tilt, 0-10 billboards near it in list order by distance, 0-12 lights with and without
    shadows, random view and shadow distances.  Returns (scene, width, height)."""
    rng = np.random.default_rng(seed)
    nx, ny, nz = int(rng.integers(8, 49)), int(rng.integers(4, 13)), int(rng.integers(8, 49))
    b = np.full((nx, ny, nz), EMPTY, dtype=np.int16)
    ids = np.array([0, 1, 2, 3, -1, -2, -3, -4, -5], dtype=np.int16)
    fill = rng.random(b.shape) < rng.uniform(0.02, 0.15)
    b[fill] = rng.choice(ids, size=int(fill.sum()))
    if rng.random() < 0.7:
        b[:, 0, :] = rng.choice(ids)
    if rng.random() < 0.5:
        wall = rng.choice(ids)
        b[0, :, :] = b[-1, :, :] = b[:, :, 0] = b[:, :, -1] = wall
    while True:  # the camera in an empty interior cell
        c = (int(rng.integers(1, nx - 1)), int(rng.integers(1, ny - 1)), int(rng.integers(1, nz - 1)))
        if b[c] == EMPTY:
            break
    cam = np.array([F(c[k] + rng.uniform(0.05, 0.95)) for k in range(3)], F)
    rotation, hrotation = F(rng.uniform(0, 2 * np.pi)), F(rng.uniform(-0.6, 0.6))
    dyn = np.zeros(int(rng.integers(0, 11)), dtype=DYN_DTYPE)
    for d in dyn:
        off = rng.uniform(1.0, 8.0) * np.array([np.sin(a := rng.uniform(0, 2 * np.pi)), 0, np.cos(a)])
        pos = np.array([cam[0] + off[0], rng.uniform(0.3, ny - 0.7), cam[2] + off[2]], F)
        to = pos - cam
        d["pos"], d["size"] = pos, (rng.uniform(0.05, 0.5), rng.uniform(0.1, 0.8))
        d["r"], d["g"], d["b"] = rng.uniform(0, 2, 3).astype(F)
        d["dist_to_camera"] = sqrtf(F(F(to[0] * to[0]) + F(to[2] * to[2])))
        d["texture_id"] = int(rng.integers(0, 2))
    dyn = dyn[np.argsort(dyn["dist_to_camera"], kind="stable")]
    lights = np.zeros(int(rng.integers(0, 13)), dtype=LIGHT_DTYPE)
    for L in lights:
        if rng.random() < 0.5:  # near the camera
            L["pos"] = np.clip(cam + rng.uniform(-6, 6, 3).astype(F), 0.2, [nx - 0.2, ny - 0.2, nz - 0.2])
        else:
            L["pos"] = (rng.uniform(0, nx), rng.uniform(0.2, ny - 0.2), rng.uniform(0, nz))
        L["intensity"] = rng.uniform(1.0, 12.0)
        L["r"], L["g"], L["b"] = rng.uniform(0.2, 1.0, 3).astype(F)
        L["shadows"] = int(rng.random() < 0.6)
    scene = VoxelScene(b, dyn, lights, tuple(float(v) for v in cam), float(rotation),
                       float(hrotation), shadow_distance=float(rng.choice([8.0, 16.0])),
                       view_distance=float(rng.choice([12.0, 24.0, 40.0])))
    w, h = [(320, 180), (256, 144), (333, 187)][seed % 3]
    return scene, w, h


def load_textures():
    """textures[0..3] and dynTextures[0..1] (World.cpp:40-45), decoded RGBA8."""
    names = ["Wall", "Floor", "Ceiling", "Block"]
    tex = []
    for n in names:
        tex.append(_load_asset(n))
    dyn = [_load_asset("dynamic"), _load_asset("Projectile")]
    return tex, dyn


def _load_asset(name):
    raw = os.path.join(ASSETS, f"{name}.rgba")
    with open(raw + ".shape") as f:
        w, h = (int(v) for v in f.read().split())
    data = np.fromfile(raw, dtype=np.uint8)
    assert data.size == w * h * 4, name
    return data, w, h


COLORS = np.array([[0, 0, 0, 255], [100, 100, 100, 255], [200, 200, 200, 255], [200, 0, 0, 255],
                   [0, 200, 0, 255], [0, 0, 200, 255]] + [[0, 0, 0, 0]] * 4, dtype=np.uint8)  # World.cpp:34-39
