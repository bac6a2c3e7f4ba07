"""ctypes binding of the CPU restatement -- TEST INFRASTRUCTURE ONLY.

Only tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke() import
this module, and only as the checker / CPU baseline.  The product path
(sfml-software-raytracer_amd/libsfrt.so) never calls it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")


class OracleSphere(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float),
                ("radius", ctypes.c_float)]


class OracleScene(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int), ("height", ctypes.c_int),
        ("cam_pos", ctypes.c_float * 3),
        ("cam_rotation", ctypes.c_float), ("cam_hrotation", ctypes.c_float),
        ("fov_h", ctypes.c_float), ("fov_v", ctypes.c_float),
        ("spheres", ctypes.POINTER(OracleSphere)), ("sphere_count", ctypes.c_int),
        ("texture", ctypes.POINTER(ctypes.c_uint8)),
        ("tex_w", ctypes.c_int), ("tex_h", ctypes.c_int),
        ("sphere_tex", ctypes.POINTER(ctypes.c_int32)),
        ("textures", ctypes.POINTER(ctypes.c_uint8) * 10),
        ("tex_ws", ctypes.c_int * 10), ("tex_hs", ctypes.c_int * 10),
    ]


class OraclePixelDump(ctypes.Structure):
    _fields_ = [
        ("pos", ctypes.c_float * 3), ("draw", ctypes.c_int), ("iters", ctypes.c_int),
        ("xcoord", ctypes.c_float), ("ycoord", ctypes.c_float), ("brightness", ctypes.c_float),
        ("texel", ctypes.c_uint * 2), ("rgba", ctypes.c_uint8 * 4),
    ]


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        L.oracle_update_image.argtypes = [P(OracleScene), P(ctypes.c_uint8), ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_render_band.argtypes = [P(OracleScene), P(ctypes.c_uint8), ctypes.c_int,
                                         ctypes.c_int]
        L.oracle_render_threaded.argtypes = [P(OracleScene), P(ctypes.c_uint8), ctypes.c_int]
        L.oracle_iteration_map.argtypes = [P(OracleScene), P(ctypes.c_int32), ctypes.c_int]
        L.oracle_trace_dump.argtypes = [P(OracleScene), ctypes.c_int, ctypes.c_int,
                                        P(OraclePixelDump)]
        L.oracle_sort_spheres.argtypes = [P(OracleSphere), ctypes.c_int, P(ctypes.c_float)]
        L.oracle_add_sphere.argtypes = [P(OracleSphere), ctypes.c_int, OracleSphere,
                                        P(ctypes.c_float)]
        L.oracle_add_sphere.restype = ctypes.c_int
        L.oracle_scene_valid.argtypes = [P(OracleScene)]
        L.oracle_scene_valid.restype = ctypes.c_int
        L.oracle_deg2rad.argtypes = [ctypes.c_float]
        L.oracle_deg2rad.restype = ctypes.c_float
        L.oracle_fnv1a64.argtypes = [P(ctypes.c_uint8), ctypes.c_size_t]
        L.oracle_fnv1a64.restype = ctypes.c_uint64
        _lib = L
    return _lib


class Oracle:
    """One scene + texture bound for repeated oracle calls."""

    def __init__(self, width, height, spheres, texture, tex_w, tex_h, cam_pos=(0, 0, 0),
                 rotation=0.0, hrotation=0.0, fov_h=None, fov_v=None, sphere_tex=None,
                 textures=None):
        """sphere_tex / textures: the per-sphere texture extension (slot per sphere;
        {slot: (rgba, w, h)} for slots 1..9); None = the reference (slot 0 only)."""
        sph = np.ascontiguousarray(np.asarray(spheres, dtype=np.float32).reshape(-1, 4))
        self._sph = sph
        self._tex = np.ascontiguousarray(np.asarray(texture, dtype=np.uint8).ravel())
        sc = OracleScene()
        sc.width, sc.height = int(width), int(height)
        for k in range(3):
            sc.cam_pos[k] = float(cam_pos[k])
        sc.cam_rotation, sc.cam_hrotation = float(rotation), float(hrotation)
        sc.fov_h = float(fov_h) if fov_h is not None else lib().oracle_deg2rad(75.0)
        sc.fov_v = float(fov_v) if fov_v is not None else lib().oracle_deg2rad(47.0)
        sc.spheres = sph.ctypes.data_as(ctypes.POINTER(OracleSphere))
        sc.sphere_count = sph.shape[0]
        sc.texture = self._tex.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        sc.tex_w, sc.tex_h = int(tex_w), int(tex_h)
        self._keep = []
        if sphere_tex is not None:
            st = np.ascontiguousarray(np.asarray(sphere_tex, dtype=np.int32))
            assert st.size == sph.shape[0]
            self._keep.append(st)
            sc.sphere_tex = st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        for k, (rgba, w, h) in (textures or {}).items():
            buf = np.ascontiguousarray(np.asarray(rgba, dtype=np.uint8).ravel())
            self._keep.append(buf)
            sc.textures[k] = buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
            sc.tex_ws[k], sc.tex_hs[k] = int(w), int(h)
        self.scene = sc

    @classmethod
    def from_scene(cls, scene, width, height, texture, tex_w, tex_h):
        return cls(width, height, scene.spheres, texture, tex_w, tex_h, scene.cam_pos,
                   scene.rotation, scene.hrotation, scene.fov_h, scene.fov_v)

    def render(self, threads: int = 1) -> np.ndarray:
        out = np.zeros(self.scene.width * self.scene.height * 4, dtype=np.uint8)
        lib().oracle_render_threaded(ctypes.byref(self.scene),
                                     out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                     int(threads))
        return out

    def update_image(self, out: np.ndarray, ystart, yadd, xstart, xadd) -> None:
        lib().oracle_update_image(ctypes.byref(self.scene),
                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                  ystart, yadd, xstart, xadd)

    def render_band(self, row0: int, rows: int) -> np.ndarray:
        out = np.zeros(self.scene.width * rows * 4, dtype=np.uint8)
        lib().oracle_render_band(ctypes.byref(self.scene),
                                 out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), row0, rows)
        return out

    def iteration_map(self, threads: int = 1) -> np.ndarray:
        """March iterations per pixel (trips of SphereWorld.cpp:362), row-major int32."""
        it = np.zeros(self.scene.width * self.scene.height, dtype=np.int32)
        lib().oracle_iteration_map(ctypes.byref(self.scene),
                                   it.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), int(threads))
        return it

    def dump(self, i: int, j: int) -> dict:
        d = OraclePixelDump()
        lib().oracle_trace_dump(ctypes.byref(self.scene), i, j, ctypes.byref(d))
        return {"pos": list(d.pos), "draw": d.draw, "iters": d.iters, "xcoord": d.xcoord,
                "ycoord": d.ycoord, "brightness": d.brightness, "texel": list(d.texel),
                "rgba": list(d.rgba)}


def fnv1a64(buf: np.ndarray) -> str:
    b = np.ascontiguousarray(buf, dtype=np.uint8).ravel()
    h = lib().oracle_fnv1a64(b.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), b.size)
    return f"{h:016x}"


def sort_spheres(spheres, cam_pos=(0.0, 0.0, 0.0)) -> np.ndarray:
    s = np.ascontiguousarray(np.asarray(spheres, dtype=np.float32).reshape(-1, 4)).copy()
    cam = (ctypes.c_float * 3)(*[float(c) for c in cam_pos])
    lib().oracle_sort_spheres(s.ctypes.data_as(ctypes.POINTER(OracleSphere)), s.shape[0], cam)
    return s


def add_spheres(adds, cam_pos=(0.0, 0.0, 0.0)) -> np.ndarray:
    """Replays AddSphere for each (x, y, z, r) in order: prune contained, re-sort."""
    adds = np.asarray(adds, dtype=np.float32).reshape(-1, 4)
    buf = np.zeros((adds.shape[0] + 1, 4), dtype=np.float32)
    cam = (ctypes.c_float * 3)(*[float(c) for c in cam_pos])
    n = 0
    for a in adds:
        n = lib().oracle_add_sphere(buf.ctypes.data_as(ctypes.POINTER(OracleSphere)), n,
                                    OracleSphere(*[float(v) for v in a]), cam)
    return buf[:n].copy()


# ---- voxel World (voxelworld_oracle.c) ----
class OvoxTexture(ctypes.Structure):
    _fields_ = [("rgba", ctypes.c_void_p), ("w", ctypes.c_int32), ("h", ctypes.c_int32)]


class OvoxScene(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32),
        ("cam_pos", ctypes.c_float * 3),
        ("cam_rotation", ctypes.c_float), ("cam_hrotation", ctypes.c_float),
        ("fov_h", ctypes.c_float), ("fov_v", ctypes.c_float),
        ("shadow_distance", ctypes.c_float), ("view_distance", ctypes.c_float),
        ("blocks", ctypes.c_void_p), ("nx", ctypes.c_int32), ("ny", ctypes.c_int32),
        ("nz", ctypes.c_int32),
        ("textures", OvoxTexture * 10), ("dyn_textures", OvoxTexture * 10),
        ("colors", (ctypes.c_uint8 * 4) * 10),
        ("dyn", ctypes.c_void_p), ("ndyn", ctypes.c_int32),
        ("lights", ctypes.c_void_p), ("nlights", ctypes.c_int32),
    ]


class VoxelOracle:
    """The voxel World restatement bound to one voxel_scenes.VoxelScene snapshot."""

    def __init__(self, scene, width, height, textures, dyn_textures, colors):
        L = lib()
        L.ovox_render_threaded.argtypes = [ctypes.POINTER(OvoxScene), ctypes.c_void_p,
                                           ctypes.c_int]
        L.ovox_update_image.argtypes = [ctypes.POINTER(OvoxScene), ctypes.c_void_p, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.ovox_bad_texel_reads.restype = ctypes.c_long
        self._keep = []
        sc = OvoxScene()
        sc.width, sc.height = int(width), int(height)
        for k in range(3):
            sc.cam_pos[k] = float(scene.cam_pos[k])
        sc.cam_rotation, sc.cam_hrotation = float(scene.rotation), float(scene.hrotation)
        sc.fov_h, sc.fov_v = float(scene.fov_h), float(scene.fov_v)
        sc.shadow_distance, sc.view_distance = float(scene.shadow_distance), float(scene.view_distance)
        blocks = np.ascontiguousarray(scene.blocks, dtype=np.int16)
        sc.blocks = blocks.ctypes.data
        sc.nx, sc.ny, sc.nz = blocks.shape
        for slot, lst in (("textures", textures), ("dyn_textures", dyn_textures)):
            arr = getattr(sc, slot)
            for k, (rgba, w, h) in enumerate(lst):
                buf = np.ascontiguousarray(rgba, dtype=np.uint8)
                self._keep.append(buf)
                arr[k].rgba, arr[k].w, arr[k].h = buf.ctypes.data, w, h
        for k in range(min(10, len(colors))):
            for c in range(4):
                sc.colors[k][c] = int(colors[k][c])
        dyn = np.ascontiguousarray(scene.dyn)
        lights = np.ascontiguousarray(scene.lights)
        sc.dyn, sc.ndyn = dyn.ctypes.data, dyn.shape[0]
        sc.lights, sc.nlights = lights.ctypes.data, lights.shape[0]
        self._keep += [blocks, dyn, lights]
        self.scene = sc

    def render(self, threads: int = 1) -> np.ndarray:
        out = np.zeros(self.scene.width * self.scene.height * 4, dtype=np.uint8)
        lib().ovox_render_threaded(ctypes.byref(self.scene), out.ctypes.data, int(threads))
        return out

    def update_image(self, out, ystart, yadd, xstart, xadd) -> None:
        lib().ovox_update_image(ctypes.byref(self.scene), out.ctypes.data, ystart, yadd, xstart,
                                xadd)

    @staticmethod
    def bad_texel_reads() -> int:
        return int(lib().ovox_bad_texel_reads())


OGLSL_DUMP_FIELDS = [
    ("dir", ctypes.c_float * 3), ("wall_pos", ctypes.c_float * 3), ("wall_dist", ctypes.c_float),
    ("wall_sphere", ctypes.c_int32), ("march_steps", ctypes.c_int32),
    ("ball_dist", ctypes.c_float), ("smooth_dist", ctypes.c_float),
    ("checkstep", ctypes.c_int32), ("draw_sphere", ctypes.c_int32),
    ("total_dist", ctypes.c_float), ("xcoord", ctypes.c_float), ("ycoord", ctypes.c_float),
    ("brightness", ctypes.c_float), ("color", ctypes.c_float * 4),
]


class OglslDump(ctypes.Structure):
    _fields_ = OGLSL_DUMP_FIELDS


class GlslOracle:
    """rayShader.frag restatement (oracle/glsl_oracle.c) for one uniform block
    (a glsl_scenes.UNIFORM_DTYPE record) and one ground texture."""

    def __init__(self, uniforms, ground, gw: int, gh: int):
        L = lib()
        vp, i = ctypes.c_void_p, ctypes.c_int
        L.oglsl_render.argtypes = [vp, vp, i, i, i, i, i, i, vp]
        L.oglsl_render.restype = ctypes.c_long
        L.oglsl_render_threaded.argtypes = [vp, vp, i, i, i, i, vp, i]
        L.oglsl_render_threaded.restype = ctypes.c_long
        L.oglsl_pixel.argtypes = [vp, vp, i, i, i, i, i, i, ctypes.POINTER(OglslDump)]
        L.oglsl_march_steps.argtypes = [vp, i, i, vp, i]
        self.u = np.ascontiguousarray(np.asarray(uniforms).reshape(()).copy())
        self.ground = np.ascontiguousarray(ground, dtype=np.uint8)
        self.gw, self.gh = int(gw), int(gh)

    def _args(self):
        return self.u.ctypes.data, self.ground.ctypes.data, self.gw, self.gh

    def render(self, width: int, height: int, threads: int = 1) -> np.ndarray:
        out = np.zeros(width * height * 4, dtype=np.uint8)
        capped = lib().oglsl_render_threaded(*self._args(), width, height, out.ctypes.data,
                                             int(threads))
        if capped:
            raise RuntimeError(f"{capped} pixels hit the march cap")
        return out

    def render_band(self, width: int, height: int, row0: int, rows: int) -> np.ndarray:
        out = np.zeros(width * rows * 4, dtype=np.uint8)
        capped = lib().oglsl_render(*self._args(), width, height, row0, rows, out.ctypes.data)
        if capped:
            raise RuntimeError(f"{capped} pixels hit the march cap")
        return out

    def pixel(self, width: int, height: int, i: int, row: int) -> dict:
        d = OglslDump()
        lib().oglsl_pixel(*self._args(), width, height, i, row, ctypes.byref(d))
        out = {}
        for name, _ in OGLSL_DUMP_FIELDS:
            v = getattr(d, name)
            out[name] = list(v) if hasattr(v, "__len__") else v
        return out

    def march_steps(self, width: int, height: int, threads: int = 1) -> np.ndarray:
        steps = np.zeros(width * height, dtype=np.int32)
        lib().oglsl_march_steps(self.u.ctypes.data, width, height, steps.ctypes.data, int(threads))
        return steps.reshape(height, width)
