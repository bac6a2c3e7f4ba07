"""Python plumbing over libsfrt.so (the C ABI in include/sfrt.h).

Used by bench.py, __graft_entry__.py and the tests.  The class ``World``
mirrors the reference's ``SphereWorld`` surface for this path
(/root/reference/Raytracing/SphereWorld.h:40-78): ``width``/``height``,
``cam``, ``AddSphere``, ``UpdateSpheres`` and ``UpdateImage(ystart, yadd,
xstart, xadd)``, plus the device-resident ``render_band`` used by the display
and multi-GPU paths.  There is no CPU fallback: if libsfrt.so is missing or
has no HIP device, construction raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# SFRT_LIB: another build of the same library (build-flag A/B timing in tools/ only;
# bench.py refuses any library whose build_flavour() is not "release").
LIB_PATH = os.environ.get("SFRT_LIB") or os.path.join(HERE, "libsfrt.so")

SFRT_OPT_CULL = 1
SFRT_OPT_RAYS_PER_LANE = 2
SFRT_OPT_TILE_ORDER = 3
ERRORS = {
    0: "SFRT_OK", -1: "SFRT_E_INVALID", -2: "SFRT_E_EMPTY", -3: "SFRT_E_NO_TEXTURE",
    -4: "SFRT_E_TOO_MANY", -5: "SFRT_E_HIP", -6: "SFRT_E_MARCH_LIMIT", -7: "SFRT_E_TEXEL",
}

# Every symbol include/sfrt.h declares (checked by tests/test_abi.py).
ABI_SYMBOLS = (
    "sfrt_world_create", "sfrt_world_destroy", "sfrt_world_set_size", "sfrt_world_get_size",
    "sfrt_world_set_camera", "sfrt_world_get_camera", "sfrt_world_load_texture",
    "sfrt_world_add_sphere", "sfrt_world_set_spheres", "sfrt_world_get_spheres",
    "sfrt_world_set_sphere_textures", "sfrt_world_get_sphere_textures",
    "sfrt_world_update_spheres", "sfrt_world_update_image", "sfrt_world_render_band",
    "sfrt_world_check", "sfrt_world_trace_points", "sfrt_world_set_option",
    "sfrt_world_submit_frame", "sfrt_world_wait_frame", "sfrt_host_alloc", "sfrt_host_free",
    "sfrt_sort_spheres", "sfrt_deg_to_rad", "sfrt_pass_threshold", "sfrt_error_string",
    "sfrt_version", "sfrt_build_flavour",
    "sfrt_voxel_create", "sfrt_voxel_destroy", "sfrt_voxel_set_size", "sfrt_voxel_set_camera",
    "sfrt_voxel_set_view", "sfrt_voxel_set_blocks", "sfrt_voxel_load_texture",
    "sfrt_voxel_load_dyn_texture", "sfrt_voxel_set_colors", "sfrt_voxel_set_dynamics",
    "sfrt_voxel_set_lights", "sfrt_voxel_light_dd_pass", "sfrt_voxel_update_image",
    "sfrt_voxel_render_band",
    "sfrt_voxel_check", "sfrt_voxel_set_option",
    "sfrt_glsl_create", "sfrt_glsl_destroy", "sfrt_glsl_set_ground", "sfrt_glsl_set_uniforms",
    "sfrt_glsl_get_uniforms", "sfrt_glsl_set_uniform", "sfrt_glsl_set_uniform_int",
    "sfrt_glsl_draw", "sfrt_glsl_draw_image", "sfrt_glsl_check", "sfrt_glsl_set_option",
    "sfrt_png_info", "sfrt_png_decode",
    "sfrt_multi_create", "sfrt_multi_destroy", "sfrt_multi_count", "sfrt_multi_world",
    "sfrt_multi_set_size", "sfrt_multi_set_camera", "sfrt_multi_load_texture",
    "sfrt_multi_set_spheres", "sfrt_multi_add_sphere", "sfrt_multi_update_spheres",
    "sfrt_multi_set_sphere_textures", "sfrt_multi_set_option", "sfrt_multi_set_bands",
    "sfrt_multi_bands", "sfrt_multi_render", "sfrt_multi_check", "sfrt_multi_update_image",
    "sfrt_world_row_costs", "sfrt_multi_cost_bands", "sfrt_multi_row_costs", "sfrt_multi_balance",
    "sfrt_multi_set_transfer", "sfrt_multi_get_transfer", "sfrt_band_packed_bytes", "sfrt_band_pack",
    "sfrt_band_unpack", "sfrt_world_alpha_binary", "sfrt_multi_transport_library",
    "sfrt_multi_use_test_transport",
)

SFRT_MULTI_AUTO, SFRT_MULTI_RCCL, SFRT_MULTI_PEER = 0, 1, 2
SFRT_TRANSFER_AUTO, SFRT_TRANSFER_RGBA, SFRT_TRANSFER_PACKED = 0, 1, 2


class SfrtError(RuntimeError):
    def __init__(self, code: int, what: str):
        self.code = code
        super().__init__(f"{what}: {ERRORS.get(code, code)} ({code})")


class Sphere(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float),
                ("radius", ctypes.c_float)]


class Camera(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_float * 3), ("rotation", ctypes.c_float),
                ("hrotation", ctypes.c_float), ("fov_h", ctypes.c_float),
                ("fov_v", ctypes.c_float)]


class PixelDump(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_float * 3), ("draw", ctypes.c_int32), ("iters", ctypes.c_int32),
                ("xcoord", ctypes.c_float), ("ycoord", ctypes.c_float),
                ("brightness", ctypes.c_float), ("texel", ctypes.c_uint32 * 2),
                ("rgba", ctypes.c_uint32)]


_lib = None


def lib() -> ctypes.CDLL:
    """Load libsfrt.so (raises if it was not built: no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run __graft_entry__.build() (make -C "
                           f"sfml-software-raytracer_amd)")
    # torch wheels bundle their own libamdhip64 (same soname).  Loading torch first
    # lets libsfrt.so bind to that one, so a process has ONE HIP runtime and torch
    # tensors / streams can be handed to render_band.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    P, c_int, c_float, vp = ctypes.POINTER, ctypes.c_int, ctypes.c_float, ctypes.c_void_p
    W = vp  # opaque sfrt_world*
    sig = {
        "sfrt_world_create": ([c_int, P(vp)], c_int),
        "sfrt_world_destroy": ([W], None),
        "sfrt_world_set_size": ([W, c_int, c_int], c_int),
        "sfrt_world_get_size": ([W, P(c_int), P(c_int)], c_int),
        "sfrt_world_set_camera": ([W, P(Camera)], c_int),
        "sfrt_world_get_camera": ([W, P(Camera)], c_int),
        "sfrt_world_load_texture": ([W, c_int, vp, c_int, c_int], c_int),
        "sfrt_world_add_sphere": ([W, c_float, c_float, c_float, c_float], c_int),
        "sfrt_world_set_spheres": ([W, vp, c_int], c_int),
        "sfrt_world_get_spheres": ([W, vp, c_int, P(c_int)], c_int),
        "sfrt_world_set_sphere_textures": ([W, vp, c_int], c_int),
        "sfrt_world_get_sphere_textures": ([W, vp, c_int, P(c_int)], c_int),
        "sfrt_world_update_spheres": ([W], c_int),
        "sfrt_world_update_image": ([W, vp, c_int, c_int, c_int, c_int], c_int),
        "sfrt_world_render_band": ([W, vp, ctypes.c_int64, c_int, c_int, vp], c_int),
        "sfrt_world_check": ([W, vp], c_int),
        "sfrt_world_row_costs": ([W, vp, c_int, P(c_int), P(c_int)], c_int),
        "sfrt_multi_cost_bands": ([vp, c_int, c_int, c_float, vp, vp], c_int),
        "sfrt_multi_row_costs": ([vp, vp, c_int], c_int),
        "sfrt_multi_balance": ([vp, c_float], c_int),
        "sfrt_world_trace_points": ([W, vp, c_int, vp], c_int),
        "sfrt_world_set_option": ([W, c_int, c_int], c_int),
        "sfrt_world_submit_frame": ([W, vp, P(ctypes.c_int64)], c_int),
        "sfrt_world_wait_frame": ([W, ctypes.c_int64], c_int),
        "sfrt_host_alloc": ([P(vp), ctypes.c_int64], c_int),
        "sfrt_host_free": ([vp], c_int),
        "sfrt_sort_spheres": ([vp, c_int, vp], c_int),
        "sfrt_deg_to_rad": ([c_float], c_float),
        "sfrt_pass_threshold": ([c_float], c_float),
        "sfrt_error_string": ([c_int], ctypes.c_char_p),
        "sfrt_version": ([], c_int),
        "sfrt_build_flavour": ([], ctypes.c_char_p),
        "sfrt_voxel_create": ([c_int, P(vp)], c_int),
        "sfrt_voxel_destroy": ([vp], None),
        "sfrt_voxel_set_size": ([vp, c_int, c_int], c_int),
        "sfrt_voxel_set_camera": ([vp, P(Camera)], c_int),
        "sfrt_voxel_set_view": ([vp, c_float, c_float], c_int),
        "sfrt_voxel_set_blocks": ([vp, vp, c_int, c_int, c_int], c_int),
        "sfrt_voxel_load_texture": ([vp, c_int, vp, c_int, c_int], c_int),
        "sfrt_voxel_load_dyn_texture": ([vp, c_int, vp, c_int, c_int], c_int),
        "sfrt_voxel_set_colors": ([vp, vp, c_int], c_int),
        "sfrt_voxel_set_dynamics": ([vp, vp, c_int], c_int),
        "sfrt_voxel_set_lights": ([vp, vp, c_int], c_int),
        "sfrt_voxel_light_dd_pass": ([ctypes.c_float], ctypes.c_float),
        "sfrt_voxel_update_image": ([vp, vp, c_int, c_int, c_int, c_int], c_int),
        "sfrt_voxel_render_band": ([vp, vp, ctypes.c_int64, c_int, c_int, vp], c_int),
        "sfrt_voxel_check": ([vp, vp], c_int),
        "sfrt_voxel_set_option": ([vp, c_int, c_int], c_int),
        "sfrt_glsl_create": ([c_int, P(vp)], c_int),
        "sfrt_glsl_destroy": ([vp], None),
        "sfrt_glsl_set_ground": ([vp, vp, c_int, c_int], c_int),
        "sfrt_glsl_set_uniforms": ([vp, vp], c_int),
        "sfrt_glsl_get_uniforms": ([vp, vp], c_int),
        "sfrt_glsl_set_uniform": ([vp, ctypes.c_char_p, vp, c_int], c_int),
        "sfrt_glsl_set_uniform_int": ([vp, ctypes.c_char_p, c_int], c_int),
        "sfrt_glsl_draw": ([vp, vp, c_int, c_int, ctypes.c_int64, c_int, c_int, vp], c_int),
        "sfrt_glsl_draw_image": ([vp, vp, c_int, c_int], c_int),
        "sfrt_glsl_check": ([vp, vp], c_int),
        "sfrt_glsl_set_option": ([vp, c_int, c_int], c_int),
        "sfrt_png_info": ([vp, ctypes.c_int64, P(c_int), P(c_int)], c_int),
        "sfrt_png_decode": ([vp, ctypes.c_int64, vp, ctypes.c_int64, P(c_int), P(c_int)], c_int),
        "sfrt_multi_create": ([vp, c_int, c_int, P(vp)], c_int),
        "sfrt_multi_destroy": ([vp], None),
        "sfrt_multi_count": ([vp, P(c_int), P(c_int)], c_int),
        "sfrt_multi_world": ([vp, c_int, P(vp)], c_int),
        "sfrt_multi_set_size": ([vp, c_int, c_int], c_int),
        "sfrt_multi_set_camera": ([vp, P(Camera)], c_int),
        "sfrt_multi_load_texture": ([vp, c_int, vp, c_int, c_int], c_int),
        "sfrt_multi_set_spheres": ([vp, vp, c_int], c_int),
        "sfrt_multi_add_sphere": ([vp, c_float, c_float, c_float, c_float], c_int),
        "sfrt_multi_update_spheres": ([vp], c_int),
        "sfrt_multi_set_sphere_textures": ([vp, vp, c_int], c_int),
        "sfrt_multi_set_option": ([vp, c_int, c_int], c_int),
        "sfrt_multi_set_bands": ([vp, vp, c_int], c_int),
        "sfrt_multi_bands": ([c_int, c_int, c_float, vp, vp], c_int),
        "sfrt_multi_render": ([vp, vp, ctypes.c_int64, vp], c_int),
        "sfrt_multi_check": ([vp], c_int),
        "sfrt_multi_set_transfer": ([vp, c_int], c_int),
        "sfrt_multi_get_transfer": ([vp, P(c_int), P(c_int)], c_int),
        "sfrt_band_packed_bytes": ([ctypes.c_int64], ctypes.c_int64),
        "sfrt_band_pack": ([vp, ctypes.c_int64, vp, vp], c_int),
        "sfrt_band_unpack": ([vp, ctypes.c_int64, vp, vp], c_int),
        "sfrt_world_alpha_binary": ([W, P(c_int)], c_int),
        "sfrt_multi_update_image": ([vp, vp], c_int),
        "sfrt_multi_transport_library": ([ctypes.c_char_p, c_int], c_int),
        "sfrt_multi_use_test_transport": ([ctypes.c_char_p], c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise SfrtError(rc, what)


def _f32_rows(spheres) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(spheres, dtype=np.float32).reshape(-1, 4))


def sort_spheres(spheres, cam_pos=(0.0, 0.0, 0.0)) -> np.ndarray:
    s = _f32_rows(spheres).copy()
    cam = (ctypes.c_float * 3)(*[float(c) for c in cam_pos])
    _check(lib().sfrt_sort_spheres(s.ctypes.data, s.shape[0], cam), "sfrt_sort_spheres")
    return s


def build_flavour() -> str:
    """sfrt_build_flavour: "release" for the shipped library, "diagnostic" / "ab" otherwise."""
    return lib().sfrt_build_flavour().decode()


def deg_to_rad(deg: float) -> float:
    return lib().sfrt_deg_to_rad(float(deg))


def pass_threshold(radius: float) -> float:
    return lib().sfrt_pass_threshold(float(radius))


class HostFrame:
    """Pinned host RGBA8 frame (sfrt_host_alloc), viewable as a numpy array."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        _check(lib().sfrt_host_alloc(ctypes.byref(p), int(nbytes)), "sfrt_host_alloc")
        self.ptr = p.value
        self.nbytes = int(nbytes)
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr))

    def free(self) -> None:
        if self.ptr:
            self.array = None
            lib().sfrt_host_free(ctypes.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class World:
    """Device-backed mirror of ``SphereWorld`` for the frame-fill path."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        _check(lib().sfrt_world_create(int(device), ctypes.byref(h)), "sfrt_world_create")
        self._h = h
        self.device = device

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().sfrt_world_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # --- state ---
    def set_size(self, width: int, height: int) -> None:
        _check(lib().sfrt_world_set_size(self._h, int(width), int(height)), "set_size")

    @property
    def size(self) -> tuple[int, int]:
        w, h = ctypes.c_int(), ctypes.c_int()
        _check(lib().sfrt_world_get_size(self._h, ctypes.byref(w), ctypes.byref(h)), "get_size")
        return w.value, h.value

    def set_camera(self, pos=(0.0, 0.0, 0.0), rotation=0.0, hrotation=0.0, fov_h=None,
                   fov_v=None) -> None:
        cur = self.camera
        cam = Camera()
        for k in range(3):
            cam.pos[k] = float(pos[k])
        cam.rotation, cam.hrotation = float(rotation), float(hrotation)
        cam.fov_h = float(fov_h) if fov_h is not None else cur.fov_h
        cam.fov_v = float(fov_v) if fov_v is not None else cur.fov_v
        _check(lib().sfrt_world_set_camera(self._h, ctypes.byref(cam)), "set_camera")

    @property
    def camera(self) -> Camera:
        cam = Camera()
        _check(lib().sfrt_world_get_camera(self._h, ctypes.byref(cam)), "get_camera")
        return cam

    def load_texture(self, rgba, tex_w: int, tex_h: int, slot: int = 0) -> None:
        buf = np.ascontiguousarray(np.asarray(rgba, dtype=np.uint8).ravel())
        if buf.size != tex_w * tex_h * 4:
            raise ValueError("texture size mismatch")
        _check(lib().sfrt_world_load_texture(self._h, slot, buf.ctypes.data, tex_w, tex_h),
               "load_texture")

    def add_sphere(self, x, y, z, radius) -> None:
        _check(lib().sfrt_world_add_sphere(self._h, float(x), float(y), float(z), float(radius)),
               "add_sphere")

    def set_spheres(self, spheres) -> None:
        s = _f32_rows(spheres)
        _check(lib().sfrt_world_set_spheres(self._h, s.ctypes.data, s.shape[0]), "set_spheres")

    @property
    def spheres(self) -> np.ndarray:
        n = ctypes.c_int()
        _check(lib().sfrt_world_get_spheres(self._h, None, 0, ctypes.byref(n)), "get_spheres")
        out = np.zeros((n.value, 4), dtype=np.float32)
        _check(lib().sfrt_world_get_spheres(self._h, out.ctypes.data, n.value, ctypes.byref(n)),
               "get_spheres")
        return out

    def set_sphere_textures(self, slots) -> None:
        """Texture slot per sphere (current order): the "all textures" extension."""
        a = np.ascontiguousarray(np.asarray(slots, dtype=np.int32).ravel())
        _check(lib().sfrt_world_set_sphere_textures(self._h, a.ctypes.data, a.size),
               "set_sphere_textures")

    @property
    def sphere_textures(self) -> np.ndarray:
        n = ctypes.c_int()
        _check(lib().sfrt_world_get_sphere_textures(self._h, None, 0, ctypes.byref(n)),
               "get_sphere_textures")
        out = np.zeros(n.value, dtype=np.int32)
        _check(lib().sfrt_world_get_sphere_textures(self._h, out.ctypes.data, n.value,
                                                    ctypes.byref(n)), "get_sphere_textures")
        return out

    def update_spheres(self) -> None:
        _check(lib().sfrt_world_update_spheres(self._h), "update_spheres")

    def set_option(self, option: int, value: int) -> None:
        _check(lib().sfrt_world_set_option(self._h, option, value), "set_option")

    def set_scene(self, scene, width: int, height: int) -> None:
        """Load a scenes.Scene (spheres verbatim, camera pose) at width x height."""
        self.set_size(width, height)
        self.set_camera(scene.cam_pos, scene.rotation, scene.hrotation, scene.fov_h, scene.fov_v)
        self.set_spheres(scene.spheres)

    # --- frame fill ---
    def update_image(self, pixels: np.ndarray, ystart=0, yadd=1, xstart=0, xadd=1) -> np.ndarray:
        """SphereWorld::UpdateImage into a host RGBA8 buffer (width*height*4 bytes)."""
        w, h = self.size
        if pixels.dtype != np.uint8 or pixels.size != w * h * 4 or not pixels.flags.c_contiguous:
            raise ValueError("pixels must be a contiguous uint8 array of width*height*4")
        _check(lib().sfrt_world_update_image(self._h, pixels.ctypes.data, ystart, yadd, xstart,
                                             xadd), "update_image")
        return pixels

    def render(self) -> np.ndarray:
        w, h = self.size
        out = np.zeros(w * h * 4, dtype=np.uint8)
        return self.update_image(out)

    def render_band(self, dev_ptr: int, pitch_bytes: int, row0: int, rows: int,
                    stream: int = 0) -> None:
        """Asynchronous device fill of rows [row0, row0+rows) at dev_ptr on `stream`."""
        _check(lib().sfrt_world_render_band(self._h, ctypes.c_void_p(dev_ptr), int(pitch_bytes),
                                            int(row0), int(rows), ctypes.c_void_p(stream or None)),
               "render_band")

    def submit_frame(self, frame: "HostFrame") -> int:
        """Pipelined full-frame fill into a pinned HostFrame; returns a ticket."""
        w, h = self.size
        if frame.nbytes < w * h * 4:
            raise ValueError("host frame too small")
        t = ctypes.c_int64()
        _check(lib().sfrt_world_submit_frame(self._h, ctypes.c_void_p(frame.ptr), ctypes.byref(t)),
               "submit_frame")
        return t.value

    def wait_frame(self, ticket: int) -> None:
        _check(lib().sfrt_world_wait_frame(self._h, int(ticket)), "wait_frame")

    def check(self, stream: int = 0) -> None:
        _check(lib().sfrt_world_check(self._h, ctypes.c_void_p(stream or None)), "check")

    def row_costs(self) -> tuple[int, np.ndarray]:
        """(row0, per-row ray-steps) of the last ordered frame fill (sfrt_world_row_costs)."""
        _, h = self.size
        out = np.zeros(max(h, 1), dtype=np.float32)
        r0, n = ctypes.c_int(), ctypes.c_int()
        _check(lib().sfrt_world_row_costs(self._h, out.ctypes.data, out.size, ctypes.byref(r0),
                                          ctypes.byref(n)), "row_costs")
        return r0.value, out[:n.value].copy()

    def alpha_binary(self) -> bool:
        """sfrt_world_alpha_binary: every loaded texel's alpha is 0 or 255 (bands pack)."""
        b = ctypes.c_int()
        _check(lib().sfrt_world_alpha_binary(self._h, ctypes.byref(b)), "alpha_binary")
        return bool(b.value)

    def trace_points(self, ij) -> list[dict]:
        ij = np.ascontiguousarray(np.asarray(ij, dtype=np.int32).reshape(-1, 2))
        out = (PixelDump * ij.shape[0])()
        _check(lib().sfrt_world_trace_points(self._h, ij.ctypes.data, ij.shape[0],
                                             ctypes.cast(out, ctypes.c_void_p)), "trace_points")
        res = []
        for d in out:
            rgba = d.rgba
            res.append({"pos": list(d.pos), "draw": d.draw, "iters": d.iters,
                        "xcoord": d.xcoord, "ycoord": d.ycoord, "brightness": d.brightness,
                        "texel": list(d.texel),
                        "rgba": [rgba & 255, (rgba >> 8) & 255, (rgba >> 16) & 255, rgba >> 24]})
        return res


class VoxelWorld:
    """Device-backed mirror of the reference's voxel ``World`` frame fill
    (World.h:58-97); the scene is a voxel_scenes.VoxelScene snapshot."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        _check(lib().sfrt_voxel_create(int(device), ctypes.byref(h)), "sfrt_voxel_create")
        self._h = h
        self.width = self.height = 0

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().sfrt_voxel_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def load_assets(self, textures, dyn_textures, colors) -> None:
        for k, (rgba, w, h) in enumerate(textures):
            buf = np.ascontiguousarray(rgba, dtype=np.uint8)
            _check(lib().sfrt_voxel_load_texture(self._h, k, buf.ctypes.data, w, h), "load_texture")
        for k, (rgba, w, h) in enumerate(dyn_textures):
            buf = np.ascontiguousarray(rgba, dtype=np.uint8)
            _check(lib().sfrt_voxel_load_dyn_texture(self._h, k, buf.ctypes.data, w, h),
                   "load_dyn_texture")
        col = np.ascontiguousarray(colors, dtype=np.uint8)
        _check(lib().sfrt_voxel_set_colors(self._h, col.ctypes.data, col.shape[0]), "set_colors")

    def load_texture(self, slot: int, rgba, w: int, h: int) -> None:
        """textures[slot] (World.h:90) alone: sfrt_voxel_load_texture, stream-ordered."""
        buf = np.ascontiguousarray(rgba, dtype=np.uint8)
        _check(lib().sfrt_voxel_load_texture(self._h, int(slot), buf.ctypes.data, int(w), int(h)),
               "load_texture")

    def set_scene(self, scene, width: int, height: int) -> None:
        self.width, self.height = int(width), int(height)
        _check(lib().sfrt_voxel_set_size(self._h, self.width, self.height), "set_size")
        cam = Camera()
        for k in range(3):
            cam.pos[k] = float(scene.cam_pos[k])
        cam.rotation, cam.hrotation = float(scene.rotation), float(scene.hrotation)
        cam.fov_h, cam.fov_v = float(scene.fov_h), float(scene.fov_v)
        _check(lib().sfrt_voxel_set_camera(self._h, ctypes.byref(cam)), "set_camera")
        _check(lib().sfrt_voxel_set_view(self._h, float(scene.shadow_distance),
                                         float(scene.view_distance)), "set_view")
        b = np.ascontiguousarray(scene.blocks, dtype=np.int16)
        _check(lib().sfrt_voxel_set_blocks(self._h, b.ctypes.data, *b.shape), "set_blocks")
        d = np.ascontiguousarray(scene.dyn)
        _check(lib().sfrt_voxel_set_dynamics(self._h, d.ctypes.data, d.shape[0]), "set_dynamics")
        l = np.ascontiguousarray(scene.lights)
        _check(lib().sfrt_voxel_set_lights(self._h, l.ctypes.data, l.shape[0]), "set_lights")

    def update_image(self, pixels: np.ndarray, ystart=0, yadd=1, xstart=0, xadd=1) -> np.ndarray:
        if pixels.dtype != np.uint8 or pixels.size != self.width * self.height * 4:
            raise ValueError("pixels must be uint8 width*height*4")
        _check(lib().sfrt_voxel_update_image(self._h, pixels.ctypes.data, ystart, yadd, xstart,
                                             xadd), "voxel_update_image")
        return pixels

    def render(self) -> np.ndarray:
        return self.update_image(np.zeros(self.width * self.height * 4, np.uint8))

    def render_band(self, dev_ptr: int, pitch_bytes: int, row0: int, rows: int,
                    stream: int = 0) -> None:
        _check(lib().sfrt_voxel_render_band(self._h, ctypes.c_void_p(dev_ptr), int(pitch_bytes),
                                            int(row0), int(rows), ctypes.c_void_p(stream or None)),
               "voxel_render_band")

    def check(self, stream: int = 0) -> None:
        _check(lib().sfrt_voxel_check(self._h, ctypes.c_void_p(stream or None)), "voxel_check")

    def set_option(self, option: int, value: int) -> None:
        _check(lib().sfrt_voxel_set_option(self._h, option, value), "voxel_set_option")


def band_packed_bytes(pixels: int) -> int:
    """sfrt_band_packed_bytes: bytes of a packed band of `pixels` pixels (3.125 B each)."""
    b = lib().sfrt_band_packed_bytes(int(pixels))
    if b < 0:
        raise SfrtError(int(b), "band_packed_bytes")
    return int(b)


def band_pack(src_ptr: int, pixels: int, dst_ptr: int, stream: int = 0) -> None:
    """sfrt_band_pack: RGBA8 device pixels -> the packed transfer format (asynchronous)."""
    _check(lib().sfrt_band_pack(ctypes.c_void_p(src_ptr), int(pixels), ctypes.c_void_p(dst_ptr),
                                ctypes.c_void_p(stream or None)), "band_pack")


def band_unpack(src_ptr: int, pixels: int, dst_ptr: int, stream: int = 0) -> None:
    """sfrt_band_unpack: the packed transfer format -> RGBA8 device pixels (asynchronous)."""
    _check(lib().sfrt_band_unpack(ctypes.c_void_p(src_ptr), int(pixels), ctypes.c_void_p(dst_ptr),
                                  ctypes.c_void_p(stream or None)), "band_unpack")


def multi_transport_library() -> str:
    """sfrt_multi_transport_library: "" before the first RCCL context, else the library behind
    SFRT_MULTI_RCCL ("librccl.so.1", or "test:<path>" for a test transport)."""
    buf = ctypes.create_string_buffer(4096)
    _check(lib().sfrt_multi_transport_library(buf, len(buf)), "sfrt_multi_transport_library")
    return buf.value.decode()


def use_test_transport(path: str) -> None:
    """TEST ONLY (sfrt_multi_use_test_transport): the RCCL C API from `path`, before the
    process's first RCCL context."""
    _check(lib().sfrt_multi_use_test_transport(path.encode()), "sfrt_multi_use_test_transport")


def multi_bands(height: int, n: int, root_factor: float = 1.0) -> list[tuple[int, int]]:
    """sfrt_multi_bands: (row0, rows) per rank, rank 0 ~root_factor x the others' rows."""
    row0 = np.zeros(n, dtype=np.int32)
    rows = np.zeros(n, dtype=np.int32)
    _check(lib().sfrt_multi_bands(int(height), int(n), float(root_factor), row0.ctypes.data,
                                  rows.ctypes.data), "sfrt_multi_bands")
    return [(int(a), int(b)) for a, b in zip(row0, rows)]


def multi_cost_bands(row_cost, n: int, root_factor: float = 1.0) -> list[tuple[int, int]]:
    """sfrt_multi_cost_bands: (row0, rows) per rank, rank 0 ~root_factor x the others' cost."""
    c = np.ascontiguousarray(np.asarray(row_cost, dtype=np.float32))
    row0 = np.zeros(n, dtype=np.int32)
    rows = np.zeros(n, dtype=np.int32)
    _check(lib().sfrt_multi_cost_bands(c.ctypes.data if c.size else None, int(c.size), int(n),
                                       float(root_factor), row0.ctypes.data, rows.ctypes.data),
           "sfrt_multi_cost_bands")
    return [(int(a), int(b)) for a, b in zip(row0, rows)]


class Multi:
    """One frame over several GPUs of this node through the C ABI (sfrt_multi_*): the scene
    setters of ``World`` broadcast to one world per device, the frame is rendered in row
    bands and gathered on devices[0] (RCCL or peer copies)."""

    def __init__(self, devices, transport: int = SFRT_MULTI_AUTO):
        devs = np.ascontiguousarray(np.asarray(devices, dtype=np.int32))
        h = ctypes.c_void_p()
        _check(lib().sfrt_multi_create(devs.ctypes.data, devs.size, int(transport),
                                       ctypes.byref(h)), "sfrt_multi_create")
        self._h = h
        self.devices = [int(d) for d in devs]
        self.width = self.height = 0

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().sfrt_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def transport(self) -> int:
        n, t = ctypes.c_int(), ctypes.c_int()
        _check(lib().sfrt_multi_count(self._h, ctypes.byref(n), ctypes.byref(t)), "multi_count")
        return t.value

    def load_texture(self, rgba, tex_w: int, tex_h: int, slot: int = 0) -> None:
        buf = np.ascontiguousarray(np.asarray(rgba, dtype=np.uint8).ravel())
        _check(lib().sfrt_multi_load_texture(self._h, slot, buf.ctypes.data, tex_w, tex_h),
               "multi_load_texture")

    def set_camera(self, pos, rotation=0.0, hrotation=0.0, fov_h=None, fov_v=None) -> None:
        cam = Camera()
        for k in range(3):
            cam.pos[k] = float(pos[k])
        cam.rotation, cam.hrotation = float(rotation), float(hrotation)
        cam.fov_h = float(fov_h) if fov_h is not None else float(deg_to_rad(75.0))
        cam.fov_v = float(fov_v) if fov_v is not None else float(deg_to_rad(47.0))
        _check(lib().sfrt_multi_set_camera(self._h, ctypes.byref(cam)), "multi_set_camera")

    def set_scene(self, scene, width: int, height: int) -> None:
        self.width, self.height = int(width), int(height)
        _check(lib().sfrt_multi_set_size(self._h, self.width, self.height), "multi_set_size")
        self.set_camera(scene.cam_pos, scene.rotation, scene.hrotation, scene.fov_h, scene.fov_v)
        s = _f32_rows(scene.spheres)
        _check(lib().sfrt_multi_set_spheres(self._h, s.ctypes.data, s.shape[0]), "multi_set_spheres")

    def set_option(self, option: int, value: int) -> None:
        _check(lib().sfrt_multi_set_option(self._h, option, value), "multi_set_option")

    def set_transfer(self, fmt: int) -> None:
        """sfrt_multi_set_transfer: SFRT_TRANSFER_AUTO / _RGBA / _PACKED."""
        _check(lib().sfrt_multi_set_transfer(self._h, int(fmt)), "multi_set_transfer")

    def transfer(self) -> tuple[int, bool]:
        """(the transfer setting, whether the last render packed its bands)."""
        f, p = ctypes.c_int(), ctypes.c_int()
        _check(lib().sfrt_multi_get_transfer(self._h, ctypes.byref(f), ctypes.byref(p)),
               "multi_get_transfer")
        return f.value, bool(p.value)

    def set_bands(self, rows=None) -> None:
        if rows is None:
            _check(lib().sfrt_multi_set_bands(self._h, None, 0), "multi_set_bands")
            return
        r = np.ascontiguousarray(np.asarray(rows, dtype=np.int32))
        _check(lib().sfrt_multi_set_bands(self._h, r.ctypes.data, r.size), "multi_set_bands")

    def row_costs(self) -> np.ndarray:
        """Per-row ray-steps of the last frame, from every rank's band (sfrt_multi_row_costs)."""
        out = np.zeros(self.height, dtype=np.float32)
        _check(lib().sfrt_multi_row_costs(self._h, out.ctypes.data, self.height), "multi_row_costs")
        return out

    def band_costs(self, rank: int) -> tuple[int, np.ndarray]:
        """(row0, per-row ray-steps) of rank `rank`'s last band (its world's row costs)."""
        wh = ctypes.c_void_p()
        _check(lib().sfrt_multi_world(self._h, int(rank), ctypes.byref(wh)), "multi_world")
        out = np.zeros(max(self.height, 1), dtype=np.float32)
        r0, n = ctypes.c_int(), ctypes.c_int()
        _check(lib().sfrt_world_row_costs(wh, out.ctypes.data, out.size, ctypes.byref(r0),
                                          ctypes.byref(n)), "row_costs")
        return r0.value, out[:n.value].copy()

    def balance(self, root_factor: float = 1.0) -> None:
        """Cost-weighted bands from the last frame (sfrt_multi_balance)."""
        _check(lib().sfrt_multi_balance(self._h, float(root_factor)), "multi_balance")

    def render(self, dev_ptr: int, pitch_bytes: int, stream: int = 0) -> None:
        _check(lib().sfrt_multi_render(self._h, ctypes.c_void_p(dev_ptr), int(pitch_bytes),
                                       ctypes.c_void_p(stream or None)), "multi_render")

    def check(self) -> None:
        _check(lib().sfrt_multi_check(self._h), "multi_check")

    def update_image(self, pixels=None) -> np.ndarray:
        if pixels is None:
            pixels = np.zeros(self.width * self.height * 4, dtype=np.uint8)
        if pixels.dtype != np.uint8 or pixels.size != self.width * self.height * 4:
            raise ValueError("pixels must be uint8 width*height*4")
        _check(lib().sfrt_multi_update_image(self._h, pixels.ctypes.data), "multi_update_image")
        return pixels


def decode_png(data: bytes) -> tuple[np.ndarray, int, int]:
    """PNG bytes -> (RGBA8 uint8 array, width, height), as sf::Image::loadFromFile."""
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    w, h = ctypes.c_int(), ctypes.c_int()
    _check(lib().sfrt_png_info(buf.ctypes.data, buf.size, ctypes.byref(w), ctypes.byref(h)),
           "png_info")
    out = np.empty(w.value * h.value * 4, dtype=np.uint8)
    _check(lib().sfrt_png_decode(buf.ctypes.data, buf.size, out.ctypes.data, out.size,
                                 ctypes.byref(w), ctypes.byref(h)), "png_decode")
    return out, w.value, h.value


class GlslShader:
    """Device-backed rayShader.frag: the uniform state of
    ``SphereWorld::shader`` plus ``rt.draw(sp, &shader)``.  Uniform blocks are
    glsl_scenes.UNIFORM_DTYPE records (the layout of sfrt_glsl_uniforms)."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        _check(lib().sfrt_glsl_create(int(device), ctypes.byref(h)), "sfrt_glsl_create")
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().sfrt_glsl_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_ground(self, rgba, w: int, h: int) -> None:
        buf = np.ascontiguousarray(rgba, dtype=np.uint8)
        if buf.size != w * h * 4:
            raise ValueError("ground size mismatch")
        _check(lib().sfrt_glsl_set_ground(self._h, buf.ctypes.data, int(w), int(h)), "set_ground")

    def set_uniforms(self, u) -> None:
        rec = np.ascontiguousarray(np.asarray(u).reshape(()))
        _check(lib().sfrt_glsl_set_uniforms(self._h, rec.ctypes.data), "set_uniforms")

    def get_uniforms(self, dtype):
        rec = np.zeros((), dtype=dtype)
        _check(lib().sfrt_glsl_get_uniforms(self._h, rec.ctypes.data), "get_uniforms")
        return rec

    def set_uniform(self, name: str, value) -> None:
        """sf::Shader::setUniform: floats/vectors by name, ints for the counts."""
        if isinstance(value, (int, np.integer)):
            _check(lib().sfrt_glsl_set_uniform_int(self._h, name.encode(), int(value)), name)
            return
        v = np.ascontiguousarray(np.atleast_1d(np.asarray(value, dtype=np.float32)))
        _check(lib().sfrt_glsl_set_uniform(self._h, name.encode(), v.ctypes.data, v.size), name)

    def draw(self, dev_ptr: int, width: int, height: int, pitch_bytes: int, row0: int = 0,
             rows: int | None = None, stream: int = 0) -> None:
        rows = height - row0 if rows is None else rows
        _check(lib().sfrt_glsl_draw(self._h, ctypes.c_void_p(dev_ptr), int(width), int(height),
                                    int(pitch_bytes), int(row0), int(rows),
                                    ctypes.c_void_p(stream or None)), "glsl_draw")

    def draw_image(self, width: int, height: int) -> np.ndarray:
        out = np.zeros(width * height * 4, dtype=np.uint8)
        _check(lib().sfrt_glsl_draw_image(self._h, out.ctypes.data, int(width), int(height)),
               "glsl_draw_image")
        return out

    def check(self, stream: int = 0) -> None:
        _check(lib().sfrt_glsl_check(self._h, ctypes.c_void_p(stream or None)), "glsl_check")

    def set_option(self, option: int, value: int) -> None:
        _check(lib().sfrt_glsl_set_option(self._h, option, value), "glsl_set_option")
