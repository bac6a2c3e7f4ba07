"""Per-wave work counters of the GLSL kernel (instrumented build from tools/instrument_glsl.py):
wall iterations, march steps, dominance tests / ball bodies, shadow visits.  GPU only."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sfml-software-raytracer_amd"))
import torch, glsl_scenes as gs, scenes, sfrt
L = sfrt.lib()
L.sfrt_glsl_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
s = sfrt.GlslShader(0); s.set_ground(*scenes.load_floor())
out = (ctypes.c_ulonglong * 8)()
names = ["waves", "wall_iters_inside", "march_steps", "ball_bodies", "ball_visits", "shadow_full", "shadow_visits", "wall_iters"]
for key, w, h, u in [("default4k", 3840, 2160, gs.default_uniforms(3840, 2160)),
                     ("frames300_4k", 3840, 2160, gs.default_uniforms(3840, 2160, 5.5, -0.4, frames=300))]:
    s.set_uniforms(u)
    L.sfrt_glsl_stats(out, 1)
    s.draw_image(w, h)
    L.sfrt_glsl_stats(out, 1)
    v = list(out)
    print(key, {n: round(v[i] / v[0], 2) for i, n in enumerate(names)}, flush=True)
