"""Diagnostic: per-tile march counters of the sphere kernel (a build with -DSFRT_EXP=32
writes, per tile, its march steps, sphere visits, visits that passed for some ray, the
mode -- 0: SGPR slots, 1: window -- and the culled sphere count into pixels 0-4 of the
tile's first row; wrong image bytes).
    SFRT_LIB=sfml-software-raytracer_amd/build_x32/libsfrt.so python tools/visit_counts.py
Prints per-step visit rates of the real kernel ("where the time goes")."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sfml-software-raytracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import scenes  # noqa: E402
import sfrt  # noqa: E402


def main():
    stream = torch.cuda.Stream()
    w = sfrt.World(0)
    w.load_texture(*scenes.load_floor())
    for name, W, H, pose, R in (("4k_lcg64", 3840, 2160, (0.0, 0.0), 4),
                                ("4k_lcg64_rot", 3840, 2160, (1.1, -0.2), 4),
                                ("1080_default10", 1920, 1080, (0.0, 0.0), 2),
                                ("4k_lcg256", 3840, 2160, (0.0, 0.0), 4)):
        sname = name.split("_", 1)[1].replace("_rot", "")
        w.set_scene(scenes.SCENES[sname]().posed(*pose), W, H)
        buf = torch.zeros(H, W * 4, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            w.render_band(buf.data_ptr(), W * 4, 0, H, stream.cuda_stream)
        torch.cuda.synchronize()
        px = buf.cpu().numpy().view(np.uint32).reshape(H, W)
        tw = 8 * R
        t = px[0::8, :(W // tw) * tw].reshape(H // 8, W // tw, tw)[:, :, :5].reshape(-1, 5).astype(np.int64)
        trips, visits, passes, mode, culled = t.T
        steps = np.maximum(trips - 1, 1)  # kernel steps (the first is on the host)
        win = mode == 1
        out = {
            "tiles": int(t.shape[0]),
            "mean_tile_steps": round(float(trips.mean()), 2),
            "window_tiles_frac": round(float(win.mean()), 3),
            "visits_per_step_all": round(float(visits.sum() / steps.sum()), 3),
            "passes_per_step_all": round(float(passes.sum() / steps.sum()), 3),
            "visits_per_step_window": round(float(visits[win].sum() / steps[win].sum()), 3),
            "passes_per_step_window": round(float(passes[win].sum() / steps[win].sum()), 3),
            "culled_mean_window": round(float(culled[win].mean()), 2),
            "culled_mean_slots": round(float(culled[~win].mean()), 2) if (~win).any() else None,
        }
        print(name, json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
