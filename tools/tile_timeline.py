"""Diagnostic: per-tile wall-clock start/end of the sphere kernel (a build with
-DSFRT_EXP=16 writes them into pixels 0-3 of each tile's first row; wrong image bytes).
    SFRT_LIB=sfml-software-raytracer_amd/build_x16/libsfrt.so python tools/tile_timeline.py [--1080]
        [--rays 2] [--dump DIR] [--entry] [--clock]
--rays forces the pixels per lane of the 4K frame (SFRT_OPT_RAYS_PER_LANE); --dump saves each case's
per-tile start, end and trips (tile order) as DIR/<case>_r<R>.npz; --entry (a -DSFRT_EXP=528 build)
reports the time from the wave's entry to its tile start; --clock (a -DSFRT_EXP=1040 build) the
shader clock over each tile (its s_memtime clocks over its s_memrealtime span).
Prints the kernel's span, the distribution of tile durations, and when the longest
tiles start and end, for a static and a turning camera."""
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
    # --1080: the 1920x1080 10-sphere frame (16x8 tiles in the adaptive order)
    W, H, R, sc = (1920, 1080, 2, scenes.default10()) if "--1080" in sys.argv else \
        (3840, 2160, 4, scenes.lcg64())
    if "--rays" in sys.argv:
        R = int(sys.argv[sys.argv.index("--rays") + 1])
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    stream = torch.cuda.Stream()
    w = sfrt.World(0)
    w.load_texture(*scenes.load_floor())
    if "--rays" in sys.argv:
        w.set_option(sfrt.SFRT_OPT_RAYS_PER_LANE, R)
    out = {}
    for name, turn, order in (("static", False, 1), ("turning", True, 1), ("static_rowmajor", False, 0)):
        w.set_scene(sc, W, H)
        w.set_option(sfrt.SFRT_OPT_TILE_ORDER, order)
        buf = torch.zeros(H, W * 4, dtype=torch.uint8, device="cuda")
        for k in range(300):
            if turn:
                w.set_camera(sc.cam_pos, 0.004 * k, 0.0)
            w.render_band(buf.data_ptr(), W * 4, 0, H, stream.cuda_stream)
        torch.cuda.synchronize()
        px = buf.cpu().numpy().view(np.uint32).reshape(H, W)
        tiles = px[0::8, :].reshape(H // 8, W // (8 * R), 8 * R)[:, :, :4].reshape(-1, 4).astype(np.int64)
        t0, t1, trips, slot = tiles[:, 0], tiles[:, 1], tiles[:, 2], tiles[:, 3]
        base = t0.min()
        t0 = (t0 - base) * 10  # ns (100 MHz)
        t1 = (t1 - base) * 10
        dur = t1 - t0
        if "--clock" in sys.argv:  # -DSFRT_EXP=1040 build: the trips field holds the tile's s_memtime clocks
            ghz = trips / np.maximum(dur, 1) 
            wsum = float((trips).sum()) / float(dur.sum())
            print(name, "shader_clock_GHz_p10_p50_p90_weighted",
                  [round(float(np.percentile(ghz, q)), 3) for q in (10, 50, 90)] + [round(wsum, 3)], flush=True)
        if "--entry" in sys.argv:  # -DSFRT_EXP=528 build: the slot field holds the entry time
            ent = (slot - base) * 10
            pro = t0 - ent
            print(name, "entry_to_tile_start_us_p10_p50_p90_p99",
                  [round(float(np.percentile(pro, q)) / 1e3, 2) for q in (10, 50, 90, 99)], flush=True)
        if dump:
            os.makedirs(dump, exist_ok=True)
            np.savez(os.path.join(dump, f"{name}_r{R}.npz"), t0=t0, t1=t1, trips=trips, slot=slot)
        top = np.argsort(-dur)[:10]
        out[name] = {
            "span_us": round(float(t1.max()) / 1e3, 1),
            "last_start_us": round(float(t0.max()) / 1e3, 1),
            "dur_us_p50_p90_p99_max": [round(float(np.percentile(dur, q)) / 1e3, 1) for q in (50, 90, 99, 100)],
            "longest": [{"trips": int(trips[i]), "start_us": round(t0[i] / 1e3, 1), "end_us": round(t1[i] / 1e3, 1),
                         "slot": int(slot[i])} for i in top],
            "sum_dur_over_8192_slots_us": round(float(dur.sum()) / 8192 / 1e3, 1),
        }
        # waves in flight per 2 us bin (8192 = every wave slot of the chip busy)
        edges = np.arange(0.0, float(t1.max()) + 2000.0, 2000.0)
        started = np.searchsorted(np.sort(t0), edges[:-1] + 1000.0)
        ended = np.searchsorted(np.sort(t1), edges[:-1] + 1000.0)
        out[name]["waves_in_flight_per_2us"] = [int(v) for v in started - ended]
        # tiles finished by the end of each 10 us
        ends10 = np.arange(10000.0, float(t1.max()) + 10000.0, 10000.0)
        out[name]["tiles_done_by_10us"] = [int(v) for v in np.searchsorted(np.sort(t1), ends10)]
        # wave-slot time inside the span that holds no wave, as a fraction of 8192 x span
        out[name]["idle_slot_frac"] = round(1.0 - float(dur.sum()) / (8192.0 * float(t1.max())), 3)
        print(name, json.dumps(out[name]), flush=True)
    w.set_option(sfrt.SFRT_OPT_TILE_ORDER, 1)
    w.set_option(sfrt.SFRT_OPT_RAYS_PER_LANE, 0)


if __name__ == "__main__":
    main()
