"""End-to-end display-path throughput: frames delivered to
host memory, PCIe copy included, the camera turning every frame.

    python tools/bench_display.py [--frames 200]

Modes: "pipelined" = sfrt_world_submit_frame / wait_frame into pinned frames,
two in flight (render k+1 overlaps the copy of k); "sync" =
sfrt_world_update_image per frame (render, copy, scatter, no overlap).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sfml-software-raytracer_amd"))

import numpy as np  # noqa: E402

import scenes  # noqa: E402
import sfrt  # noqa: E402


def run(w, width, height, frames, mode):
    scene = scenes.lcg64()
    w.set_scene(scene, width, height)
    if mode == "pipelined":
        bufs = [sfrt.HostFrame(width * height * 4) for _ in range(2)]
        pending = []
        t0 = time.perf_counter()
        for k in range(frames):
            w.set_camera(scene.cam_pos, 0.002 * k, 0.0)
            pending.append(w.submit_frame(bufs[k % 2]))
            if len(pending) == 2:
                w.wait_frame(pending.pop(0))
        for t in pending:
            w.wait_frame(t)
        dt = time.perf_counter() - t0
        for b in bufs:
            b.free()
    else:
        out = np.zeros(width * height * 4, np.uint8)
        t0 = time.perf_counter()
        for k in range(frames):
            w.set_camera(scene.cam_pos, 0.002 * k, 0.0)
            w.update_image(out)
        dt = time.perf_counter() - t0
    return {"fps": round(frames / dt, 1), "Mrays_per_s": round(width * height * frames / dt / 1e6, 1),
            "GB_per_s_to_host": round(width * height * 4 * frames / dt / 1e9, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    args = ap.parse_args()
    w = sfrt.World(0)
    w.load_texture(*scenes.load_floor())
    res = {}
    for width, height in [(1920, 1080), (3840, 2160)]:
        for mode in ("pipelined", "sync"):
            run(w, width, height, 10, mode)  # warm-up
            res[f"{width}x{height}/{mode}"] = run(w, width, height, args.frames, mode)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
