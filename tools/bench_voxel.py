"""Voxel World frame fill throughput on MI355X vs the CPU
restatement on the host cores, same frames, bytes compared.

    python tools/bench_voxel.py [--steps 30]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sfml-software-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import sfrt  # noqa: E402
import voxel_scenes as vs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--orders", default="0",
                    help="comma list of SFRT_OPT_TILE_ORDER values (0 row-major = the default "
                         "here, 1 adaptive; entries get /ordered)")
    ap.add_argument("--set", choices=("all", "bench"), default="all",
                    help="bench: only the two frames bench.py times (1080p and 4K at the default "
                         "pose), one frame per launch size, so that rocprof summaries per launch "
                         "size map 1:1 to bench lines")
    args = ap.parse_args()
    import oracle  # CPU baseline / checker only
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    tex, dyn = vs.load_textures()
    w = sfrt.VoxelWorld(0)
    w.load_assets(tex, dyn, vs.COLORS)
    res = {}
    threads = max(1, min(16, os.cpu_count() or 1))
    frames = [(1920, 1080, ((15.5, 1.9, 15.5), 0.0, 0.0)),
              (3840, 2160, ((15.5, 1.9, 15.5), 0.0, 0.0)),
              (3840, 2160, ((47.5, 1.5, 60.1), 4.0, -0.3))]
    if args.set == "bench":
        frames = frames[:2]
    runs = [(wd, ht, ps, od) for wd, ht, ps in frames
            for od in [int(x) for x in args.orders.split(",")]]
    for width, height, pose, order in runs:
        w.set_option(sfrt.SFRT_OPT_TILE_ORDER, order)
        scene = vs.default_world(*pose)
        w.set_scene(scene, width, height)
        buf = torch.empty(height, width * 4, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            w.render_band(buf.data_ptr(), width * 4, 0, height, stream.cuda_stream)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for a, b in ev:
            a.record(stream)
            w.render_band(buf.data_ptr(), width * 4, 0, height, stream.cuda_stream)
            b.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        w.check(stream.cuda_stream)
        kms = sorted(a.elapsed_time(b) for a, b in ev)[len(ev) // 2]
        ent = {"gpu_kernel_ms_median": round(kms, 4),
               "gpu_Mrays_per_s": round(width * height * args.steps / wall / 1e6, 1)}
        if not args.no_cpu:
            o = oracle.VoxelOracle(scene, width, height, tex, dyn, vs.COLORS)
            t0 = time.perf_counter()
            cpu = o.render(threads)
            cpu_s = time.perf_counter() - t0
            ent.update({"cpu_Mrays_per_s": round(width * height / cpu_s / 1e6, 2),
                        "cpu_threads": threads,
                        "bit_identical": bool(np.array_equal(cpu, buf.cpu().numpy().ravel()))})
        res[f"{width}x{height}@{pose[0]}/{pose[1]},{pose[2]}" + ("/ordered" if order else "")] = ent
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
