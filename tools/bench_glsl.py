"""GLSL renderer throughput on MI355X vs the CPU
restatement on the host cores, same frames, bytes compared.

    python tools/bench_glsl.py [--steps 30]
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

import glsl_scenes as gs  # noqa: E402
import scenes  # noqa: E402
import sfrt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--orders", default="1",
                    help="SFRT_OPT_TILE_ORDER values (1 adaptive = the library's default since "
                         "round 4, 0 row-major; keys of 0 get /rowmajor)")
    ap.add_argument("--set", choices=("all", "bench"), default="all",
                    help="bench: only the two frames bench.py times (1080p and 4K, rot (0,0)), "
                         "one frame per launch size (rocprof summaries per launch size)")
    args = ap.parse_args()
    import oracle  # CPU baseline / checker only
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    floor = scenes.load_floor()
    s = sfrt.GlslShader(0)
    s.set_ground(*floor)
    res = {}
    threads = max(1, min(16, os.cpu_count() or 1))
    cases = [(1920, 1080, (0.0, 0.0), 0), (3840, 2160, (0.0, 0.0), 0), (3840, 2160, (5.5, -0.4), 300)]
    for width, height, rot, frames in (cases[:2] if args.set == "bench" else cases):
        u = gs.default_uniforms(width, height, *rot, frames=frames)
        s.set_uniforms(u)
        buf = torch.empty(height, width * 4, dtype=torch.uint8, device="cuda")
        for order in [int(v) for v in args.orders.split(",")]:
            s.set_option(sfrt.SFRT_OPT_TILE_ORDER, order)
            r = time_one(s, buf, width, height, u, rot, frames, 0, args, stream, floor,
                         threads, oracle)
            res.update({(k + ("" if order else "/rowmajor")): v for k, v in r.items()})
        s.set_option(sfrt.SFRT_OPT_TILE_ORDER, 1)
    print(json.dumps(res, indent=1))


def time_one(s, buf, width, height, u, rot, frames, var, args, stream, floor, threads, oracle):
    """Kernel time (HIP events, median) and wall rate of one frame size and variant."""
    for _ in range(3):
        s.draw(buf.data_ptr(), width, height, width * 4, 0, height, stream.cuda_stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        s.draw(buf.data_ptr(), width, height, width * 4, 0, height, stream.cuda_stream)
        b.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    s.check(stream.cuda_stream)
    kms = sorted(a.elapsed_time(b) for a, b in ev)[len(ev) // 2]
    ent = {"gpu_kernel_ms_median": round(kms, 4),
           "gpu_Mfrags_per_s": round(width * height * args.steps / wall / 1e6, 1),
           "gpu_Mfrags_per_s_kernel": round(width * height / kms / 1e3, 1)}
    if not args.no_cpu:
        o = oracle.GlslOracle(u, *floor)
        t0 = time.perf_counter()
        cpu = o.render(width, height, threads)
        cpu_s = time.perf_counter() - t0
        ent.update({"cpu_Mfrags_per_s": round(width * height / cpu_s / 1e6, 2),
                    "cpu_threads": threads,
                    "bit_identical": bool(np.array_equal(cpu, buf.cpu().numpy().ravel()))})
    return {f"{width}x{height}@{rot[0]:g},{rot[1]:g}/frames{frames}": ent}


if __name__ == "__main__":
    main()
