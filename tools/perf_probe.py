"""Kernel-time ablations in one process (HIP events on one stream), e.g.
    python tools/perf_probe.py            # default variant table
    SFRT_LIB=path/to/other/libsfrt.so python tools/perf_probe.py   # a build-flag A/B
Variants isolate the kernel's phases without changing its code:
  march       = scene as given (setup + cull + march + shade)
  nocull      = SFRT_OPT_CULL 0 (every sphere visited)
  outside     = camera outside every sphere -> first iteration ends the march
                (setup + cull + shade only)
  outside_nc  = outside + cull off (setup + shade only)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sfml-software-raytracer_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import scenes  # noqa: E402
import sfrt  # noqa: E402


def time_kernel(w, buf, width, height, reps, stream):
    for _ in range(3):
        w.render_band(buf.data_ptr(), width * 4, 0, height, stream.cuda_stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        w.render_band(buf.data_ptr(), width * 4, 0, height, stream.cuda_stream)
        b.record(stream)
    torch.cuda.synchronize()
    w.check(stream.cuda_stream)
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2], t[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="march,nocull,outside,outside_nc")
    ap.add_argument("--rays", default="0",
                    help="comma list of SFRT_OPT_RAYS_PER_LANE values (0 = the kernel table's "
                         "choice), interleaved per round")
    ap.add_argument("--orders", default="1",
                    help="comma list of SFRT_OPT_TILE_ORDER values (1 adaptive, 0 row-major); "
                         "keys get /o0 for row-major")
    ap.add_argument("--big", action="store_true", help="add the 7680x4320 frame")
    args = ap.parse_args()
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    floor = scenes.load_floor()
    w = sfrt.World(0)
    w.load_texture(*floor)
    out = {}
    cases = [("4k_lcg64", 3840, 2160, scenes.lcg64()),
             ("4k_lcg64_rot", 3840, 2160, scenes.lcg64().posed(1.1, -0.2)),
             ("1080_default10", 1920, 1080, scenes.default10())]
    if args.big:
        cases.append(("8k_lcg64", 7680, 4320, scenes.lcg64()))
    buf = torch.empty(4320 if args.big else 2160, (7680 if args.big else 3840) * 4,
                      dtype=torch.uint8, device="cuda")
    for rnd in range(args.rounds):
        for name, width, height, sc in cases:
            outside = scenes.Scene(sc.name, sc.spheres, cam_pos=(0.0, 200.0, 0.0),
                                   rotation=sc.rotation, hrotation=sc.hrotation)
            allv = (("march", sc, 1), ("nocull", sc, 0), ("outside", outside, 1),
                    ("outside_nc", outside, 0))
            for var, scene, cull in (v for v in allv if v[0] in args.variants.split(",")):
                for kv in [int(x) for x in args.rays.split(",")]:
                    for order in [int(x) for x in args.orders.split(",")]:
                        w.set_scene(scene, width, height)
                        w.set_option(sfrt.SFRT_OPT_CULL, cull)
                        w.set_option(sfrt.SFRT_OPT_RAYS_PER_LANE, kv)
                        w.set_option(sfrt.SFRT_OPT_TILE_ORDER, order)
                        med, best = time_kernel(w, buf, width, height, args.reps, stream)
                        tag = "" if order else "/o0"
                        out.setdefault(f"{name}/{var}/r{kv}{tag}", []).append(round(med * 1e3, 2))
    w.set_option(sfrt.SFRT_OPT_CULL, 1)
    w.set_option(sfrt.SFRT_OPT_RAYS_PER_LANE, 0)
    w.set_option(sfrt.SFRT_OPT_TILE_ORDER, 1)
    for k, v in out.items():
        print(f"{k:32s} us(median per round) {v}")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
