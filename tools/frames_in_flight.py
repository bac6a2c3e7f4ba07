"""Frames in flight: wall time per frame of back-to-back frame fills on one HIP stream
(each frame starts when the previous one has drained) against two streams taking frames in
turn (frame k+1 starts while frame k drains; each stream has its own tile-order chain,
sfrt_sched.h TileChains).  Bytes of the last frames compared.
    python tools/frames_in_flight.py [--frames 400]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sfml-software-raytracer_amd"))
import torch  # noqa: E402
import hashlib  # noqa: E402
import scenes  # noqa: E402
import sfrt  # noqa: E402


def run(w, W, H, nstreams, frames, turn, sc):
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    bufs = [torch.empty(H, W * 4, dtype=torch.uint8, device="cuda") for _ in range(nstreams)]
    def go(k):
        if turn:
            w.set_camera(sc.cam_pos, 0.004 * k, 0.0)
        s = streams[k % nstreams]
        w.render_band(bufs[k % nstreams].data_ptr(), W * 4, 0, H, s.cuda_stream)
    for k in range(200):  # settle + chain warm-up
        go(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(frames):
        go(200 + k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for s in streams:
        w.check(s.cuda_stream)
    return dt / frames * 1e6, hashlib.sha256(bufs[(200 + frames - 1) % nstreams].cpu().numpy().tobytes()).hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--order", default="1,2,1,2,1,2", help="stream counts, in run order")
    ap.add_argument("--cases", default="4k,4k_turn,1080")
    a = ap.parse_args()
    w = sfrt.World(0)
    w.load_texture(*scenes.load_floor())
    out = {}
    cases = {"4k": (3840, 2160, "lcg64", False), "4k_turn": (3840, 2160, "lcg64", True),
             "1080": (1920, 1080, "default10", False)}
    for name in a.cases.split(","):
        W, H, sname, turn = cases[name]
        sc = scenes.SCENES[sname]()
        res = {}
        for n in (int(x) for x in a.order.split(",")):
            if True:
                w.set_scene(sc, W, H)
                us, h = run(w, W, H, n, a.frames, turn, sc)
                res.setdefault(f"{n}_stream_us_per_frame", []).append(round(us, 2))
                res.setdefault("last_frame_fnv", set()).add(h)
        res["last_frame_fnv"] = sorted(res["last_frame_fnv"])
        out[name] = res
        print(name, json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
