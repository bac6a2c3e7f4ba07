"""Packed band transfer kernels (csrc/band_pack.hip) on one GPU: time per band and HBM rate.

Algorithmic bytes per pixel: pack reads 4 and writes 3.125, unpack reads 3.125 and writes 4
(7.125 B per pixel each way).  Bands: a 4K frame's rows at N = 8 (1646-row bands at the
~3.5 root factor DESIGN.md 7 models), a 4K band, and a 16384^2 frame's 2048-row band.
Prints one JSON object."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sfml-software-raytracer_amd"))
import sfrt  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    stream = torch.cuda.Stream()
    out = {}
    for w, h in ((3840, 1646), (3840, 2160), (16384, 2048)):
        p = w * h
        rng = np.random.default_rng(p)
        by = rng.integers(0, 256, size=(p, 4), dtype=np.uint8)
        by[:, 3] = rng.choice(np.array([0, 255], np.uint8), size=p)
        src = torch.from_numpy(by.ravel()).cuda()
        packed = torch.empty(sfrt.band_packed_bytes(p), dtype=torch.uint8, device="cuda")
        back = torch.empty_like(src)
        res = {}
        for name, fn in (("pack", lambda: sfrt.band_pack(src.data_ptr(), p, packed.data_ptr(),
                                                          stream.cuda_stream)),
                         ("unpack", lambda: sfrt.band_unpack(packed.data_ptr(), p, back.data_ptr(),
                                                             stream.cuda_stream))):
            for _ in range(20):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 200
            e0.record(stream)
            for _ in range(n):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / n * 1e3
            gbs = 7.125 * p / (us * 1e-6) / 1e9
            res[name] = {"us": round(us, 2), "GB_per_s": round(gbs, 1),
                         "hbm_frac": round(gbs / HBM_PEAK_GBS, 3)}
        torch.cuda.synchronize()
        res["round_trip_exact"] = bool(torch.equal(src, back))
        res["wire_bytes"] = {"rgba8": 4 * p, "packed": sfrt.band_packed_bytes(p)}
        out[f"{w}x{h}"] = res
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
