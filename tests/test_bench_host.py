"""bench.py's host logic (CPU): every timed line names a golden frame that exists, and the
frame check (SHA-256 of the device frame's bytes, hashlib) accepts the golden bytes and
rejects a flipped byte.  The GPU side runs in tests/test_bench_rehearsal.py."""
import json
import os
import zlib

import numpy as np
import torch

import scenes
from conftest import ROOT

GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))


def test_golden_keys_of_bench_lines_exist():
    import bench
    want = {  # (w, h, scene) of every sphere-path line bench.py checks -> golden key
        (3840, 2160, "lcg64"): "c3_3840x2160_lcg64@0,0",
        (1920, 1080, "default10"): "c2_1920x1080_default10@0,0",
        (7680, 4320, "lcg64"): "c4_7680x4320_lcg64@0,0",
        (16384, 16384, "lcg64"): "c5_16384x16384_lcg64@0,0",
        (16384, 16384, "default10"): "c5_16384x16384_default10@0,0",
        (3840, 2160, "lcg256"): "x_3840x2160_lcg256@0,0",
        (3840, 4320, "lcg64"): "w2_3840x4320_lcg64@0,0",
        (3840, 8640, "lcg64"): "w4_3840x8640_lcg64@0,0",
        (3840, 17280, "lcg64"): "w8_3840x17280_lcg64@0,0",
    }
    for (w, h, s), key in want.items():
        assert scenes.golden_key(w, h, s) == key
        assert len(GOLDEN["frames"][key]["sha256"]) == 64
    for frames in bench.EXTRA_FRAMES.values():
        for w, h, s in frames:
            assert scenes.golden_key(w, h, s) in GOLDEN["frames"], (w, h, s)
    for n in (1, 2, 4, 8):  # the headline frame at every GPU count of the SCALE run
        assert scenes.golden_key(bench.WIDTH, bench.ROWS_PER_GPU * n, "lcg64") in GOLDEN["frames"]
    assert scenes.golden_key(3840, 2160, "lcg64", (0.5, 0.0)) is None
    for sec, key in (("all_textures", "3840x2160_lcg64@0,0"), ("glsl", "default@1920x1080"),
                     ("glsl", "default@3840x2160"), ("voxel", "1920x1080@15.5,1.9,15.5/0,0"),
                     ("voxel", "3840x2160@15.5,1.9,15.5/0,0")):
        assert len(GOLDEN[sec][key]["sha256"]) == 64, (sec, key)


def test_verify_frame_against_golden():
    import bench
    g = GOLDEN["frames"]["c1_320x240_one_sphere@0,0"]
    raw = zlib.decompress(open(os.path.join(ROOT, "tests", "golden", g["frame_file"]), "rb").read())
    frame = torch.from_numpy(np.frombuffer(raw, np.uint8).copy()).reshape(240, 320 * 4)
    ok = bench.verify_frame(frame, "frames", "c1_320x240_one_sphere@0,0")
    assert ok == {"golden": "frames/c1_320x240_one_sphere@0,0", "bit_identical": True}
    frame[17, 5] ^= 1
    assert bench.verify_frame(frame, "frames", "c1_320x240_one_sphere@0,0")["bit_identical"] is False
    none = bench.verify_frame(frame, "frames", None)
    assert none["golden"] is None and len(none["sha256"]) == 64
