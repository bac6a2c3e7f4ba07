"""The CPU restatement (oracle/) against the survey's sanity checks and the committed golden
fixtures.

PARITY UNPINNED: the reference cannot be built here (it needs SFML,
SphereWorld.h:3) and ships no tests or fixtures, so nothing pins the oracle to the reference's
own output.  The survey ran the reference TU against a stub SFML and recorded, per config, the
march-iteration statistics of every pixel; reproducing them is a sanity
check of everything up to the shading tail, not a pin.  The shading tail's transcendentals are
checked against the host libm exhaustively (test_math_exhaustive.py).  The survey's frame
hashes from the same stub build do not reproduce (its Image/Color semantics are unrecorded).
tests/golden/ holds hashes generated from the oracle itself (tests/golden/make_golden.py).
"""
import json
import os
import zlib

import numpy as np
import pytest

import oracle
import scenes
from conftest import ROOT, host_threads

GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))

# probe of the unmodified reference (glibc 2.35, g++ -O2).
# Means are compared at the precision the survey quotes them ("mean_decimals").
SURVEY_ITERATIONS = {
    ("c1_320x240_one_sphere", (0.0, 0.0)): {"mean": "2", "max": 2},
    ("c2_1920x1080_default10", (0.0, 0.0)): {"mean": "7.29", "p99": 20, "max": 44},
    ("c2_1920x1080_default10", (0.7, 0.3)): {"mean": "6.50"},
    ("c3_3840x2160_lcg64", (0.0, 0.0)): {"mean": "12.9", "max": 95},
    ("c3_3840x2160_lcg64", (1.1, -0.2)): {"mean": "11.3", "max": 70},
}


@pytest.fixture(scope="module", autouse=True)
def _build():
    oracle.build()


@pytest.mark.parametrize("cfg,pose", list(SURVEY_ITERATIONS))
def test_iteration_statistics_match_reference_probe(floor, cfg, pose):
    width, height, sname, _ = scenes.CONFIGS[cfg]
    o = oracle.Oracle.from_scene(scenes.SCENES[sname]().posed(*pose), width, height, *floor)
    it = o.iteration_map(host_threads())
    want = SURVEY_ITERATIONS[(cfg, pose)]
    decimals = len(want["mean"].split(".")[1]) if "." in want["mean"] else 0
    assert f"{float(it.mean()):.{decimals}f}" == want["mean"]
    if "p99" in want:
        assert int(np.percentile(it, 99)) == want["p99"]
    if "max" in want:
        assert int(it.max()) == want["max"]


# The CPU suite re-renders golden frames up to 8K (a few seconds each on 8 cores); the larger
# ones (16384^2, the 3840 x 8640 / 17280 weak-scaling frames) take minutes on the oracle and
# are checked where they are used: the GPU frame against the hash (test_gpu_parity.py
# test_large_frame_matches_golden_hash, test_gpu_bands.py, bench.py's bit_identical fields).
FRAME_KEYS = sorted(k for k, g in GOLDEN["frames"].items() if g["width"] * g["height"] <= 7680 * 4320)


@pytest.mark.parametrize("key", FRAME_KEYS)
def test_oracle_frame_matches_golden(floor, key):
    g = GOLDEN["frames"][key]
    o = oracle.Oracle.from_scene(scenes.SCENES[g["scene"]]().posed(*g["pose"]), g["width"],
                                 g["height"], *floor)
    frame = o.render(host_threads())
    if "row_fnv1a64" in g:
        rows = frame.reshape(g["height"], -1)
        bad = [j for j in range(g["height"]) if oracle.fnv1a64(rows[j]) != g["row_fnv1a64"][j]]
        assert not bad, f"{key}: {len(bad)} rows differ, first {bad[:5]}"
    assert oracle.fnv1a64(frame) == g["fnv1a64"]
    if "frame_file" in g:
        raw = zlib.decompress(open(os.path.join(ROOT, "tests", "golden", g["frame_file"]), "rb").read())
        assert np.array_equal(np.frombuffer(raw, np.uint8), frame)


def test_oracle_dumps_match_golden(floor):
    for key, dumps in GOLDEN["dumps"].items():
        g = GOLDEN["frames"][key]
        o = oracle.Oracle.from_scene(scenes.SCENES[g["scene"]]().posed(*g["pose"]), g["width"],
                                     g["height"], *floor)
        for d in dumps[:300]:
            got = o.dump(d["i"], d["j"])
            for k in ("draw", "iters", "texel", "rgba"):
                assert got[k] == d[k], (key, d["i"], d["j"], k)
            for k in ("xcoord", "ycoord", "brightness"):
                assert np.float32(got[k]) == np.float32(d[k])


def test_texture_fixture():
    import hashlib
    tex, w, h = scenes.load_floor()
    assert (w, h) == (128, 128)
    assert hashlib.sha256(tex.tobytes()).hexdigest() == GOLDEN["texture_sha256"]
    # 3,376 Floor.png texels are fully transparent
    assert int((tex.reshape(-1, 4)[:, 3] == 0).sum()) == 3376


def test_threads_and_interleave_do_not_change_bytes(floor):
    o = oracle.Oracle.from_scene(scenes.default10().posed(0.7, 0.3), 320, 180, *floor)
    one = o.render(1)
    assert np.array_equal(one, o.render(7))
    # RenderThread: 8 threads x 4 column cycles (Source.cpp:17-28)
    canvas = np.zeros_like(one)
    for t in range(8):
        for cyc in range(4):
            o.update_image(canvas, t, 8, cyc, 4)
    assert np.array_equal(canvas, one)


def test_band_rendering_tiles_frame(floor):
    o = oracle.Oracle.from_scene(scenes.lcg64().posed(0.2, 0.1), 256, 144, *floor)
    full = o.render(1)
    parts = [o.render_band(r0, r1 - r0) for r0, r1 in [(0, 37), (37, 100), (100, 144)]]
    assert np.array_equal(np.concatenate(parts), full)
