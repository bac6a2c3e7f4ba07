"""A long parity sweep on the GPU, run on demand (SFRT_PARITY_SWEEP=<scenes per renderer>; skipped
otherwise, so the default GPU suite keeps its length): random scenes beyond the seeds the regular
tests use, every frame against the CPU restatement byte for byte --

* sphere world: tests/test_gpu_parity.py `_fuzz_scene` (sphere counts on both sides of every
  kernel switch, cameras at centres / inside / near surfaces / outside, any pose and field of
  view, ragged frames), the default kernel table and, for every fourth scene, 32x8 tiles forced;
  a third of the scenes through render_band with the adaptive tile order, the rest row-major;
* GLSL mode: `glsl_scenes.random_uniforms` (3-60 walls, 0-3 lights, 0-11 balls, a quarter with a
  wide field of view) through the ordered kernel (adaptive tile order, wall cull), and every
  second scene through the row-major kernel (draw_image) as well;
* voxel World: `voxel_scenes.random_world` (grids, billboards, lights and shadows, view distances),
  every second scene with the adaptive tile order.

The summary (scenes, pixels and mismatches per renderer) goes to $SFRT_PARITY_SWEEP_OUT
(profiles/r6ps_parity_sweep.json is one such run).
    SFRT_PARITY_SWEEP=1000 python -m pytest tests/test_parity_sweep.py -m gpu
"""
import json
import os

import numpy as np
import pytest

import glsl_scenes as gs
import voxel_scenes as vs
from conftest import host_threads, poisoned

N = int(os.environ.get("SFRT_PARITY_SWEEP", "0"))
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(N <= 0, reason="on demand: SFRT_PARITY_SWEEP=<scenes per renderer>")]
RESULTS = {}


def _progress(name, i, bad):
    if i % 25 == 0:  # a line now and then: a long sweep must not look hung
        print(f"{name}: {i} of {N} scenes, {len(bad)} mismatched", flush=True)


def _record(name, scenes, pixels, bad):
    RESULTS[name] = {"scenes": scenes, "pixels": pixels, "mismatched_scenes": bad}
    out = os.environ.get("SFRT_PARITY_SWEEP_OUT")
    if out:
        with open(out, "w") as f:
            json.dump({"per_renderer": RESULTS, "scenes_per_renderer": N}, f, indent=1)


def test_sphere_sweep(built, floor):
    import oracle
    import sfrt
    from test_gpu_parity import _fuzz_scene, diff_report
    bad, pixels = [], 0
    with sfrt.World(0) as world:
        world.load_texture(*floor)
        for seed in range(20000, 20000 + N):
            sc, w, h = _fuzz_scene(seed)
            world.set_option(sfrt.SFRT_OPT_RAYS_PER_LANE, 4 if seed % 4 == 0 else 0)
            world.set_scene(sc, w, h)
            if seed % 3 == 1:  # render_band: the adaptive tile order in use from the third frame
                b = poisoned((h, w * 4))
                for _ in range(3):
                    world.render_band(b.data_ptr(), w * 4, 0, h, 0)
                world.check(0)
                got = b.cpu().numpy().ravel()
            else:  # update_image: row-major
                got = world.render()
            want = oracle.Oracle.from_scene(sc, w, h, *floor).render(host_threads())
            msg = diff_report(got, want, w)
            if msg:
                bad.append({"seed": seed, "diff": msg})
            pixels += w * h
            _progress("sphere", seed - 20000 + 1, bad)
    _record("sphere", N, pixels, bad)
    assert not bad, bad[:3]


def test_glsl_sweep(built, floor):
    import oracle
    import sfrt
    rng = np.random.default_rng(20000)
    bad, pixels = [], 0
    s = sfrt.GlslShader(0)
    try:
        s.set_ground(*floor)
        for seed in range(20000, 20000 + N):
            nw, nl, nb = int(rng.integers(3, 61)), int(rng.integers(0, 4)), int(rng.integers(0, 12))
            w, h = [(160, 90), (96, 64), (133, 47)][seed % 3]
            u = gs.random_uniforms(seed, nw, nl, nb, w, h)
            if seed % 4 == 0:
                u["fov"] = (np.float32(rng.uniform(1.5, 2.6)), np.float32(rng.uniform(1.0, 2.0)))
            s.set_uniforms(u)
            b = poisoned((h, w * 4))
            for _ in range(3):  # the adaptive order in use from the third draw
                s.draw(b.data_ptr(), w, h, w * 4, 0, h, 0)
            s.check(0)
            got = b.cpu().numpy().ravel()
            want = oracle.GlslOracle(u, *floor).render(w, h, host_threads())
            if not np.array_equal(got, want):
                n = int(np.count_nonzero(np.any(got.reshape(-1, 4) != want.reshape(-1, 4), axis=1)))
                bad.append({"seed": seed, "walls": nw, "pixels_differ": n})
            elif seed % 2 == 1:  # and the row-major kernel without the wall cull (draw_image)
                got = s.draw_image(w, h)
                if not np.array_equal(got, want):
                    n = int(np.count_nonzero(np.any(got.reshape(-1, 4) != want.reshape(-1, 4), axis=1)))
                    bad.append({"seed": seed, "walls": nw, "pixels_differ": n, "kernel": "row-major"})
            pixels += w * h
            _progress("glsl", seed - 20000 + 1, bad)
    finally:
        s.close()
    _record("glsl", N, pixels, bad)
    assert not bad, bad[:3]


def test_voxel_sweep(built):
    import oracle
    import sfrt
    tex, dyn = vs.load_textures()
    bad, pixels = [], 0
    v = sfrt.VoxelWorld(0)
    try:
        v.load_assets(tex, dyn, vs.COLORS)
        for seed in range(20000, 20000 + N):
            scene, w, h = vs.random_world(seed)
            v.set_option(sfrt.SFRT_OPT_TILE_ORDER, seed % 2)  # off by default; on: LPT order
            v.set_scene(scene, w, h)
            b = poisoned((h, w * 4))
            for _ in range(1 + 2 * (seed % 2)):  # the order in use from the third frame
                v.render_band(b.data_ptr(), w * 4, 0, h, 0)
            v.check(0)
            got = b.cpu().numpy().ravel()
            want = oracle.VoxelOracle(scene, w, h, tex, dyn, vs.COLORS).render(host_threads())
            if not np.array_equal(got, want):
                n = int(np.count_nonzero(np.any(got.reshape(-1, 4) != want.reshape(-1, 4), axis=1)))
                bad.append({"seed": seed, "pixels_differ": n})
            pixels += w * h
            _progress("voxel", seed - 20000 + 1, bad)
    finally:
        v.close()
    _record("voxel", N, pixels, bad)
    assert not bad, bad[:3]
