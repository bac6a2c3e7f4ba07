"""Frames past 2^31 pixels (46400 x 46400: 2.15 G pixels, 8.6 GB of RGBA8 in HBM): every
renderer's indexing runs in 64 bits where a 32-bit pixel index would wrap.  The GPU fills the
whole frame; rows at the top, in the middle and at the bottom (the last ones lie past pixel 2^31)
are compared with the restatements' rows byte for byte."""
import numpy as np
import pytest

import glsl_scenes as gs
import oracle
import scenes
import voxel_scenes as vs
from conftest import poisoned

W = H = 46400
ROWS = [(0, 4), (H // 2 - 2, 4), (H - 8, 8)]
assert W * H > 2 ** 31 and (H - 8) * W > 2 ** 31


def _rows(buf):
    return {r0: buf[r0:r0 + n].cpu().numpy().ravel() for r0, n in ROWS}


@pytest.mark.gpu
def test_sphere_frame_past_2_31_pixels(built, floor):
    import sfrt
    import torch
    sc = scenes.lcg64()
    buf = poisoned((H, W * 4))
    with sfrt.World(0) as world:
        world.load_texture(*floor)
        world.set_scene(sc, W, H)
        for _ in range(3):  # the adaptive tile order in use from the third frame
            world.render_band(buf.data_ptr(), W * 4, 0, H, 0)
        world.check(0)
    got = _rows(buf)
    del buf
    torch.cuda.empty_cache()
    o = oracle.Oracle.from_scene(sc, W, H, *floor)
    for r0, n in ROWS:
        assert np.array_equal(got[r0], o.render_band(r0, n)), f"rows {r0}..{r0 + n}"


@pytest.mark.gpu
def test_glsl_frame_past_2_31_pixels(built, floor):
    import sfrt
    import torch
    u = gs.default_uniforms(W, H, 0.3, 0.1, frames=40)
    buf = poisoned((H, W * 4))
    s = sfrt.GlslShader(0)
    try:
        s.set_ground(*floor)
        s.set_uniforms(u)
        for _ in range(3):
            s.draw(buf.data_ptr(), W, H, W * 4, 0, H, 0)
        s.check(0)
    finally:
        s.close()
    got = _rows(buf)
    del buf
    torch.cuda.empty_cache()
    o = oracle.GlslOracle(u, *floor)
    for r0, n in ROWS:
        assert np.array_equal(got[r0], o.render_band(W, H, r0, n)), f"rows {r0}..{r0 + n}"


@pytest.mark.gpu
def test_voxel_frame_past_2_31_pixels(built):
    import sfrt
    import torch
    tex, dyn = vs.load_textures()
    scene = vs.default_world((20.5, 2.2, 40.5), 1.0, 0.1)
    buf = poisoned((H, W * 4))
    v = sfrt.VoxelWorld(0)
    try:
        v.load_assets(tex, dyn, vs.COLORS)
        v.set_scene(scene, W, H)
        v.render_band(buf.data_ptr(), W * 4, 0, H, 0)
        v.check(0)
    finally:
        v.close()
    got = _rows(buf)
    del buf
    torch.cuda.empty_cache()
    o = oracle.VoxelOracle(scene, W, H, tex, dyn, vs.COLORS)
    full = np.zeros(W * H * 4, np.uint8)  # calloc'd: only the rows the oracle writes are touched
    for r0, n in ROWS:
        for r in range(r0, r0 + n):
            o.update_image(full, r, H, 0, 1)  # UpdateImage's subset: row r alone
        want = full[r0 * W * 4:(r0 + n) * W * 4]
        assert np.array_equal(got[r0], want), f"rows {r0}..{r0 + n}"
