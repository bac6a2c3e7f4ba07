"""Per-sphere texture extension ("64 spheres + all textures").

The reference samples textures[0] only (SphereWorld.cpp:376-377); the
extension gives every sphere a texture slot (default 0 = the reference).
CPU: slot 0 everywhere reproduces the reference frame; the all-textures
frames match their golden hashes.  GPU: the kernel equals the oracle with
every texture resident, and slots travel with their spheres through
AddSphere / UpdateSpheres.
"""
import json
import os

import numpy as np
import pytest

import oracle
import scenes
from conftest import ROOT, host_threads

GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
# the 4K pose (0, 0) case is bench.py's "3840x2160_lcg64_all_textures" line
CASES = [(1920, 1080, (0.0, 0.0)), (3840, 2160, (1.1, -0.2)), (3840, 2160, (0.0, 0.0))]


def key(w, h, pose):
    return f"{w}x{h}_lcg64@{pose[0]:g},{pose[1]:g}"


def tex_oracle(w, h, pose, slots=None):
    tex = scenes.load_all_textures()
    scene = scenes.lcg64().posed(*pose)
    n = scene.spheres.shape[0]
    slots = scenes.all_texture_slots(n) if slots is None else slots
    return oracle.Oracle(w, h, scene.spheres, *tex[0], scene.cam_pos, scene.rotation,
                         scene.hrotation, scene.fov_h, scene.fov_v, sphere_tex=slots,
                         textures={k: tex[k] for k in range(1, len(tex))})


def test_slot_zero_is_the_reference():
    w, h = 320, 180
    scene = scenes.lcg64()
    floor = scenes.load_floor()
    ref = oracle.Oracle.from_scene(scene, w, h, *floor).render(host_threads())
    ext = tex_oracle(w, h, (0.0, 0.0), np.zeros(scene.spheres.shape[0], np.int32))
    assert np.array_equal(ext.render(host_threads()), ref)
    assert not np.array_equal(tex_oracle(w, h, (0.0, 0.0)).render(host_threads()), ref)


@pytest.mark.parametrize("case", CASES[:1], ids=[key(*c) for c in CASES[:1]])
def test_oracle_all_textures_golden(case):
    frame = tex_oracle(*case).render(host_threads())
    assert oracle.fnv1a64(frame) == GOLDEN["all_textures"][key(*case)]["fnv1a64"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[key(*c) for c in CASES])
def test_gpu_all_textures(built, case):
    import sfrt
    w, h, pose = case
    tex = scenes.load_all_textures()
    with sfrt.World(0) as world:
        for slot, (rgba, tw, th) in enumerate(tex):
            world.load_texture(rgba, tw, th, slot=slot)
        world.set_scene(scenes.lcg64().posed(*pose), w, h)
        world.set_sphere_textures(scenes.all_texture_slots(64))
        got = world.render()
    want = tex_oracle(w, h, pose).render(host_threads())
    assert np.array_equal(got, want)
    assert oracle.fnv1a64(got) == GOLDEN["all_textures"][key(*case)]["fnv1a64"]


@pytest.mark.gpu
def test_gpu_slots_follow_their_spheres(built):
    """AddSphere prunes and UpdateSpheres re-sorts; each slot stays with its sphere."""
    import sfrt
    tex = scenes.load_all_textures()
    with sfrt.World(0) as world:
        for slot, (rgba, tw, th) in enumerate(tex):
            world.load_texture(rgba, tw, th, slot=slot)
        world.set_size(320, 180)
        for s in scenes.lcg_spheres(20, 777):
            world.add_sphere(*s)
        sph = world.spheres.copy()
        slots = (np.arange(sph.shape[0]) * 7 % 6).astype(np.int32)
        world.set_sphere_textures(slots)
        tagged = {tuple(s): int(k) for s, k in zip(sph.tolist(), slots)}
        world.set_camera((3.0, 1.0, -2.0), 0.3, 0.1)
        world.update_spheres()
        world.add_sphere(0.5, 0.5, 0.5, 1.0)   # new sphere: slot 0
        after = dict(zip(map(tuple, world.spheres.tolist()), world.sphere_textures.tolist()))
        for s, k in after.items():
            assert k == tagged.get(s, 0)
        with pytest.raises(sfrt.SfrtError):
            world.set_sphere_textures(np.zeros(3, np.int32))           # wrong count
        bad = world.sphere_textures
        bad[0] = 9                                                      # slot never loaded
        world.set_sphere_textures(bad)
        with pytest.raises(sfrt.SfrtError, match="NO_TEXTURE"):
            world.render()
