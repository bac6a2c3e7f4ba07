"""A long parity sweep on the GPU, run on demand (SFRT_PARITY_SWEEP=<scenes per renderer>; skipped
otherwise, so the default GPU suite keeps its length): random scenes beyond the seeds the regular
tests use, every frame against the CPU restatement byte for byte --

* sphere world: tests/test_gpu_parity.py `_fuzz_scene` (sphere counts on both sides of every
  kernel switch, cameras at centres / inside / near surfaces / outside, any pose and field of
  view, ragged frames), the default kernel table and, for every fourth scene, 32x8 tiles forced;
  a third of the scenes through render_band with the adaptive tile order, the rest row-major;
  every seventh with random per-sphere texture slots (the "all textures" extension), every sixth
  drawn as an UpdateImage pixel subset on a poisoned canvas;
* GLSL mode: `glsl_scenes.random_uniforms` (3-60 walls, 0-3 lights, 0-11 balls, a quarter with a
  wide field of view) through the ordered kernel (adaptive tile order, wall cull), and every
  second scene through the row-major kernel (draw_image) as well; every fourth scene is instead
  the reference's own world after 0-600 UpdateWorld steps, in any pose;
* voxel World: `voxel_scenes.random_world` (grids, billboards, lights and shadows, view distances),
  every second scene with the adaptive tile order; every fourth scene is instead the reference's
  default world seen from a random empty cell.

* the multi-GPU object (sfrt_multi): N / 10 sphere scenes over 2-4 ranks on cuda:0.

Every fifth scene is drawn as 2-4 random row bands (global row indices, as the multi-GPU bands).
SFRT_PARITY_SWEEP_MODE=adversarial pushes each generator to its degenerate corners;
SFRT_PARITY_SWEEP_SIZE=WxH draws every scene at that size.  The summary (scenes, pixels and
mismatches per renderer) goes to $SFRT_PARITY_SWEEP_OUT (profiles/r6ps_*, r6pa_*, r6p1_*, r6p4_*,
r6pm_* are such runs).
    SFRT_PARITY_SWEEP=1000 python -m pytest tests/test_parity_sweep.py -m gpu -s
"""
import json
import os

import numpy as np
import pytest

import glsl_scenes as gs
import voxel_scenes as vs
from conftest import host_threads, poisoned

N = int(os.environ.get("SFRT_PARITY_SWEEP", "0"))
# "adversarial": the same generators pushed to their degenerate corners (below)
MODE = os.environ.get("SFRT_PARITY_SWEEP_MODE", "random")
SEED0 = 20000 if MODE == "random" else 50000
# "WxH": every scene at that frame size instead of the generators' small ragged ones (a 4K
# sweep reaches the kernels' large-frame choices: 32x8 tiles by the tile count, ordered launches)
SIZE = tuple(int(v) for v in os.environ["SFRT_PARITY_SWEEP_SIZE"].split("x")) \
    if os.environ.get("SFRT_PARITY_SWEEP_SIZE") else None
if SIZE:
    SEED0 += 100000
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(N <= 0, reason="on demand: SFRT_PARITY_SWEEP=<scenes per renderer>")]
RESULTS = {}


def _progress(name, i, bad):
    if i % 25 == 0 or SIZE:  # a line now and then: a long sweep must not look hung
        print(f"{name}: {i} of {N} scenes, {len(bad)} mismatched", flush=True)


def _record(name, scenes, pixels, bad, skipped=0):
    RESULTS[name] = {"scenes": scenes, "pixels": pixels, "mismatched_scenes": bad,
                     "skipped_march_cap_both_sides": skipped, "mode": MODE}
    _record_flush()


def _record_flush():
    out = os.environ.get("SFRT_PARITY_SWEEP_OUT")
    if out:
        with open(out, "w") as f:
            json.dump({"per_renderer": RESULTS, "scenes_per_renderer": N}, f, indent=1)


def _bands(seed, h):
    """Row bands [(row0, rows), ...] of an h-row frame: 2-4 random cuts for every fifth scene
    (seed % 5 == 2; global row indices, as the multi-GPU bands use them), else the whole frame."""
    if seed % 5 != 2 or h < 4:
        return [(0, h)]
    rng = np.random.default_rng(seed + 3)
    cuts = sorted(set(int(c) for c in rng.integers(1, h, int(rng.integers(1, 4)))))
    edges = [0] + cuts + [h]
    return [(a, b - a) for a, b in zip(edges, edges[1:])]


F = np.float32
QUARTER_TURNS = [F(0.0), F(np.pi / 2), F(np.pi), F(-np.pi / 2), F(2 * np.pi)]


def _sphere_adversarial(seed):
    """_fuzz_scene pushed to degenerate corners: integer centres and radii with the camera at a
    centre, on a surface or at a tangent point; spheres tangent to each other or duplicated;
    radii at the 0.01 pass threshold; huge coordinates; quarter-turn poses (axis-parallel
    rays); tiny or very wide fields of view."""
    from test_gpu_parity import _fuzz_scene
    sc, w, h = _fuzz_scene(seed)
    rng = np.random.default_rng(seed + 7)
    sp = np.array(sc.spheres, dtype=F)
    n = sp.shape[0]
    if rng.random() < 0.5:
        sp = np.round(sp).astype(F)
        sp[:, 3] = np.maximum(sp[:, 3], F(1))
    if rng.random() < 0.3 and n > 1:  # tangent pairs along an axis
        for k in range(1, n, 2):
            ax = int(rng.integers(3))
            sp[k, :3] = sp[k - 1, :3]
            sp[k, ax] = F(sp[k - 1, ax] + sp[k - 1, 3] + sp[k, 3])
    if rng.random() < 0.2 and n > 1:  # duplicates
        sp[n // 2:] = sp[: n - n // 2]
    if rng.random() < 0.2:  # radii at the pass threshold
        sp[rng.random(n) < 0.3, 3] = rng.choice([F(0.01), np.nextafter(F(0.01), F(1)), F(0.02)])
    if rng.random() < 0.1:  # huge coordinates
        sp[:, :3] *= F(1000)
        sp[:, 3] *= F(rng.choice([1.0, 1000.0]))
    k = int(rng.integers(n))
    cam = np.array(sc.cam_pos, dtype=F)
    pick = rng.random()
    if pick < 0.25:
        cam = sp[k, :3].copy()                                   # at a centre
    elif pick < 0.5:
        cam = sp[k, :3].copy()
        cam[int(rng.integers(3))] += sp[k, 3] * F(rng.choice([1, -1]))  # on the surface
    elif pick < 0.6:
        cam = np.round(cam).astype(F)
    sc.spheres = sp
    sc.cam_pos = tuple(float(x) for x in cam)
    if rng.random() < 0.4:
        sc.rotation = float(rng.choice(QUARTER_TURNS))
        sc.hrotation = float(rng.choice([F(0.0), F(np.pi / 2), F(-np.pi / 2), F(0.0)]))
    if rng.random() < 0.15:
        sc.fov_h, sc.fov_v = F(rng.choice([1e-4, 2.9])), F(rng.choice([1e-4, 1.5]))
    return sc, w, h


def _glsl_adversarial(seed, w, h):
    """random_uniforms pushed to degenerate corners: positions and radii on a 0.5 grid; shadow
    balls on the segment from a light to the camera (cosines at -1 and 1); a shadow ball on a
    light; zero radii; duplicated balls; the camera at a wall centre or with -0.0 components;
    quarter-turn poses."""
    rng = np.random.default_rng(seed)
    nw, nl, nb = int(rng.integers(1, 20)), int(rng.integers(0, 4)), int(rng.integers(0, 12))
    u = gs.random_uniforms(seed, nw, nl, nb, w, h)
    sc, lc, al = int(u["sphere_count"]), int(u["light_count"]), int(u["all_spheres_count"])
    S = u["spheres"]
    if rng.random() < 0.4:
        S[:al] = (np.round(S[:al] * 2) / 2).astype(F)
        S[:sc, 3] = np.maximum(S[:sc, 3], F(1))
    cam = np.array(u["campos"], dtype=F)
    if lc and al > sc + lc and rng.random() < 0.6:
        for j in range(sc + lc, al):
            i = sc + int(rng.integers(lc))
            t = F(rng.choice([0.25, 0.5, 0.75, 1.5]))
            S[j, :3] = (S[i, :3] + t * (cam - S[i, :3])).astype(F)
    if lc and al > sc + lc and rng.random() < 0.15:
        S[sc + lc, :3] = S[sc, :3]                      # a shadow ball on a light
    if al > sc and rng.random() < 0.15:
        S[sc + int(rng.integers(al - sc)), 3] = F(0)   # zero radius
    if al > sc + 1 and rng.random() < 0.15:
        S[al - 1] = S[al - 2]                           # duplicate
    if rng.random() < 0.15:
        cam = S[int(rng.integers(sc)), :3].copy()       # at a wall centre
    if rng.random() < 0.1:
        cam = np.array([-0.0, cam[1], -0.0], dtype=F)
    u["campos"] = cam
    if rng.random() < 0.4:
        u["rotation"] = (rng.choice(QUARTER_TURNS), F(rng.choice([0.0, 0.0, 0.5])))
    return u, nw


def _voxel_adversarial(seed):
    """random_world with the camera on cell boundaries (integer and half coordinates),
    quarter-turn and zero-tilt poses, lights on cell corners, long view distances."""
    scene, w, h = vs.random_world(seed)
    rng = np.random.default_rng(seed + 11)
    cam = np.array(scene.cam_pos, dtype=F)
    if rng.random() < 0.5:
        cam = (np.floor(cam) + F(rng.choice([0.0, 0.5]))).astype(F)
    scene.cam_pos = tuple(float(x) for x in cam)
    if rng.random() < 0.5:
        scene.rotation = float(rng.choice(QUARTER_TURNS))
        scene.hrotation = float(rng.choice([F(0.0), F(0.5), F(-0.5)]))
    if scene.lights.shape[0] and rng.random() < 0.5:
        scene.lights["pos"] = np.round(scene.lights["pos"])
    if rng.random() < 0.3:
        scene.view_distance = 64.0
    return scene, w, h


def test_sphere_sweep(built, floor):
    import oracle
    import sfrt
    from test_gpu_parity import _fuzz_scene, diff_report
    import scenes
    bad, pixels = [], 0
    tex = scenes.load_all_textures()  # slot 0 is the floor (the reference's textures[0])
    with sfrt.World(0) as world:
        for slot, (rgba, tw, th) in enumerate(tex):
            world.load_texture(rgba, tw, th, slot=slot)
        for seed in range(SEED0, SEED0 + N):
            sc, w, h = _fuzz_scene(seed) if MODE == "random" else _sphere_adversarial(seed)
            w, h = SIZE or (w, h)
            world.set_option(sfrt.SFRT_OPT_RAYS_PER_LANE, 4 if seed % 4 == 0 else 0)
            world.set_scene(sc, w, h)
            n = np.asarray(sc.spheres).shape[0]
            # every seventh scene with the per-sphere texture slots (the "all textures" extension)
            slots = np.random.default_rng(seed).integers(0, len(tex), n).astype(np.int32) \
                if seed % 7 == 3 else np.zeros(n, np.int32)
            world.set_sphere_textures(slots)
            try:
                if seed % 3 == 1 or seed % 5 == 2:  # render_band (the adaptive tile order in use
                    b = poisoned((h, w * 4))        # from the third frame), in row bands at times
                    for _ in range(3):
                        for r0, n in _bands(seed, h):
                            world.render_band(b[r0].data_ptr(), w * 4, r0, n, 0)
                    world.check(0)
                    got = b.cpu().numpy().ravel()
                elif seed % 6 == 5:  # an UpdateImage pixel subset on a poisoned canvas
                    sub = np.random.default_rng(seed + 5).integers(1, 5, 2)
                    got = np.full(w * h * 4, 0xA5, np.uint8)
                    subset = (int(seed % int(sub[0])), int(sub[0]), int(seed % int(sub[1])), int(sub[1]))
                    world.update_image(got, *subset)
                else:  # update_image: row-major
                    got = world.render()
            except sfrt.SfrtError as e:  # the kernel's march cap or texel check
                bad.append({"seed": seed, "error": str(e)})
                continue
            if seed % 7 == 3:
                o = oracle.Oracle(w, h, sc.spheres, *tex[0], sc.cam_pos, sc.rotation, sc.hrotation,
                                  sc.fov_h, sc.fov_v, sphere_tex=slots,
                                  textures={k: tex[k] for k in range(1, len(tex))})
            else:
                o = oracle.Oracle.from_scene(sc, w, h, *floor)
            if seed % 6 == 5 and seed % 3 != 1 and seed % 5 != 2:
                want = np.full(w * h * 4, 0xA5, np.uint8)
                o.update_image(want, *subset)
            else:
                want = o.render(host_threads())
            msg = diff_report(got, want, w)
            if msg:
                bad.append({"seed": seed, "diff": msg})
            pixels += w * h
            _progress("sphere", seed - SEED0 + 1, bad)
    _record("sphere", N, pixels, bad)
    assert not bad, bad[:3]


def test_glsl_sweep(built, floor):
    import oracle
    import sfrt
    rng = np.random.default_rng(SEED0)
    bad, pixels, skipped = [], 0, 0
    sw = gs.ShaderWorld(0)  # the constructor's world, then UpdateWorld steps (Source.cpp:129)
    world_frames = []
    for _ in range(600):
        world_frames.append(sw.uniforms(16, 16))
        sw.update_world()
    s = sfrt.GlslShader(0)
    try:
        s.set_ground(*floor)
        for seed in range(SEED0, SEED0 + N):
            nw, nl, nb = int(rng.integers(3, 61)), int(rng.integers(0, 4)), int(rng.integers(0, 12))
            w, h = SIZE or [(160, 90), (96, 64), (133, 47)][seed % 3]
            if seed % 4 == 1:  # the reference's own world after k UpdateWorld steps, any pose
                u = world_frames[int(rng.integers(0, len(world_frames)))].copy()
                u["rotation"] = (np.float32(rng.uniform(0, 6.28)), np.float32(rng.uniform(-0.6, 0.6)))
                u["size"] = (np.float32(w), np.float32(h))
            elif MODE == "random":
                u = gs.random_uniforms(seed, nw, nl, nb, w, h)
            else:
                u, nw = _glsl_adversarial(seed, w, h)
            if seed % 4 == 0:
                u["fov"] = (np.float32(rng.uniform(1.5, 2.6)), np.float32(rng.uniform(1.0, 2.0)))
            s.set_uniforms(u)
            b = poisoned((h, w * 4))
            for _ in range(3):  # the adaptive order in use from the third draw; row bands at times
                for r0, n in _bands(seed, h):
                    s.draw(b[r0].data_ptr(), w, h, w * 4, r0, n, 0)
            try:
                want = oracle.GlslOracle(u, *floor).render(w, h, host_threads())
            except RuntimeError:  # the restatement's march cap: no defined frame to compare
                want = None
            try:
                s.check(0)
            except RuntimeError:
                if want is None:
                    skipped += 1
                    continue
                raise
            if want is None:
                bad.append({"seed": seed, "walls": nw, "oracle": "march cap"})
                continue
            got = b.cpu().numpy().ravel()
            if not np.array_equal(got, want):
                n = int(np.count_nonzero(np.any(got.reshape(-1, 4) != want.reshape(-1, 4), axis=1)))
                bad.append({"seed": seed, "walls": nw, "pixels_differ": n})
            elif seed % 2 == 1:  # and the row-major kernel without the wall cull (draw_image)
                got = s.draw_image(w, h)
                if not np.array_equal(got, want):
                    n = int(np.count_nonzero(np.any(got.reshape(-1, 4) != want.reshape(-1, 4), axis=1)))
                    bad.append({"seed": seed, "walls": nw, "pixels_differ": n, "kernel": "row-major"})
            pixels += w * h
            _progress("glsl", seed - SEED0 + 1, bad)
    finally:
        s.close()
    _record("glsl", N, pixels, bad, skipped)
    assert not bad, bad[:3]


def test_voxel_sweep(built):
    import oracle
    import sfrt
    tex, dyn = vs.load_textures()
    bad, pixels, ub = [], 0, 0
    v = sfrt.VoxelWorld(0)
    try:
        v.load_assets(tex, dyn, vs.COLORS)
        for seed in range(SEED0, SEED0 + N):
            if seed % 4 == 1:  # the reference's default world from a random empty cell and pose
                r4 = np.random.default_rng(seed)
                blocks = vs.default_blocks()
                while True:
                    c = (int(r4.integers(1, 99)), int(r4.integers(1, 9)), int(r4.integers(1, 99)))
                    if blocks[c] == vs.EMPTY:
                        break
                scene = vs.default_world(tuple(float(F(c[k] + r4.uniform(0.05, 0.95))) for k in range(3)),
                                         float(r4.uniform(0, 6.28)), float(r4.uniform(-0.6, 0.6)))
                w, h = [(320, 180), (256, 144), (333, 187)][seed % 3]
            else:
                scene, w, h = vs.random_world(seed) if MODE == "random" else _voxel_adversarial(seed)
            w, h = SIZE or (w, h)
            v.set_option(sfrt.SFRT_OPT_TILE_ORDER, seed % 2)  # off by default; on: LPT order
            v.set_scene(scene, w, h)
            b = poisoned((h, w * 4))
            for _ in range(1 + 2 * (seed % 2)):  # the order in use from the third frame
                for r0, n in _bands(seed, h):
                    v.render_band(b[r0].data_ptr(), w * 4, r0, n, 0)
            flagged = False
            try:
                v.check(0)
            except sfrt.SfrtError as e:  # SFRT_E_TEXEL: the reference reads outside a texture
                if e.code != -7:  # SFRT_E_TEXEL
                    bad.append({"seed": seed, "error": str(e)})
                    continue
                flagged = True
            got = b.cpu().numpy().ravel()
            before = oracle.VoxelOracle.bad_texel_reads()
            want = oracle.VoxelOracle(scene, w, h, tex, dyn, vs.COLORS).render(host_threads())
            oob = oracle.VoxelOracle.bad_texel_reads() > before
            if flagged != oob:  # both read the same stand-in texel, and both must say so
                bad.append({"seed": seed, "texel_outside": {"gpu": flagged, "oracle": oob}})
            elif flagged:
                ub += 1
            if not np.array_equal(got, want):
                n = int(np.count_nonzero(np.any(got.reshape(-1, 4) != want.reshape(-1, 4), axis=1)))
                bad.append({"seed": seed, "pixels_differ": n})
            pixels += w * h
            _progress("voxel", seed - SEED0 + 1, bad)
    finally:
        v.close()
    _record("voxel", N, pixels, bad)
    RESULTS["voxel"]["texel_outside_both_sides"] = ub  # reference UB, stand-in texel on both
    _record_flush()
    assert not bad, bad[:3]


def test_multi_sweep(built, floor):
    """The one-process multi-GPU object (sfrt_multi, devices listed twice or more on cuda:0: the
    peer-copy transport) on random scenes: 2-4 ranks, random band rows (sfrt_multi_set_bands) that
    change from frame to frame (band buffers grow and are retired), RGBA or packed transfers;
    every gathered frame equals the restatement's."""
    import oracle
    import sfrt
    from test_gpu_parity import _fuzz_scene, diff_report
    rng = np.random.default_rng(SEED0 + 7)
    bad, pixels = [], 0
    n_multi = max(1, N // 10)  # each scene renders on several worlds
    objs = {}
    try:
        for seed in range(SEED0, SEED0 + n_multi):
            sc, w, h = _fuzz_scene(seed) if MODE == "random" else _sphere_adversarial(seed)
            w, h = SIZE or (w, h)
            ranks = int(rng.integers(2, 5))
            if ranks not in objs:
                objs[ranks] = sfrt.Multi([0] * ranks, sfrt.SFRT_MULTI_PEER)
                objs[ranks].load_texture(*floor)
            m = objs[ranks]
            m.set_scene(sc, w, h)
            if h >= ranks and rng.random() < 0.7:
                cuts = np.sort(rng.choice(np.arange(1, h), ranks - 1, replace=False))
                rows = np.diff(np.concatenate([[0], cuts, [h]])).astype(int).tolist()
                m.set_bands(rows)
            else:
                m.set_bands(None)  # the equal split
            m.set_transfer(int(rng.choice([sfrt.SFRT_TRANSFER_AUTO, sfrt.SFRT_TRANSFER_RGBA])))
            got = m.update_image()
            want = oracle.Oracle.from_scene(sc, w, h, *floor).render(host_threads())
            msg = diff_report(got, want, w)
            if msg:
                bad.append({"seed": seed, "ranks": ranks, "diff": msg})
            pixels += w * h
            _progress("multi", seed - SEED0 + 1, bad)
    finally:
        for m in objs.values():
            m.close()
    _record("multi", n_multi, pixels, bad)
    assert not bad, bad[:3]
