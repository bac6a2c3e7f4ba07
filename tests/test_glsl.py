"""GLSL renderer: rayShader.frag run per render-target pixel,
/root/reference/Raytracing/rayShader.frag:1-179, uniforms from
SphereWorld.cpp:214-238 and Source.cpp:143-146.

CPU: the uniform replay (glsl_scenes.py) reproduces the survey's srand(0)
scene; the restatement (oracle/glsl_oracle.c) is deterministic across threads
and bands and matches its committed golden hashes (tests/golden/golden.json
"glsl").  GPU: libsfrt.so's GLSL kernel equals the restatement byte for byte.
Parity against the reference's own OpenGL output is unpinned (no GL context
can run here; DESIGN.md 4b fixes the semantics the shader leaves open).
"""
import ctypes
import ctypes.util
import json
import os

import numpy as np
import pytest

import glsl_scenes as gs
import oracle
import scenes
from conftest import ROOT, host_threads, poisoned

GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))

# (key, width, height, uniform builder)
GLSL_CASES = [
    ("default@320x180", 320, 180, lambda w, h: gs.default_uniforms(w, h)),
    ("default@1920x1080", 1920, 1080, lambda w, h: gs.default_uniforms(w, h)),
    ("default@1920x1080/0.7,0.3", 1920, 1080, lambda w, h: gs.default_uniforms(w, h, 0.7, 0.3)),
    ("frames300@1920x1080/5.5,-0.4", 1920, 1080,
     lambda w, h: gs.default_uniforms(w, h, 5.5, -0.4, frames=300)),
    ("default@3840x2160/2.5,-0.2", 3840, 2160, lambda w, h: gs.default_uniforms(w, h, 2.5, -0.2)),
    ("random1(1,0,0)@320x180", 320, 180, lambda w, h: gs.random_uniforms(1, 1, 0, 0, w, h)),
    ("random2(12,2,14)@320x180", 320, 180, lambda w, h: gs.random_uniforms(2, 12, 2, 14, w, h)),
    ("random3(40,4,50)@640x360", 640, 360, lambda w, h: gs.random_uniforms(3, 40, 4, 50, w, h)),
    ("random4(5,0,9)@333x97", 333, 97, lambda w, h: gs.random_uniforms(4, 5, 0, 9, w, h)),
    # bench.py's "glsl_3840x2160" line (its 1080p line is default@1920x1080)
    ("default@3840x2160", 3840, 2160, lambda w, h: gs.default_uniforms(w, h)),
]
CPU_CASES = [c for c in GLSL_CASES if c[1] * c[2] <= 640 * 360]


def synthetic_ground(w=64, h=32, seed=5):
    return np.random.default_rng(seed).integers(0, 256, w * h * 4, dtype=np.uint8), w, h


@pytest.fixture(scope="module")
def floor():
    return scenes.load_floor()


def glsl_oracle(case, floor):
    _, w, h, make = case
    return oracle.GlslOracle(make(w, h), *floor)


# ---------------- CPU ----------------

def test_constructor_replay_reproduces_default10():
    """srand(0) + the constructor's rand() order gives the survey's default10
    walls -- pins the uniform fixture."""
    w = gs.ShaderWorld(0)
    walls = np.array([(*b.pos, b.radius) for b in w.spheres], np.float32)
    assert np.array_equal(walls, scenes.default10().spheres)
    u = w.uniforms()
    assert (int(u["sphere_count"]), int(u["light_count"]), int(u["all_spheres_count"])) == (10, 1, 21)
    # history: the light's uvs slot keeps osphere 0's value from before AddLight
    assert u["uvs"][10].tolist() == [0.5, 1.0, 0.5, 0.0]
    assert u["lights"][10].tolist() == [1.0, 1.0, 1.0, 1.0]
    assert np.all(u["lights"][11:21] == np.float32([0.5, 1, 1, 1]))
    assert set(u["spheres"][11:21, 3].tolist()) == {float(np.float32(0.3)), float(np.float32(0.6))}


def test_glibc_rand_emulation():
    libc = ctypes.CDLL(ctypes.util.find_library("c"))
    for seed in (0, 1, 42, 2**31 - 1):
        libc.srand(seed)
        r = gs.GlibcRand(seed)
        assert [libc.rand() for _ in range(500)] == [r() for _ in range(500)]


def test_update_world_moves_ospheres_only():
    w = gs.ShaderWorld(0)
    before = w.uniforms()
    for _ in range(50):
        w.update_world()
    after = w.uniforms()
    assert np.array_equal(before["spheres"][:11], after["spheres"][:11])
    assert not np.array_equal(before["spheres"][11:21], after["spheres"][11:21])


@pytest.mark.parametrize("case", CPU_CASES, ids=[c[0] for c in CPU_CASES])
def test_oracle_matches_golden(case, floor):
    o = glsl_oracle(case, floor)
    frame = o.render(case[1], case[2], host_threads())
    assert oracle.fnv1a64(frame) == GOLDEN["glsl"][case[0]]["fnv1a64"]


def test_oracle_threads_and_bands_agree(floor):
    case = GLSL_CASES[6]
    o = glsl_oracle(case, floor)
    w, h = case[1], case[2]
    full = o.render(w, h, 1)
    assert np.array_equal(full, o.render(w, h, 7))
    parts = [o.render_band(w, h, r0, min(37, h - r0)) for r0 in range(0, h, 37)]
    assert np.array_equal(full, np.concatenate(parts))


def test_oracle_known_answers(floor):
    """Spot values the shader's formulas fix exactly (rayShader.frag:153-158)."""
    u = gs.default_uniforms(320, 180)
    o = oracle.GlslOracle(u, *floor)
    frame = o.render(320, 180, host_threads()).reshape(180, 320, 4)
    assert (frame[..., 3] == 255).all()
    seen = set()
    for row in range(0, 180, 6):
        for i in range(0, 320, 6):
            d = o.pixel(320, 180, i, row)
            ds = d["draw_sphere"]
            assert 0 <= ds < 21
            if d["checkstep"] == 0 and ds == 10:       # the light: 0.5 * rgb * (2 + fog)
                assert frame[row, i, :3].tolist() == [255, 255, 255]
                seen.add("light")
            if d["checkstep"] == 1:
                assert ds < 10 and d["total_dist"] == d["wall_dist"]
                seen.add("wall")
            if d["checkstep"] == 0 and ds > 10:
                seen.add("ball")
    assert seen == {"light", "wall", "ball"}


def test_march_steps_are_bounded(floor):
    o = oracle.GlslOracle(gs.default_uniforms(320, 180), *floor)
    steps = o.march_steps(320, 180, host_threads())
    assert steps.min() >= 1 and steps.max() < 100


# ---------------- GPU ----------------

@pytest.fixture(scope="module")
def shader(built, floor):
    import sfrt
    s = sfrt.GlslShader(0)
    s.set_ground(*floor)
    return s


def draw(shader, u, w, h):
    shader.set_uniforms(u)
    return shader.draw_image(w, h)


def first_diff(got, want, w):
    bad = np.nonzero(np.any(got.reshape(-1, 4) != want.reshape(-1, 4), axis=1))[0]
    if bad.size == 0:
        return ""
    k = int(bad[0])
    return f"{bad.size} pixels differ, first ({k % w}, {k // w}): {got.reshape(-1, 4)[k]} vs " \
           f"{want.reshape(-1, 4)[k]}"


@pytest.mark.gpu
@pytest.mark.parametrize("case", GLSL_CASES, ids=[c[0] for c in GLSL_CASES])
def test_gpu_matches_oracle(shader, floor, case):
    key, w, h, make = case
    u = make(w, h)
    got = draw(shader, u, w, h)
    want = oracle.GlslOracle(u, *floor).render(w, h, host_threads())
    assert np.array_equal(got, want), first_diff(got, want, w)
    assert oracle.fnv1a64(got) == GOLDEN["glsl"][key]["fnv1a64"]


def draw_ordered(shader, u, w, h):
    """The ordered kernel (sfrt_glsl_draw into a device frame: the adaptive tile order and the
    per-wave wall cull), after a warm-up draw so that the tile order is in use."""
    import torch
    shader.set_uniforms(u)
    b = poisoned((h, w * 4))
    for _ in range(3):
        shader.draw(b.data_ptr(), w, h, w * 4, 0, h, 0)
    shader.check(0)
    return b.cpu().numpy().ravel()


@pytest.mark.gpu
@pytest.mark.parametrize("case", GLSL_CASES, ids=[c[0] for c in GLSL_CASES])
def test_gpu_ordered_kernel_matches_oracle(shader, floor, case):
    """The ordered kernel bench.py times culls each wave's walls to those its rays can meet
    (glsl_trace.hip wall_mask): the same bytes as the oracle and as the row-major kernel, which
    visits every wall."""
    key, w, h, make = case
    u = make(w, h)
    got = draw_ordered(shader, u, w, h)
    assert oracle.fnv1a64(got) == GOLDEN["glsl"][key]["fnv1a64"], key
    if w * h <= 640 * 360:
        want = oracle.GlslOracle(u, *floor).render(w, h, host_threads())
        assert np.array_equal(got, want), first_diff(got, want, w)


@pytest.mark.gpu
def test_gpu_wall_cull_random_scenes(shader, floor):
    """The wall cull on 48 random scenes (3-60 walls, random camera and rotation, some with a
    wide field of view): the ordered kernel's frame equals the oracle's."""
    rng = np.random.default_rng(5)
    for seed in range(48):
        nw, nl, nb = int(rng.integers(3, 61)), int(rng.integers(0, 4)), int(rng.integers(0, 12))
        w, h = (160, 90) if seed % 3 else (96, 64)
        u = gs.random_uniforms(100 + seed, nw, nl, nb, w, h)
        if seed % 4 == 0:
            u["fov"] = (np.float32(rng.uniform(1.5, 2.6)), np.float32(rng.uniform(1.0, 2.0)))
        got = draw_ordered(shader, u, w, h)
        want = oracle.GlslOracle(u, *floor).render(w, h, host_threads())
        assert np.array_equal(got, want), (seed, nw, first_diff(got, want, w))


def _sweep_uniforms(seed):
    """The uniforms scene `seed` of tests/test_parity_sweep.py's GLSL sweep draws (its random
    sequence replayed from the first scene)."""
    rng = np.random.default_rng(20000)
    for s in range(20000, seed + 1):
        nw, nl, nb = int(rng.integers(3, 61)), int(rng.integers(0, 4)), int(rng.integers(0, 12))
        w, h = [(160, 90), (96, 64), (133, 47)][s % 3]
        fov = (np.float32(rng.uniform(1.5, 2.6)), np.float32(rng.uniform(1.0, 2.0))) if s % 4 == 0 else None
    u = gs.random_uniforms(seed, nw, nl, nb, w, h)
    if fov is not None:
        u["fov"] = fov
    return u, w, h


# (seed, pixel): a shadow ball whose cosine to the light rounds to -1.0000001 there
SHADOW_NAN_CASES = [(20904, (143, 25)), (23983, (38, 23))]


@pytest.mark.parametrize("case", SHADOW_NAN_CASES, ids=[str(c[0]) for c in SHADOW_NAN_CASES])
def test_oracle_shadow_cosine_below_minus_one_is_nan(floor, case):
    """The restatement's semantics at the edge the parity sweep found (profiles/r6ps_*): a
    shadow ball straight behind the point from the light gives dot(-tolightnorm, u) =
    -1.0000001 in binary32, acos (glibc acosf) is NaN, the GLSL clamp formula passes NaN on,
    and the pixel's colour converts to 0."""
    seed, (x, y) = case
    u, w, h = _sweep_uniforms(seed)
    d = oracle.GlslOracle(u, *floor).pixel(w, h, x, y)
    assert np.isnan(d["brightness"]) and d["color"][3] == 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("case", SHADOW_NAN_CASES, ids=[str(c[0]) for c in SHADOW_NAN_CASES])
def test_gpu_shadow_cosine_below_minus_one(shader, floor, case):
    """The kernel's exact shadow skip (cosang <= cos_lit: the clamp's argument >= 1) must not
    take a cosine below -1, whose acos is NaN: both kernels equal the oracle on the two scenes
    of the 10,000-scene sweep that had one such pixel each."""
    seed, _ = case
    u, w, h = _sweep_uniforms(seed)
    want = oracle.GlslOracle(u, *floor).render(w, h, host_threads())
    got = draw_ordered(shader, u, w, h)
    assert np.array_equal(got, want), first_diff(got, want, w)
    got = draw(shader, u, w, h)
    assert np.array_equal(got, want), first_diff(got, want, w)


@pytest.mark.gpu
def test_gpu_synthetic_ground_mips(shader, floor):
    """Non-square ground (64x32: 2x1 box levels) over the default uniforms."""
    import sfrt
    g = synthetic_ground()
    s = sfrt.GlslShader(0)
    s.set_ground(*g)
    for w, h, rot in [(320, 180, (0.0, 0.0)), (400, 300, (1.9, 0.45))]:
        u = gs.default_uniforms(w, h, *rot, frames=120)
        got = draw(s, u, w, h)
        want = oracle.GlslOracle(u, *g).render(w, h, host_threads())
        assert np.array_equal(got, want), first_diff(got, want, w)
    s.close()


def _negzero_cam(w, h):
    u = gs.random_uniforms(6, 8, 2, 12, w, h)
    u["campos"] = (-0.0, 0.25, -0.0)
    return u


def _far_balls(w, h):
    """Balls far outside the walls: no dominance, long march, shadow pairs far away."""
    u = gs.default_uniforms(w, h, 0.4, 0.2)
    u["spheres"][11:21, :3] += np.float32(3000.0)
    return u


def _no_walls(w, h):
    u = gs.random_uniforms(7, 1, 1, 6, w, h)
    u["spheres"][:-1] = u["spheres"][1:].copy()     # drop the wall: sphereCount 0
    u["uvs"][:-1] = u["uvs"][1:].copy()
    u["lights"][:-1] = u["lights"][1:].copy()
    u["sphere_count"], u["all_spheres_count"] = 0, int(u["all_spheres_count"]) - 1
    return u


def _walls_only(w, h):
    return gs.random_uniforms(8, 9, 0, 0, w, h)


def _empty(w, h):
    u = gs.random_uniforms(9, 1, 0, 0, w, h)
    u["sphere_count"] = u["all_spheres_count"] = 0
    return u


def _camera_outside(w, h):
    u = gs.default_uniforms(w, h, 0.2, 0.1)
    u["campos"] = (30.0, 2.0, -25.0)
    return u


EDGE = [_negzero_cam, _far_balls, _no_walls, _walls_only, _empty, _camera_outside]


@pytest.mark.parametrize("make", EDGE, ids=[m.__name__.strip("_") for m in EDGE])
def test_oracle_edge_uniforms_run(floor, make):
    """Degenerate uniform blocks the shader accepts render without hitting the march cap."""
    o = oracle.GlslOracle(make(96, 54), *floor)
    assert o.render(96, 54, host_threads()).size == 96 * 54 * 4


@pytest.mark.gpu
@pytest.mark.parametrize("make", EDGE, ids=[m.__name__.strip("_") for m in EDGE])
def test_gpu_edge_uniforms(shader, floor, make):
    w, h = 320, 181
    u = make(w, h)
    got = draw(shader, u, w, h)
    want = oracle.GlslOracle(u, *floor).render(w, h, host_threads())
    assert np.array_equal(got, want), first_diff(got, want, w)


@pytest.mark.gpu
def test_gpu_bands_tile_the_frame(shader, floor):
    import torch
    w, h = 1920, 1080
    u = gs.default_uniforms(w, h, 0.3, 0.1, frames=40)
    shader.set_uniforms(u)
    full = shader.draw_image(w, h)
    buf = poisoned((h, w * 4 + 64), 0)
    stream = torch.cuda.Stream()
    for r0 in range(0, h, 250):
        rows = min(250, h - r0)
        shader.draw(buf[r0].data_ptr(), w, h, buf.stride(0), r0, rows, stream.cuda_stream)
    stream.synchronize()
    shader.check(stream.cuda_stream)
    got = buf[:, : w * 4].cpu().numpy().ravel()
    assert np.array_equal(got, full)


@pytest.mark.gpu
def test_gpu_set_uniform_by_name_replay(built, floor):
    """UpdateSpheres + main()'s setUniform calls by name give the same frame as
    the uniform block (SphereWorld.cpp:214-238, Source.cpp:143-146)."""
    import sfrt
    w, h = 480, 270
    u = gs.default_uniforms(w, h, 1.2, 0.2, frames=10)
    s = sfrt.GlslShader(0)
    s.set_ground(*floor)
    n = int(u["all_spheres_count"])
    for k in range(n):
        s.set_uniform(f"spheres[{k}]", u["spheres"][k])
        s.set_uniform(f"lights[{k}]", u["lights"][k])
        s.set_uniform(f"uvs[{k}]", u["uvs"][k])
    s.set_uniform("lightCount", int(u["light_count"]))
    s.set_uniform("sphereCount", int(u["sphere_count"]))
    s.set_uniform("allSpheresCount", int(u["all_spheres_count"]))
    for name in ("campos", "rotation", "fov", "size"):
        s.set_uniform(name, u[name])
    got = s.draw_image(w, h)
    want = oracle.GlslOracle(u, *floor).render(w, h, host_threads())
    assert np.array_equal(got, want), first_diff(got, want, w)
    back = s.get_uniforms(gs.UNIFORM_DTYPE)
    assert back.tobytes() == np.asarray(u).tobytes()
    with pytest.raises(sfrt.SfrtError):
        s.set_uniform("spheres[100]", [0, 0, 0, 1])
    with pytest.raises(sfrt.SfrtError):
        s.set_uniform("nosuch", [1.0, 2.0])
    with pytest.raises(sfrt.SfrtError):
        s.set_uniform("campos", [1.0, 2.0])
    s.close()


@pytest.mark.gpu
def test_gpu_errors_fail_loudly(built, floor):
    import sfrt
    s = sfrt.GlslShader(0)
    u = gs.default_uniforms(64, 64)
    s.set_uniforms(u)
    with pytest.raises(sfrt.SfrtError, match="NO_TEXTURE"):
        s.draw_image(64, 64)
    with pytest.raises(sfrt.SfrtError, match="INVALID"):
        s.set_ground(np.zeros(48 * 32 * 4, np.uint8), 48, 32)
    s.set_ground(*floor)
    bad = u.copy()
    bad["spheres"][3][1] = np.nan
    s.set_uniforms(bad)
    with pytest.raises(sfrt.SfrtError, match="INVALID"):
        s.draw_image(64, 64)
    bad = u.copy()
    bad["all_spheres_count"] = 101
    s.set_uniforms(bad)
    with pytest.raises(sfrt.SfrtError, match="INVALID"):
        s.draw_image(64, 64)
    bad = u.copy()
    bad["size"] = (0.0, 64.0)
    s.set_uniforms(bad)
    with pytest.raises(sfrt.SfrtError, match="INVALID"):
        s.draw_image(64, 64)
    s.set_uniforms(u)
    assert s.draw_image(64, 64).size == 64 * 64 * 4
    s.close()


@pytest.mark.gpu
def test_gpu_adaptive_tile_order_same_bytes(shader, floor):
    """SFRT_OPT_TILE_ORDER on the GLSL renderer (sfrt_glsl_draw dispatches 8x8 tiles
    longest-first by the metaball-march steps of two frames back): frames drawn back to back
    on one stream -- static uniforms, moving ospheres, size changes, a row band -- equal
    draw_image's frames (the row-major kernel) and, for two of them, the oracle."""
    import torch
    seq = [(gs.default_uniforms(640, 360, 0.0, 0.0), 640, 360, 0, 360)] * 4 + \
          [(gs.default_uniforms(640, 360, 0.3 * k, 0.1, frames=20 * k), 640, 360, 0, 360)
           for k in range(4)] + \
          [(gs.random_uniforms(3, 40, 4, 50, 333, 211), 333, 211, 0, 211)] * 3 + \
          [(gs.default_uniforms(640, 360, 2.5, -0.2), 640, 360, 40, 200)] * 3
    import sfrt
    stream = torch.cuda.Stream()
    frames = []
    shader.set_option(sfrt.SFRT_OPT_TILE_ORDER, 1)  # the default since round 4
    with torch.cuda.stream(stream):
        for u, w, h, r0, rows in seq:
            shader.set_uniforms(u)
            b = poisoned((h, w * 4))
            shader.draw(b[r0].data_ptr(), w, h, w * 4, r0, rows, stream.cuda_stream)
            frames.append(b)
    shader.check(stream.cuda_stream)
    torch.cuda.synchronize()
    shader.set_option(sfrt.SFRT_OPT_TILE_ORDER, 0)
    try:
        for k, ((u, w, h, r0, rows), b) in enumerate(zip(seq, frames)):
            full = draw(shader, u, w, h)
            want = np.full(w * h * 4, 0xA5, dtype=np.uint8)
            want[r0 * w * 4:(r0 + rows) * w * 4] = full[r0 * w * 4:(r0 + rows) * w * 4]
            got = b.cpu().numpy().ravel()
            assert np.array_equal(got, want), (k, first_diff(got, want, w))
            if k in (3, 10):
                assert np.array_equal(full, oracle.GlslOracle(u, *floor).render(w, h, host_threads())), k
    finally:
        shader.set_option(sfrt.SFRT_OPT_TILE_ORDER, 1)


def test_march_dominance_test_implies_round3_test():
    """glsl_trace.hip's dominance test (two fmas, bounds inflated by (1+6e-6) and rounded up:
    kThrMul, kThrAdd, the host's r_skip) implies the round-3 test it replaced,
    ss >= (r + t*(1+1e-5) + 1e-4)^2 * 1.00001f on the shader's own ss, whose sufficiency for
    skipping a ball exactly is argued in DESIGN.md 5c.  binary32 emulated in numpy (products of
    two binary32 values are exact in binary64; fma = one rounding of the exact sum, here a
    binary64 sum rounded once more, good to far below the 1e-6 slack).  Borderline samples sit
    within 1e-5 of the new test's threshold."""
    f32 = np.float32
    rng = np.random.default_rng(7)
    n = 400_000
    r = (rng.random(n) * 40.0).astype(f32)
    r[: n // 10] = 0.0
    t = (np.float64(0.5) + rng.random(n) * 60.0).astype(f32)      # max(smooth+0.5, shortest, 0.5)
    k_mul, k_add, k_r = f32(float.fromhex("0x1.00010ep+0")), f32(float.fromhex("0x1.a36ed4p-14")), \
        f32(float.fromhex("0x1.000065p+0"))
    r_skip = np.nextafter((r * k_r).astype(f32), f32(np.inf))
    thr_new = ((t * k_mul).astype(f32) + k_add).astype(f32)
    thr_old = ((t * f32(1.00001)).astype(f32) + f32(1e-4)).astype(f32)
    bnd_new = (r_skip + thr_new).astype(f32)
    lim_new = (bnd_new * bnd_new).astype(f32)
    bnd_old = (r + thr_old).astype(f32)
    lim_old = ((bnd_old * bnd_old).astype(f32) * f32(1.00001)).astype(f32)
    # points whose fma'd squared length lands around the new threshold (and some far off)
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1)[:, None]
    scale = np.sqrt(lim_new.astype(np.float64)) * (1.0 + (rng.random(n) - 0.5) * 2e-5)
    scale[: n // 20] *= 1.0 + rng.random(n // 20) * 3.0
    o = (u * scale[:, None]).astype(f32)
    ox, oy, oz = (o[:, i].astype(np.float64) for i in range(3))
    inner = (oy * oy + (oz * oz).astype(f32).astype(np.float64)).astype(f32).astype(np.float64)
    ssf = (ox * ox + inner).astype(f32)
    ss = ((((ox * ox).astype(f32) + (oy * oy).astype(f32)).astype(f32)
           + (oz * oz).astype(f32)).astype(f32))
    new = ssf >= lim_new
    old = ss >= lim_old
    assert new.sum() > n // 4 and (~new).sum() > n // 4        # both outcomes well sampled
    bad = np.nonzero(new & ~old)[0]
    assert bad.size == 0, (bad.size, r[bad[0]], t[bad[0]], o[bad[0]])


@pytest.mark.gpu
def test_gpu_tables_reused_across_streams(shader, floor):
    """ADVICE r4 (sfrt_host.h TableSlot): per-draw tables staged on stream A behind queued work,
    then reused at once by a draw on stream B with no host sync between: B must wait for A's
    staging copy and draw the new uniforms."""
    import torch
    w, h = 320, 180
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for k in range(3):
        u = gs.default_uniforms(w, h, 0.6 + 0.3 * k, 0.1, frames=5 + k)
        shader.set_uniforms(u)
        ba = poisoned((h, w * 4))
        bb = poisoned((h, w * 4))
        torch.cuda.synchronize()
        with torch.cuda.stream(a):
            torch.cuda._sleep(100_000_000)  # ~50 ms of queued work ahead of A's staging copy
        shader.draw(ba.data_ptr(), w, h, w * 4, 0, h, a.cuda_stream)   # stages on A
        shader.draw(bb.data_ptr(), w, h, w * 4, 0, h, b.cuda_stream)   # reuses on B at once
        outs.append((u, ba, bb))
    torch.cuda.synchronize()
    shader.check(a.cuda_stream)
    shader.check(b.cuda_stream)
    for u, ba, bb in outs:
        want = oracle.GlslOracle(u, *floor).render(w, h, host_threads())
        got_a, got_b = ba.cpu().numpy().ravel(), bb.cpu().numpy().ravel()
        assert np.array_equal(got_a, want), first_diff(got_a, want, w)
        assert np.array_equal(got_b, want), first_diff(got_b, want, w)


@pytest.mark.gpu
def test_gpu_tables_restaged_after_every_uniform_setter(shader, floor):
    """The per-draw tables (walls, balls, light/shadow pairs, materials) are staged once and
    reused while the uniforms do not change (sfrt_glsl.cpp u_version): a repeated draw equals
    the first, and each setter alone -- the block, a float uniform by name, an int uniform by
    name -- is seen by the next draw (compared with the oracle of the uniforms it was given)."""
    import torch
    w, h = 320, 180
    stream = torch.cuda.Stream()

    def frame():
        b = poisoned((h, w * 4))
        shader.draw(b.data_ptr(), w, h, w * 4, 0, h, stream.cuda_stream)
        shader.check(stream.cuda_stream)
        return b.cpu().numpy().ravel()

    def want(u):
        return oracle.GlslOracle(u, *floor).render(w, h, host_threads())

    u = gs.default_uniforms(w, h, 0.6, 0.1, frames=5)
    shader.set_uniforms(u)
    first = frame()
    assert np.array_equal(first, want(u)), first_diff(first, want(u), w)
    assert np.array_equal(frame(), first)                      # reused tables
    u2 = np.array(u, copy=True)                                # a ball moved, by name
    k = int(u2["sphere_count"]) + int(u2["light_count"])       # the first shadow ball
    u2["spheres"][k, 0] += np.float32(0.75)
    shader.set_uniform(f"spheres[{k}]", u2["spheres"][k])
    got = frame()
    assert np.array_equal(got, want(u2)), first_diff(got, want(u2), w)
    u3 = np.array(u2, copy=True)                               # one light fewer, by name
    u3["light_count"] = int(u3["light_count"]) - 1
    shader.set_uniform("lightCount", int(u3["light_count"]))
    got = frame()
    assert np.array_equal(got, want(u3)), first_diff(got, want(u3), w)
    shader.set_uniforms(u)                                     # the block again
    assert np.array_equal(frame(), first)


@pytest.mark.gpu
def test_gpu_ground_change_is_stream_ordered(built, floor):
    """sfrt_glsl_set_ground without a device-wide wait (sfrt_glsl.cpp, sfrt::SharedBuffer): a draw
    on stream B queued behind ~50 ms of work still reads the ground it was queued with when a new
    ground is set right after (the upload waits, on the device, for that draw); the call and the
    draw on A return while B's queue is still busy; each frame equals the restatement with its own
    ground.  Then a larger ground (a new buffer) and back.  The draw on A
    does not wait on the host for B's either: each stream has its own tile-order chain
    (sfrt_sched.h TileChains, since round 6 also for the GLSL and voxel renderers)."""
    import sfrt
    import torch
    w, h = 320, 180
    u = gs.default_uniforms(w, h, 0.4, 0.1, frames=7)
    grounds = [floor, synthetic_ground(), synthetic_ground(128, 256, seed=9), floor]
    s = sfrt.GlslShader(0)
    try:
        s.set_ground(*grounds[0])
        s.set_uniforms(u)
        # B at high priority: the object's own stream, where the upload runs, never shares B's
        # hardware queue (two streams that share one run in order, GPU_MAX_HW_QUEUES)
        a, b = torch.cuda.Stream(), torch.cuda.Stream(priority=-1)
        warm = torch.empty((h, w * 4), dtype=torch.uint8, device="cuda:0")
        s.draw(warm.data_ptr(), w, h, w * 4, 0, h, a.cuda_stream)
        torch.cuda.synchronize()
        frames = []
        for k in range(1, len(grounds)):
            old, new = poisoned((h, w * 4)), poisoned((h, w * 4))  # filled before B is busy
            with torch.cuda.stream(b):
                torch.cuda._sleep(100_000_000)
            s.draw(old.data_ptr(), w, h, w * 4, 0, h, b.cuda_stream)   # reads grounds[k - 1]
            assert not b.query(), "B drained before the calls (the test's own setup waited)"
            s.set_ground(*grounds[k])
            busy = {"set_ground": not b.query()}
            s.draw(new.data_ptr(), w, h, w * 4, 0, h, a.cuda_stream)   # reads grounds[k]
            busy["draw on A"] = not b.query()
            frames.append((grounds[k - 1], old, grounds[k], new, busy))
            torch.cuda.synchronize()
        s.check(a.cuda_stream)
        s.check(b.cuda_stream)
        for g_old, old, g_new, new, busy in frames:
            assert all(busy.values()), f"waited for the queued draw on B: {busy}"
            for g, buf in ((g_old, old), (g_new, new)):
                want = oracle.GlslOracle(u, *g).render(w, h, host_threads())
                got = buf.cpu().numpy().ravel()
                assert np.array_equal(got, want), first_diff(got, want, w)
    finally:
        s.close()
