"""Build-flag A/B of libsfrt.so builds, interleaved across processes, bytes checked.

    python tools/ab_libs.py --libs a.so,b.so,a.so@3 [--rounds 3] [--reps 40] [--cases 4k,4k_rot,...]
(lib@R forces R pixels per lane, SFRT_OPT_RAYS_PER_LANE; lib^O sets SFRT_OPT_TILE_ORDER=O on every
renderer; lib#K sets SFRT_AB_KNOB=K for an
experimental build that reads it -- r2_ab28 read it as SFRT_SPLIT; the product reads none)

Each round starts one process per library (SFRT_LIB=<lib>, the same sfrt.py), which
times every case with HIP events (median kernel time, event-pair overhead subtracted;
adaptive tile order, frames back to back on one stream, camera turning in the *_turn
cases) and hashes one frame per case.  The parent prints per-case medians over rounds
and fails if any library's frame hash differs from the first library's.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = {
    "4k": (3840, 2160, "lcg64", (0.0, 0.0), False),
    "4k_rot": (3840, 2160, "lcg64", (1.1, -0.2), False),
    "4k_turn": (3840, 2160, "lcg64", (0.0, 0.0), True),
    "8k": (7680, 4320, "lcg64", (0.0, 0.0), False),
    "1080": (1920, 1080, "default10", (0.0, 0.0), False),
    "4k_256": (3840, 2160, "lcg256", (0.0, 0.0), False),
    # the other renderers: scene = "voxel:<x>,<y>,<z>" / "glsl", pose = rot
    "vox1080": (1920, 1080, "voxel:15.5,1.9,15.5", (0.0, 0.0), False),
    "vox4k": (3840, 2160, "voxel:15.5,1.9,15.5", (0.0, 0.0), False),
    "vox4k_rot": (3840, 2160, "voxel:47.5,1.5,60.1", (4.0, -0.3), False),
    "glsl1080": (1920, 1080, "glsl", (0.0, 0.0), False),
    "glsl4k": (3840, 2160, "glsl", (0.0, 0.0), False),
    # the live loop's UpdateWorld every frame (Source.cpp:143-153): the world advanced one step
    # per frame, the camera turning 0.004 rad per frame
    "glsl4k_move": (3840, 2160, "glsl", (0.0, 0.0), True),
    "glsl1080_move": (1920, 1080, "glsl", (0.0, 0.0), True),
}


def renderer(sfrt, scenes, sname, pose, width, height, rays):
    """An object with render_band(ptr, pitch, row0, rows, stream) / check(stream) for a case."""
    order = os.environ.get("SFRT_AB_TILE_ORDER")  # "lib^O": the 8f renderers' tile order
    if sname.startswith("voxel:"):
        import voxel_scenes as vs
        v = sfrt.VoxelWorld(0)
        if order is not None:
            v.set_option(sfrt.SFRT_OPT_TILE_ORDER, int(order))
        tex, dyn = vs.load_textures()
        v.load_assets(tex, dyn, vs.COLORS)
        v.set_scene(vs.default_world(tuple(float(c) for c in sname[6:].split(",")), *pose),
                    width, height)
        return v, None
    if sname == "glsl":
        import glsl_scenes as gs
        g = sfrt.GlslShader(0)
        if order is not None:
            g.set_option(sfrt.SFRT_OPT_TILE_ORDER, int(order))
        g.set_ground(*scenes.load_floor())
        g.set_uniforms(gs.default_uniforms(width, height, *pose))

        class Draw:
            def __init__(self):
                self.world = gs.ShaderWorld(0)

            def render_band(self, ptr, pitch, row0, rows, stream):
                g.draw(ptr, width, height, pitch, row0, rows, stream)

            def set_camera(self, _pos, rotation, hrotation):  # a moving case: one UpdateWorld
                self.world.update_world()
                g.set_uniforms(self.world.uniforms(width, height, rotation, hrotation))

            def check(self, stream):
                g.check(stream)
        return Draw(), g
    return None, None


def child(cases, reps, rays):
    sys.path.insert(0, os.path.join(ROOT, "sfml-software-raytracer_amd"))
    import numpy as np
    import torch
    import hashlib
    import scenes
    import sfrt
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    w = sfrt.World(0)
    w.load_texture(*scenes.load_floor())
    w.set_option(sfrt.SFRT_OPT_RAYS_PER_LANE, rays)
    pairs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
             for _ in range(64)]
    for a, b in pairs:
        a.record(stream)
        b.record(stream)
    torch.cuda.synchronize()
    gap = float(np.median([a.elapsed_time(b) for a, b in pairs]))
    out = {}
    sphere_world = w
    for name in cases:
        width, height, sname, pose, turn = CASES[name]
        w, keep = renderer(sfrt, scenes, sname, pose, width, height, rays)
        sc = None
        if w is None:
            w = sphere_world
            if os.environ.get("SFRT_AB_TILE_ORDER") is not None:  # "lib^O" on the sphere world too
                w.set_option(sfrt.SFRT_OPT_TILE_ORDER, int(os.environ["SFRT_AB_TILE_ORDER"]))
            sc = scenes.SCENES[sname]().posed(*pose)
            w.set_scene(sc, width, height)
        cam_pos = sc.cam_pos if sc is not None else None
        buf = torch.empty(height, width * 4, dtype=torch.uint8, device="cuda")
        for k in range(20):  # warm-up (clock ramp, tile-order chain)
            if turn:
                w.set_camera(cam_pos, 0.004 * k, 0.0)
            w.render_band(buf.data_ptr(), width * 4, 0, height, stream.cuda_stream)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(reps)]
        for k, (a, b) in enumerate(ev):
            if turn:
                w.set_camera(cam_pos, 0.004 * (20 + k), 0.0)
            a.record(stream)
            w.render_band(buf.data_ptr(), width * 4, 0, height, stream.cuda_stream)
            b.record(stream)
        torch.cuda.synchronize()
        w.check(stream.cuda_stream)
        t = sorted(a.elapsed_time(b) for a, b in ev)
        # the same frames back to back with no markers between them: wall time per frame
        # (kernel plus the launch boundary a frame loop pays)
        import time
        t0 = time.perf_counter()
        for k in range(reps):
            if turn:
                w.set_camera(cam_pos, 0.004 * (20 + reps + k), 0.0)
            w.render_band(buf.data_ptr(), width * 4, 0, height, stream.cuda_stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        out[name] = {"us": round((t[len(t) // 2] - gap) * 1e3, 2), "wall_us": round(wall * 1e6, 2),
                     "fnv": hashlib.sha256(buf.cpu().numpy().tobytes()).hexdigest()[:16]}
    print("RESULT " + json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--cases", default="4k,4k_rot,4k_turn,8k,1080")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--rays", type=int, default=0, help="(child) SFRT_OPT_RAYS_PER_LANE")
    a = ap.parse_args()
    cases = a.cases.split(",")
    if a.child:
        child(cases, a.reps, a.rays)
        return
    libs = a.libs.split(",")
    res = {lib: {c: [] for c in cases} for lib in libs}
    walls = {lib: {c: [] for c in cases} for lib in libs}
    hashes = {}
    for rnd in range(a.rounds):
        for lib in libs:  # "path" or "path@R" (R = SFRT_OPT_RAYS_PER_LANE); "path!" = timing probe
            probe = lib.endswith("!")
            spec, _, order = lib.rstrip("!").partition("^")  # "^O": 8f renderers' tile order
            spec, _, knob = spec.partition("#")  # "#K": SFRT_AB_KNOB=K for an A/B build
            path, _, rays = spec.partition("@")
            env = dict(os.environ, SFRT_LIB=os.path.abspath(path))
            if knob:
                env["SFRT_AB_KNOB"] = knob
            if order:
                env["SFRT_AB_TILE_ORDER"] = order
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--libs", lib,
                                "--cases", a.cases, "--reps", str(a.reps), "--rays", rays or "0"],
                               capture_output=True, text=True, env=env, timeout=600)
            line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
            if r.returncode != 0 or not line:
                print(r.stdout[-2000:], r.stderr[-2000:])
                raise SystemExit(f"{lib}: child failed")
            d = json.loads(line[0][7:])
            for c in cases:
                res[lib][c].append(d[c]["us"])
                walls[lib][c].append(d[c].get("wall_us", 0.0))
                if probe:
                    continue  # a probe build writes other bytes by design
                hashes.setdefault(c, d[c]["fnv"])
                if d[c]["fnv"] != hashes[c]:
                    raise SystemExit(f"{lib}: {c} bytes differ ({d[c]['fnv']} vs {hashes[c]})")
    summary = {}
    for lib in libs:
        summary[lib] = {c: sorted(v)[len(v) // 2] for c, v in res[lib].items()}
        print(f"{lib:40s} " + "  ".join(f"{c} {summary[lib][c]:8.2f}" for c in cases))
    wsum = {lib: {c: sorted(v)[len(v) // 2] for c, v in walls[lib].items()} for lib in libs}
    for lib in libs:
        print(f"wall {lib:35s} " + "  ".join(f"{c} {wsum[lib][c]:8.2f}" for c in cases))
    print(json.dumps({"median_us": summary, "median_wall_us": wsum, "rounds": res, "bytes_identical": True}))


if __name__ == "__main__":
    main()
