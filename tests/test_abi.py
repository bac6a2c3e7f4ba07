"""The C-ABI library loads without a GPU, exports every symbol include/sfrt.h
declares, and its host-side helpers agree with the restatement."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
import scenes
from conftest import ROOT


@pytest.fixture(scope="module")
def lib(built):
    import sfrt
    return sfrt.lib()


def header_symbols():
    text = open(os.path.join(ROOT, "include", "sfrt.h")).read()
    return sorted(set(re.findall(r"^SFRT_API [^;]*?\b(sfrt_\w+)\s*\(", text, re.M)))


def test_exports_every_declared_symbol(lib):
    import sfrt
    names = header_symbols()
    assert len(names) >= 20
    assert set(names) == set(sfrt.ABI_SYMBOLS)
    for n in names:
        assert hasattr(lib, n), n


def test_only_abi_symbols_are_exported():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only",
                          os.path.join(ROOT, "sfml-software-raytracer_amd", "libsfrt.so")],
                         capture_output=True, text=True, check=True).stdout
    funcs = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert funcs == set(header_symbols())


def test_world_create_without_gpu_fails_loudly(lib):
    import sfrt
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    h = ctypes.c_void_p()
    assert lib.sfrt_world_create(0, ctypes.byref(h)) == -5  # SFRT_E_HIP, no CPU fallback
    with pytest.raises(sfrt.SfrtError):
        sfrt.World(0)


def test_error_strings(lib):
    for code in range(0, -8, -1):
        assert lib.sfrt_error_string(code)
    assert lib.sfrt_version() >= 3


def test_in_tree_library_is_release_build(lib):
    """The shipped libsfrt.so reports the release flavour (bench.py refuses any other:
    diagnostic -DSFRT_EXP builds write wrong bytes by design, A/B builds carry extra flags)."""
    assert lib.sfrt_build_flavour() == b"release"


def test_deg_to_rad_matches_reference_expression(lib):
    for d in (75.0, 47.0, 90.0, 1.0, 123.456):
        assert np.float32(lib.sfrt_deg_to_rad(d)) == scenes.deg2rad(d)
        assert np.float32(lib.sfrt_deg_to_rad(d)) == np.float32(oracle.lib().oracle_deg2rad(d))


def _passes(r, s):
    r, s = np.float32(r), np.float32(s)
    return bool(np.float32(r - np.sqrt(s)) > np.float32(0.01))


def test_pass_threshold_is_exact(lib):
    rng = np.random.default_rng(5)
    radii = np.concatenate([np.arange(1, 9, dtype=np.float32),
                            rng.uniform(0.005, 500, 300).astype(np.float32),
                            np.float32([0.01, 0.0100001, 0.02, 1e-6, 3e7])])
    for r in radii:
        t = np.float32(lib.sfrt_pass_threshold(float(r)))
        if t == 0:
            assert not _passes(r, 0.0)
            continue
        below = np.nextafter(t, np.float32(0))
        assert _passes(r, below) and not _passes(r, t), r
        # spot-check monotonicity further away on both sides
        for s in (t * np.float32(0.5), below * np.float32(0.999)):
            assert _passes(r, s)
        for s in (t * np.float32(1.001), t * np.float32(2)):
            assert not _passes(r, s)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_sort_spheres_matches_update_spheres(lib, seed):
    import sfrt
    rng = np.random.default_rng(seed)
    sp = np.concatenate([scenes.lcg_spheres(count=40, seed=seed),
                         # exact key ties exercise the "insert after equal keys" rule
                         np.float32([[3, 0, 0, 2], [0, 3, 0, 2], [0, 0, -3, 2], [3, 0, 0, 2]])])
    rng.shuffle(sp)
    cam = tuple(rng.uniform(-2, 2, 3).astype(np.float32))
    a = sfrt.sort_spheres(sp, cam)
    b = oracle.sort_spheres(sp, cam)
    c = scenes.sort_spheres(sp, cam)
    assert np.array_equal(a, b) and np.array_equal(a, c)


def test_lcg64_scene_shape():
    s = scenes.lcg64().spheres
    assert s.shape == (64, 4)
    assert (s[:, 3] >= 2).all() and (s[:, 3] <= 7).all()
    # first draws of the MSVC LCG, seed 12345 (s = s*214013 + 2531011, r = (s >> 16) & 0x7fff)
    st, r = scenes.msvc_rand(12345)
    assert r == ((12345 * 214013 + 2531011) & 0xFFFFFFFF) >> 16 & 0x7FFF


def test_cpp_header_builds(built, tmp_path):
    """include/sfrt.hpp (the C++ mirror of SphereWorld / World / sf::Shader) compiles and
    links against libsfrt.so; run on the GPU by test_gpu_parity.py::test_cpp_host_api."""
    lib_dir = os.path.join(ROOT, "sfml-software-raytracer_amd")
    exe = tmp_path / "cpp_api_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-I",
                    os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "cpp_api_check.cpp"), "-L", lib_dir,
                    "-lsfrt", f"-Wl,-rpath,{lib_dir}", "-Wl,-rpath-link,/opt/rocm/lib",
                    "-lpthread", "-o", str(exe)], check=True)
    assert exe.exists()


def test_multi_bands_match_band_tuner(lib):
    """sfrt_multi_bands (the C-ABI partition of sfrt_multi) equals bands.root_weighted_spans
    (the partition the torch.distributed path tunes), row for row, and tiles the frame."""
    import bands
    import sfrt
    for world_size in (1, 2, 3, 4, 8):
        for height in (0, 1, 7, 90, 1080, 2160, 4320, 16384, 17280):
            for factor in (1.0,) + bands.DEFAULT_FACTORS + (0.5, 10.0):
                got = sfrt.multi_bands(height, world_size, factor)
                assert got == bands.root_weighted_spans(height, world_size, factor), \
                    (height, world_size, factor)
                bands.check_spans(got, height)
    assert sfrt.multi_bands(4320, 2) == [(0, 2160), (2160, 2160)]
    assert sfrt.multi_bands(16384, 8) == [(r * 2048, 2048) for r in range(8)]
    with pytest.raises(sfrt.SfrtError):
        sfrt.multi_bands(100, 0)
    with pytest.raises(sfrt.SfrtError):
        sfrt.multi_bands(100, 2, float("nan"))


def test_multi_cost_bands_match_band_tuner(lib):
    """sfrt_multi_cost_bands (cost-weighted band edges, SURVEY 8e "Balance") equals
    bands.cost_weighted_spans row for row; the bands tile the frame on 8-row edges, give
    rank 0 about `factor` shares of the cost, and fall back to the row-weighted split for
    costs that carry no information."""
    import bands
    import sfrt
    rng = np.random.default_rng(7)
    for world_size in (1, 2, 3, 4, 8):
        for height in (0, 1, 7, 90, 1080, 2160, 4320):
            for kind in ("random", "uniform", "ramp", "spike"):
                if kind == "random":
                    cost = rng.gamma(2.0, 50.0, height).astype(np.float32)
                elif kind == "uniform":
                    cost = np.full(height, 3840.0, np.float32)
                elif kind == "ramp":
                    cost = np.linspace(1.0, 100.0, height, dtype=np.float32)
                else:
                    cost = np.ones(height, np.float32)
                    cost[height // 3: height // 3 + 8] = 1e4
                for factor in (1.0, 1.5, 2.0, 3.0, 0.5):
                    got = sfrt.multi_cost_bands(cost, world_size, factor)
                    assert got == bands.cost_weighted_spans(cost, world_size, factor), \
                        (height, world_size, kind, factor)
                    bands.check_spans(got, height)
                    assert all(r0 % bands.ALIGN == 0 or r0 == height for r0, _ in got)
    # balance: equal cost shares within one tile row's cost of the target
    cost = np.concatenate([np.full(2000, 10.0), np.full(2320, 100.0)]).astype(np.float32)
    spans = sfrt.multi_cost_bands(cost, 4, 1.0)
    share = [float(cost[r0:r0 + n].sum()) for r0, n in spans]
    assert max(share) - min(share) <= 2 * 8 * 100.0, (spans, share)
    assert spans[0][1] > spans[3][1]  # the cheap rows go to fewer ranks
    spans2 = sfrt.multi_cost_bands(cost, 4, 2.0)
    s2 = [float(cost[r0:r0 + n].sum()) for r0, n in spans2]
    assert abs(s2[0] / s2[1] - 2.0) < 0.1, s2
    # no information -> the row-weighted split
    for bad in (np.zeros(4320, np.float32), np.full(4320, -1.0, np.float32),
                np.full(4320, np.nan, np.float32)):
        assert sfrt.multi_cost_bands(bad, 4, 2.0) == sfrt.multi_bands(4320, 4, 2.0)
        assert bands.cost_weighted_spans(bad, 4, 2.0) == bands.root_weighted_spans(4320, 4, 2.0)
    with pytest.raises(sfrt.SfrtError):
        sfrt.multi_cost_bands(cost, 0, 1.0)


def test_multi_create_without_gpu_fails_loudly(lib):
    import sfrt
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    devs = (ctypes.c_int * 2)(0, 1)
    h = ctypes.c_void_p()
    assert lib.sfrt_multi_create(devs, 2, sfrt.SFRT_MULTI_AUTO, ctypes.byref(h)) == -5
    assert lib.sfrt_multi_create(devs, 0, sfrt.SFRT_MULTI_AUTO, ctypes.byref(h)) == -1


def test_bench_c_abi_line_failure_is_isolated():
    """bench.py runs the single-process multi-GPU line in a child process: a child that fails
    (here: no HIP device in this container) yields {"error": ...} for that line instead of
    ending the parent, so the headline JSON line is never lost to it."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    out = bench.c_abi_multi_isolated([0, 1], 20, 5, 0.0)
    assert out["devices"] == [0, 1]
    assert "error" in out and "exit" in out["error"], out
