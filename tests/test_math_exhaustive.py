"""sfrt_math.h (the kernels' atanf / atan2f / asinf / acosf) == host libm, bit for bit.

Host build of the same header the kernel uses, compiled with
-ffp-contract=off, checked against glibc 2.35 over every binary32 input of
asinf, atanf and acosf (2^32 each) and 10^8 atan2f pairs (random bit patterns and
the |coord| < 64 range hit points live in).  The gfx950 build of the header
is checked the same way in test_gpu_parity.py::test_device_math_matches_libm.
"""
import os
import subprocess

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def math_check(tmp_path_factory):
    exe = tmp_path_factory.mktemp("math") / "math_check"
    src = os.path.join(ROOT, "tests", "native", "math_check.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fopenmp", "-w", src, "-o",
                    str(exe)], check=True)
    return str(exe)


@pytest.mark.parametrize("args", [["asinf"], ["atanf"], ["acosf"], ["atan2f", "100000000", "1"],
                                  ["atan2f_x1"], ["atan2f_y1"], ["divpi"],
                                  ["divrecip", "1000000000"]])
def test_restated_math_matches_libm(math_check, args):
    r = subprocess.run([math_check] + args, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and "mismatches=0" in r.stdout, r.stdout + r.stderr
