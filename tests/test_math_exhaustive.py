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


def test_div255_exact():
    """sfrt_device.h div255: q = RN(c * y), y = RN(1/255), then RN(q + RN(c - 255 q) * y) by two
    fmas, equals the correctly rounded c / 255 for every integer c in [0, 255] (exact rationals;
    the GLSL kernel's texel channels, rayShader.frag's texture() / 255)."""
    from fractions import Fraction as Fr

    import numpy as np

    def rn(x: Fr) -> Fr:  # round to nearest binary32, ties to even (normal range)
        if x == 0:
            return Fr(0)
        sign = -1 if x < 0 else 1
        x = abs(x)
        e = 0
        while x >= 2:
            x /= 2
            e += 1
        while x < 1:
            x *= 2
            e -= 1
        m = x * 2 ** 23
        fl = m.numerator // m.denominator
        rem = m - fl
        if rem > Fr(1, 2) or (rem == Fr(1, 2) and fl % 2 == 1):
            fl += 1
        return sign * Fr(fl) * Fr(2) ** (e - 23)

    y = rn(Fr(1, 255))
    assert y == Fr(float.fromhex("0x1.010102p-8"))
    for c in range(256):
        q = rn(c * y)
        r = rn(c - 255 * q)  # fma(-255, q, c)
        q2 = rn(q + r * y)   # fma(r, y, q)
        assert q2 == rn(Fr(c, 255)), c
        assert float(q2) == float(np.float32(np.float32(c) / np.float32(255))), c
