"""Decode the reference's Floor.png into the committed raw RGBA8 asset.

Runs only in the build container (the GPU box has no /root/reference):
    python tools/make_assets.py
Floor.png is the only texel source on the sphere-cave path
(/root/reference/Raytracing/SphereWorld.cpp:52,376-377), so it is the only
asset committed.  Expected sha256 of the decoded bytes:
70a502bf...2690316d.
"""
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "sfml-software-raytracer_amd"))

from pngdecode import load_png_rgba  # noqa: E402

SRC = "/root/reference/Raytracing/Floor.png"
DST = os.path.join(ROOT, "sfml-software-raytracer_amd", "assets", "floor_128x128.rgba")
SHA = "70a502bfe27bffac852ce272fa26203f68df3ec9d25067226985f99d2690316d"

if __name__ == "__main__":
    rgba, w, h = load_png_rgba(SRC)
    assert (w, h) == (128, 128)
    digest = hashlib.sha256(rgba.tobytes()).hexdigest()
    assert digest == SHA, digest
    os.makedirs(os.path.dirname(DST), exist_ok=True)
    with open(DST, "wb") as f:
        f.write(rgba.tobytes())
    print(f"wrote {DST} sha256={digest}")
