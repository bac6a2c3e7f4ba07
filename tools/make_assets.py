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
sys.path.insert(0, HERE)

from pngdecode import load_png_rgba  # noqa: E402

SRC = "/root/reference/Raytracing/Floor.png"
DST = os.path.join(ROOT, "sfml-software-raytracer_amd", "assets", "floor_128x128.rgba")
SHA = "70a502bfe27bffac852ce272fa26203f68df3ec9d25067226985f99d2690316d"

# The voxel World renderer samples these (World.cpp:40-45);
# the file in the reference is "dynamic.png" (the code asks for "Dynamic.png").
VOXEL_ASSETS = ["Wall", "Ceiling", "Block", "dynamic", "Projectile", "Floor"]


def write_voxel_assets():
    out_dir = os.path.join(ROOT, "sfml-software-raytracer_amd", "assets")
    for name in VOXEL_ASSETS:
        rgba, w, h = load_png_rgba(f"/root/reference/Raytracing/{name}.png")
        with open(os.path.join(out_dir, f"{name}.rgba"), "wb") as f:
            f.write(rgba.tobytes())
        with open(os.path.join(out_dir, f"{name}.rgba.shape"), "w") as f:
            f.write(f"{w} {h}\n")
        print(f"wrote {name}.rgba {w}x{h} sha256={hashlib.sha256(rgba.tobytes()).hexdigest()[:16]}")


if __name__ == "__main__":
    write_voxel_assets()
    rgba, w, h = load_png_rgba(SRC)
    assert (w, h) == (128, 128)
    digest = hashlib.sha256(rgba.tobytes()).hexdigest()
    assert digest == SHA, digest
    os.makedirs(os.path.dirname(DST), exist_ok=True)
    with open(DST, "wb") as f:
        f.write(rgba.tobytes())
    print(f"wrote {DST} sha256={digest}")
