"""Render the headline frame (3840x2160, lcg64, pose (0,0), adaptive order) N times on one
stream with whatever library SFRT_LIB names -- a driver for rocprofv3 --pmc passes of
diagnostic or A/B builds (bench.py refuses non-release libraries).
    SFRT_LIB=sfml-software-raytracer_amd/build_x64/libsfrt.so python tools/frame_loop.py [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sfml-software-raytracer_amd"))
import torch  # noqa: E402
import scenes  # noqa: E402
import sfrt  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    stream = torch.cuda.Stream()
    w = sfrt.World(0)
    w.load_texture(*scenes.load_floor())
    w.set_scene(scenes.lcg64(), 3840, 2160)
    buf = torch.empty(2160, 3840 * 4, dtype=torch.uint8, device="cuda")
    for _ in range(n):
        w.render_band(buf.data_ptr(), 3840 * 4, 0, 2160, stream.cuda_stream)
    torch.cuda.synchronize()
    print("frames", n, "library", sfrt.lib()._name if hasattr(sfrt.lib(), "_name") else "")


if __name__ == "__main__":
    main()
