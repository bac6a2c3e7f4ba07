"""Where the GLSL kernel's wave time goes, block by block.

    python tools/glsl_block_profile.py build      # here: an instrumented copy of libsfrt.so
    python tools/glsl_block_profile.py run        # GPU: per-block shares, JSON on stdout

`build` copies the package's Makefile, csrc/ and include/ to sfml-software-raytracer_amd/build_glslprof/,
patches the copy of glsl_trace.hip (never the product source) with shader-clock reads
(s_memtime) at the boundaries of fragment()'s blocks -- ray setup, the wall pass
(rayShader.frag:71-85), the metaball march (:94-112), the texture (:123-126), the lighting
with its soft shadows (:128-151), colour and store (:153-158) -- accumulated per wave into a
device array by lane 0, and builds libsfrt.so there (build flavour "ab": it is never a product
library).  `run` renders the bench.py GLSL frames (1080p and 4K, default uniforms) through it
and prints each block's share of the wave-clock cycles, with the per-wave work counts that go
with them.  The clock reads add their own waits, so the shares are attributions, not a
timeline; the kernel's VALU total comes from the PMC passes (profiles/*_glsl_traffic.json).
"""
import ctypes
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sfml-software-raytracer_amd")
BASE = os.path.join(PKG, "build_glslprof")
OUT = os.path.join(BASE, "pkg")  # BASE/include beside it: the Makefile's ../include
BLOCKS = ["setup", "walls", "march", "texture", "lighting", "store"]

PATCHES = [
    ("__device__ __forceinline__ void fragment(",
     "__device__ unsigned long long g_block_clk[8];\n"
     "__device__ unsigned long long g_block_cnt[4];\n"
     "__device__ __forceinline__ void fragment("),
    ("  const float fx = (float)i + 0.5f;\n",
     "  const unsigned long long c0 = __builtin_amdgcn_s_memtime();\n"
     "  unsigned long long clk[6];\n"
     "  unsigned long long n_wall = 0, n_march = 0, n_ball = 0, n_shadow = 0;\n"
     "  const float fx = (float)i + 0.5f;\n"),
    ("  // ---- furthest wall: 3 passes over the walls (:71-85) ----\n",
     "  clk[0] = __builtin_amdgcn_s_memtime();\n"
     "  // ---- furthest wall: 3 passes over the walls (:71-85) ----\n"),
    ("    const GlslWall w = ld(walls, k);\n",
     "    const GlslWall w = ld(walls, k);\n    n_wall++;\n"),
    ("  // ---- metaball march over lights + ospheres (:87-112) ----\n",
     "  clk[1] = __builtin_amdgcn_s_memtime();\n"
     "  // ---- metaball march over lights + ospheres (:87-112) ----\n"),
    ("    if (++steps > kGlslMarchCap) {",
     "    n_march++;\n    if (++steps > kGlslMarchCap) {"),
    ("      const float other = sqrt_cr(ss) - b.r;\n",
     "      n_ball++;\n      const float other = sqrt_cr(ss) - b.r;\n"),
    ("  // ---- wall or ball (:114-120) ----\n",
     "  clk[2] = __builtin_amdgcn_s_memtime();\n"
     "  // ---- wall or ball (:114-120) ----\n"),
    ("  // ---- lighting (:128-151) ----\n",
     "  clk[3] = __builtin_amdgcn_s_memtime();\n"
     "  // ---- lighting (:128-151) ----\n"),
    ("        float sangle = sfrt_math::acosf(cosang);\n",
     "        n_shadow++;\n        float sangle = sfrt_math::acosf(cosang);\n"),
    ("  // ---- colour (:153-158) ----\n",
     "  clk[4] = __builtin_amdgcn_s_memtime();\n"
     "  // ---- colour (:153-158) ----\n"),
    ("        unorm8(cr) | (unorm8(cg) << 8) | (unorm8(cbl) << 16) | (255u << 24);\n}\n",
     "        unorm8(cr) | (unorm8(cg) << 8) | (unorm8(cbl) << 16) | (255u << 24);\n"
     "  clk[5] = __builtin_amdgcn_s_memtime();\n"
     "  if ((threadIdx.x & 63) == 0) {\n"
     "    unsigned long long prev = c0;\n"
     "    for (int q = 0; q < 6; q++) { atomicAdd(&g_block_clk[q], clk[q] - prev); prev = clk[q]; }\n"
     "    atomicAdd(&g_block_clk[6], 1ull);\n"
     "    atomicAdd(&g_block_cnt[0], n_wall); atomicAdd(&g_block_cnt[1], n_march);\n"
     "    atomicAdd(&g_block_cnt[2], n_ball); atomicAdd(&g_block_cnt[3], n_shadow);\n"
     "  }\n}\n"),
    ("}  // namespace\n\nlong long glsl_tile_key(",
     "}  // namespace\n\n"
     "extern \"C\" __attribute__((visibility(\"default\"))) int sfrt_glsl_block_clocks("
     "unsigned long long* out, int reset) {\n"
     "  if (hipDeviceSynchronize() != hipSuccess) return -1;\n"
     "  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_block_clk), 7 * 8) != hipSuccess) return -1;\n"
     "  if (hipMemcpyFromSymbol(out + 7, HIP_SYMBOL(g_block_cnt), 4 * 8) != hipSuccess) return -1;\n"
     "  if (reset) {\n"
     "    unsigned long long z[8] = {};\n"
     "    if (hipMemcpyToSymbol(HIP_SYMBOL(g_block_clk), z, 8 * 8) != hipSuccess) return -1;\n"
     "    if (hipMemcpyToSymbol(HIP_SYMBOL(g_block_cnt), z, 4 * 8) != hipSuccess) return -1;\n"
     "  }\n"
     "  return 0;\n}\n\nlong long glsl_tile_key("),
]


def build():
    if os.path.exists(BASE):
        shutil.rmtree(BASE)
    os.makedirs(OUT)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(BASE, "include"))
    shutil.copy(os.path.join(PKG, "Makefile"), OUT)
    shutil.copytree(os.path.join(PKG, "csrc"), os.path.join(OUT, "csrc"))
    p = os.path.join(OUT, "csrc", "glsl_trace.hip")
    s = open(p).read()
    for old, new in PATCHES:
        if s.count(old) != 1:
            raise SystemExit(f"patch anchor not found once: {old[:60]!r}")
        s = s.replace(old, new)
    open(p, "w").write(s)
    subprocess.run(["make", "-s", "-j", "8", "-C", OUT, "EXTRA=-DSFRT_GLSL_BLOCK_PROFILE"], check=True)
    print(os.path.join(OUT, "libsfrt.so"))


def run():
    os.environ["SFRT_LIB"] = os.path.join(OUT, "libsfrt.so")
    sys.path.insert(0, PKG)
    import torch
    import glsl_scenes as gs
    import scenes
    import sfrt
    L = sfrt.lib()
    L.sfrt_glsl_block_clocks.argtypes = [ctypes.c_void_p, ctypes.c_int]
    s = sfrt.GlslShader(0)
    s.set_ground(*scenes.load_floor())
    out = (ctypes.c_ulonglong * 11)()
    res = {}
    for w, h in ((1920, 1080), (3840, 2160)):
        s.set_uniforms(gs.default_uniforms(w, h))
        buf = torch.empty(h, w * 4, dtype=torch.uint8, device="cuda")
        for _ in range(5):
            s.draw(buf.data_ptr(), w, h, w * 4, 0, h, 0)
        L.sfrt_glsl_block_clocks(out, 1)
        frames = 20
        for _ in range(frames):
            s.draw(buf.data_ptr(), w, h, w * 4, 0, h, 0)
        s.check()
        L.sfrt_glsl_block_clocks(out, 1)
        v = list(out)
        waves = v[6]
        tot = sum(v[:6])
        res[f"{w}x{h}"] = {
            "share_of_wave_clocks": {b: round(v[q] / tot, 4) for q, b in enumerate(BLOCKS)},
            "clocks_per_wave": round(tot / waves, 1),
            "per_wave": {"wall_iterations": round(v[7] / waves, 2),
                         "march_steps": round(v[8] / waves, 2),
                         "ball_bodies": round(v[9] / waves, 2),
                         "shadow_bodies": round(v[10] / waves, 2)},
            "frames": frames}
    s.close()
    print(json.dumps({"tool": "tools/glsl_block_profile.py", "library": os.environ["SFRT_LIB"],
                      "note": "s_memtime clocks per block summed over waves (instrumented copy)",
                      "frames": res}, indent=1))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
