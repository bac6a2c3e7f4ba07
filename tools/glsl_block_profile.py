"""Where the GLSL kernel's VALU instructions go, block by block.

    python tools/glsl_block_profile.py static     # here: static VALU per block of the release ISA
    python tools/glsl_block_profile.py build      # here: an instrumented copy of libsfrt.so
    python tools/glsl_block_profile.py run        # GPU: per-wave executions of each block (JSON)
    python tools/glsl_block_profile.py combine COUNTS.json [--pmc profiles/<tag>_glsl_traffic.json]

VALU per wave = sum over the shader's blocks of (the block's VALU per execution, counted in the
release kernel's ISA) x (the block's executions per wave, counted on the GPU by an instrumented
copy).  `combine` prints that attribution and compares its total with the PMC pass's
SQ_INSTS_VALU / SQ_WAVES for the same launch size.

Blocks (fragment() in csrc/glsl_trace.hip, rayShader.frag lines):
  setup          ray direction, wall-pass preamble (:63-70)
  wall_test      one wall-pass iteration: the wall record and the inside test (:71-85)
  wall_inside    its body when a lane of the wave is inside the wall
  march_step     one metaball-march step outside the ball loop (:94-112)
  ball_test      one ball's dominance test inside a march step
  ball_body      its body (polsmin, normal) when a lane is not dominated
  texture        wall-or-ball resolve and the mipmapped texture (:114-126)
  light          one light of the lighting loop outside its shadow loop (:128-151)
  shadow_test    one shadow ball's cone test
  shadow_body    its soft-shadow body
  colour         colour, fog and the store (:153-158)
  rare           the keep_branch fallbacks (plain division, full sqrt lowering) that no wave of
                 these frames takes, and the ordered kernel's tile sorter (one workgroup per
                 launch) -- counted separately, excluded from the expected total

`static` compiles the product source with -gline-tables-only (the ISA is checked identical to the
release build's) and assigns each basic block of k_glsl_ordered (the kernel bench.py times) to a
block by the ISA's loop structure and the source lines in it.  `build` copies the package's
Makefile, csrc/ and include/ to sfml-software-raytracer_amd/build_glslprof/, patches the copy of
glsl_trace.hip (never the product source) with per-block execution counters -- the first active
lane of the wave counts each execution, so a divergent loop counts its wave iterations -- summed
over the wave and added to a device array by lane 0, and builds libsfrt.so there (build flavour
"ab": never a product library).  `run` renders the bench.py GLSL frames (1080p and 4K, default
uniforms) through it.  (Round 3's version of this tool read s_memtime at block boundaries; the
compiler moves those reads across the arithmetic and the sums came out several times the waves'
lifetimes, so clocks were dropped for instruction counts.)
"""
import argparse
import ctypes
import json
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sfml-software-raytracer_amd")
SRC = os.path.join(PKG, "csrc", "glsl_trace.hip")
BASE = os.path.join(PKG, "build_glslprof")
OUT = os.path.join(BASE, "pkg")  # BASE/include beside it: the Makefile's ../include
# the ordered kernel sfrt_glsl_draw launches by default since round 4 (fragment() is the same
# inlined body in k_glsl, the row-major kernel of draw_image)
KERNEL = "_ZN4sfrt12_GLOBAL__N_114k_glsl_orderedENS_9GlslFrameEi"
COUNTED = ["wall_test", "wall_inside", "march_step", "ball_test", "ball_body", "light",
           "shadow_test", "shadow_body"]
ONCE = ["setup", "texture", "colour"]

# Source anchors (one line each in glsl_trace.hip) that identify the loops and bodies.
ANCHORS = {
    "wall_loop": "const bool inside = s <= w.s_in;",
    "wall_inside_first": "moved |= inside_mask != 0;",
    "wall_inside_last": "total = total + tosurf;",
    "march_loop": "ball_dist += smooth + 0.01f;",
    "ball_loop": "const bool dominated = ssf >= bnd * bnd;",
    "ball_body_first": "const float ss = (ox * ox + oy * oy) + oz * oz;",
    "ball_body_last": "thr = fmaxf(fmaxf(smooth + 0.5f, shortest), 0.5f) * kThrMul",
    "light_loop": "const float tlx = L.x - px, tly = L.y - py, tlz = L.z - pz;",
    "shadow_loop": "const float cosang = (-tnx * P.ux + -tny * P.uy) + -tnz * P.uz;",
    "shadow_body_first": "float sangle = sfrt_math::acosf(cosang);",
    "shadow_body_last": "shadow *= gclamp(sangle / P.sanglet",
}


def anchor_lines(src_lines):
    out = {}
    for k, a in ANCHORS.items():
        hits = [i + 1 for i, l in enumerate(src_lines) if a in l]
        if len(hits) != 1:
            raise SystemExit(f"anchor {k!r} found {len(hits)} times in {SRC}")
        out[k] = hits[0]
    return out


FLAGS = ["-DSFRT_BUILD_FLAVOUR=\"release\"", "-O3", "-fno-slp-vectorize", "-std=c++17", "-fPIC",
         "-fvisibility=hidden", "-ffp-contract=off", "-fno-fast-math", "-I../include", "-Icsrc"]
LLVM = "/opt/rocm/lib/llvm/bin"


def compile_device(extra, out, kind):
    """The product source's gfx950 code: assembly (kind "-S") or a code object (kind "-c")."""
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950"] + FLAGS + extra +
                   ["-x", "hip", "--offload-device-only", "--no-gpu-bundle-output", kind, "-o", out,
                    "csrc/glsl_trace.hip"], cwd=PKG, check=True, stderr=subprocess.DEVNULL)
    return out


def kernel_lines(path):
    lines = open(path).read().splitlines()
    st = next(i for i, l in enumerate(lines) if l.startswith(KERNEL + ":"))
    en = next(i for i in range(st, len(lines)) if "s_endpgm" in lines[i])
    return lines[st + 1:en + 1]


def parse_blocks(body):
    """Basic blocks of the kernel's assembly: name, innermost loop header, parent loop header,
    instruction mnemonics in order, and whether the block holds keep_branch's empty asm
    statement (a rare fallback path)."""
    blocks, cur, prev_asm = [], None, False
    for line in body:
        m = re.match(r"^(\.LBB\d+_\d+):(.*)", line) or re.match(r"^; (%bb\.\d+):(.*)", line)
        if m or cur is None:
            cur = {"name": m.group(1) if m else "entry", "header": None, "parent": None,
                   "insts": [], "rare": False}
            blocks.append(cur)
            tail = m.group(2) if m else line
        else:
            tail = line
        h = re.search(r"Header=BB(\d+_\d+)", tail)
        if h:
            cur["header"] = ".LBB" + h.group(1)
        if re.search(r"=>\s*This (Inner )?Loop Header", tail):
            cur["header"] = cur["name"]
        p = re.search(r"Parent Loop BB(\d+_\d+)", tail)
        if p:
            cur["parent"] = ".LBB" + p.group(1)
        if m:
            continue
        t = line.strip()
        if t == ";;#ASMEND" and prev_asm:
            cur["rare"] = True  # keep_branch(): an empty asm statement
        prev_asm = t == ";;#ASMSTART"
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        cur["insts"].append(t.split()[0])
    return blocks


def fragment_lines(co):
    """(mnemonic, line of fragment() the instruction belongs to -- through inlined helpers, by
    llvm-symbolizer --inlining -- or None outside fragment) for k_glsl, in address order."""
    dis = subprocess.run([LLVM + "/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                         capture_output=True, text=True).stdout.splitlines()
    st = next(i for i, l in enumerate(dis) if l.endswith(f"<{KERNEL}>:"))
    insts = []
    for l in dis[st + 1:]:
        m = re.match(r"\s+(\S+).*//\s+([0-9A-Fa-f]+):", l)
        if not m:
            continue
        insts.append((m.group(1), int(m.group(2), 16)))
        if m.group(1) == "s_endpgm":
            break
    sym = subprocess.run([LLVM + "/llvm-symbolizer", "--obj=" + co, "--inlining",
                          "--functions=short"], input="".join(f"0x{a:x}\n" for _, a in insts),
                         check=True, capture_output=True, text=True).stdout
    frames = [f.strip().splitlines() for f in sym.strip().split("\n\n")]
    if len(frames) != len(insts):
        raise SystemExit("llvm-symbolizer returned a different number of entries")
    out = []
    for (mn, _), fr in zip(insts, frames):
        line = None
        for k in range(0, len(fr) - 1, 2):
            if fr[k] == "fragment":
                line = int(fr[k + 1].split(":")[-2])
            if fr[k].startswith("sort_tiles"):
                line = -1  # the ordered kernel's tile sorter (workgroup 0)
        out.append((mn, line))
    return out


def static():
    isa = os.path.join(PKG, "build", "isa")
    plain = compile_device([], os.path.join(isa, "glsl_trace_plain.s"), "-S")
    lined = compile_device(["-gline-tables-only"], os.path.join(isa, "glsl_trace_lines.s"), "-S")
    co = compile_device(["-gline-tables-only"], os.path.join(isa, "glsl_trace_lines.co"), "-c")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_compare
    (a, am), (b, bm) = isa_compare.kernels(plain), isa_compare.kernels(lined)
    if a.get(KERNEL) != b.get(KERNEL) or am.get(KERNEL) != bm.get(KERNEL):
        raise SystemExit("the line-table build's k_glsl ISA differs from the release build's")
    src = open(SRC).read().splitlines()
    A = anchor_lines(src)
    sec = {k: next(i + 1 for i, l in enumerate(src) if v in l) for k, v in
           (("texture", "// ---- wall or ball"), ("lighting", "// ---- lighting"))}
    blocks = parse_blocks(kernel_lines(lined))
    lines = fragment_lines(co)
    seq = [mn for bl in blocks for mn in bl["insts"]]
    if [mn for mn, _ in lines] != seq:
        raise SystemExit("the code object's instruction sequence differs from the assembly's")
    it = iter(lines)
    for bl in blocks:
        bl["lines"] = [next(it)[1] for _ in bl["insts"]]
    parent = {bl["name"]: bl["parent"] for bl in blocks if bl["header"] == bl["name"]}

    def loop_of(key):
        hs = {bl["header"] for bl in blocks if A[key] in bl["lines"] and bl["header"]}
        if len(hs) != 1:
            raise SystemExit(f"source line {A[key]} ({key}) is in loops {hs}")
        return hs.pop()

    loops = {k: loop_of(k) for k in ("wall_loop", "march_loop", "ball_loop", "light_loop",
                                     "shadow_loop")}
    if parent.get(loops["ball_loop"]) != loops["march_loop"] or \
            parent.get(loops["shadow_loop"]) != loops["light_loop"]:
        raise SystemExit("unexpected loop nesting")

    def region(bl, line):
        h = bl["header"]
        inr = lambda a, z: line is not None and A[a] <= line <= A[z]
        if bl["rare"] or line == -1:
            return "rare"
        if h == loops["wall_loop"]:
            return "wall_inside" if inr("wall_inside_first", "wall_inside_last") else "wall_test"
        if h == loops["ball_loop"]:
            return "ball_body" if inr("ball_body_first", "ball_body_last") else "ball_test"
        if h == loops["march_loop"]:
            return "march_step"
        if h == loops["shadow_loop"]:
            return "shadow_body" if inr("shadow_body_first", "shadow_body_last") else "shadow_test"
        if h == loops["light_loop"]:
            return "light"
        if h is not None:
            if line is None:  # not fragment(): the tile sorter of the ordered kernel (workgroup 0)
                return "rare"
            raise SystemExit(f"block {bl['name']} in an unexpected loop {h}")
        if line is None or line < sec["texture"]:
            return "setup"
        return "texture" if line < sec["lighting"] else "colour"

    per, per_block = {}, []
    for bl in blocks:
        v = {}
        for mn, line in zip(bl["insts"], bl["lines"]):
            if mn.startswith("v_"):
                r = region(bl, line)
                v[r] = v.get(r, 0) + 1
        for r, n in v.items():
            per[r] = per.get(r, 0) + n
        per_block.append({"name": bl["name"], "valu": v})
    return {"kernel": KERNEL, "valu_per_execution": per, "valu_total_static": sum(per.values()),
            "blocks": per_block,
            "isa": "release flags + -gline-tables-only (k_glsl ISA checked identical); each VALU "
                   "instruction assigned by its ISA loop and its line in fragment() "
                   "(llvm-symbolizer --inlining)"}


PATCHES = [
    ("__device__ __forceinline__ void fragment(",
     "__device__ unsigned long long g_block_cnt[8];\n"
     "__device__ __forceinline__ uint32_t first_lane_here() {\n"
     "  const uint64_t e = __builtin_amdgcn_read_exec();\n"
     "  return (uint32_t)((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(e));\n"
     "}\n"
     "__device__ __forceinline__ void fragment("),
    ("  const float fx = (float)i + 0.5f;\n",
     "  uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};\n"
     "  const float fx = (float)i + 0.5f;\n"),
    ("    const GlslWall w = ld(walls, k);\n",
     "    const GlslWall w = ld(walls, k);\n    cnt[0] += first_lane_here();\n"),
    ("      moved |= inside_mask != 0;\n",
     "      moved |= inside_mask != 0;\n      cnt[1] += first_lane_here();\n"),
    ("    if (++steps > kGlslMarchCap) {",
     "    cnt[2] += first_lane_here();\n    if (++steps > kGlslMarchCap) {"),
    ("      const GlslBall b = ld(balls, k);\n",
     "      const GlslBall b = ld(balls, k);\n      cnt[3] += first_lane_here();\n"),
    ("      const float ss = (ox * ox + oy * oy) + oz * oz;  // the shader's length(), :100\n",
     "      cnt[4] += first_lane_here();\n"
     "      const float ss = (ox * ox + oy * oy) + oz * oz;  // the shader's length(), :100\n"),
    ("    const GlslBall L = ld(balls, li);\n",
     "    const GlslBall L = ld(balls, li);\n    cnt[5] += first_lane_here();\n"),
    ("        const float cosang = (-tnx * P.ux + -tny * P.uy) + -tnz * P.uz;\n",
     "        cnt[6] += first_lane_here();\n"
     "        const float cosang = (-tnx * P.ux + -tny * P.uy) + -tnz * P.uz;\n"),
    ("        float sangle = sfrt_math::acosf(cosang);\n",
     "        cnt[7] += first_lane_here();\n        float sangle = sfrt_math::acosf(cosang);\n"),
    ("        unorm8(cr) | (unorm8(cg) << 8) | (unorm8(cbl) << 16) | (255u << 24);\n}\n",
     "        unorm8(cr) | (unorm8(cg) << 8) | (unorm8(cbl) << 16) | (255u << 24);\n"
     "  for (int q = 0; q < 8; q++) {\n"
     "    uint32_t v = cnt[q];\n"
     "    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);\n"
     "    if ((threadIdx.x & 63) == 0) atomicAdd(&g_block_cnt[q], (unsigned long long)v);\n"
     "  }\n"
     "  if ((threadIdx.x & 63) == 0) atomicAdd(&g_block_waves, 1ull);\n}\n"),
    ("__device__ unsigned long long g_block_cnt[8];\n",
     "__device__ unsigned long long g_block_cnt[8];\n__device__ unsigned long long g_block_waves;\n"),
    ("}  // namespace\n\nlong long glsl_tile_key(",
     "}  // namespace\n\n"
     "extern \"C\" __attribute__((visibility(\"default\"))) int sfrt_glsl_block_counts("
     "unsigned long long* out, int reset) {\n"
     "  if (hipDeviceSynchronize() != hipSuccess) return -1;\n"
     "  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_block_cnt), 8 * 8) != hipSuccess) return -1;\n"
     "  if (hipMemcpyFromSymbol(out + 8, HIP_SYMBOL(g_block_waves), 8) != hipSuccess) return -1;\n"
     "  if (reset) {\n"
     "    unsigned long long z[9] = {};\n"
     "    if (hipMemcpyToSymbol(HIP_SYMBOL(g_block_cnt), z, 8 * 8) != hipSuccess) return -1;\n"
     "    if (hipMemcpyToSymbol(HIP_SYMBOL(g_block_waves), z, 8) != hipSuccess) return -1;\n"
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
    L.sfrt_glsl_block_counts.argtypes = [ctypes.c_void_p, ctypes.c_int]
    s = sfrt.GlslShader(0)
    s.set_ground(*scenes.load_floor())
    out = (ctypes.c_ulonglong * 9)()
    res = {}
    for w, h in ((1920, 1080), (3840, 2160)):
        s.set_uniforms(gs.default_uniforms(w, h))
        buf = torch.empty(h, w * 4, dtype=torch.uint8, device="cuda")
        s.draw(buf.data_ptr(), w, h, w * 4, 0, h, 0)
        L.sfrt_glsl_block_counts(out, 1)
        frames = 3
        for _ in range(frames):
            s.draw(buf.data_ptr(), w, h, w * 4, 0, h, 0)
        s.check()
        L.sfrt_glsl_block_counts(out, 1)
        v = list(out)
        waves = v[8]
        res[str(w * h)] = {"frame": f"{w}x{h}", "waves": waves // frames,
                           "per_wave": {k: round(v[q] / waves, 3) for q, k in enumerate(COUNTED)}}
    s.close()
    print(json.dumps({"tool": "tools/glsl_block_profile.py run",
                      "note": "block executions per wave (first active lane counts; instrumented "
                              "copy of the kernel, default uniforms, rot (0,0))",
                      "launches": res}, indent=1))


def combine(counts_path, pmc_path):
    st = static()
    counts = json.load(open(counts_path))["launches"]
    pmc = json.load(open(pmc_path)) if pmc_path else None
    out = {"static": st["valu_per_execution"], "launches": {}}
    for key, ent in counts.items():
        per = dict(ent["per_wave"], **{k: 1.0 for k in ONCE})
        valu = {k: st["valu_per_execution"].get(k, 0) * per[k] for k in COUNTED + ONCE}
        tot = sum(valu.values())
        row = {"frame": ent["frame"], "executions_per_wave": per,
               "valu_per_wave": {k: round(v, 1) for k, v in valu.items()},
               "share": {k: round(v / tot, 4) for k, v in valu.items()},
               "predicted_valu_per_wave": round(tot, 1),
               "rare_fallback_valu_static": st["valu_per_execution"].get("rare", 0)}
        if pmc:
            tab = pmc.get("per_launch_pixels", pmc.get("per_grid_threads", {}))
            t = tab.get(str(int(key) + 64)) or tab.get(key)  # the ordered launch: + the sorter
            if t:
                row["pmc_valu_per_wave"] = round(t["SQ_INSTS_VALU"] / t["SQ_WAVES"], 1)
                row["predicted_over_pmc"] = round(tot / row["pmc_valu_per_wave"], 4)
                row["pmc_source"] = os.path.relpath(pmc_path, ROOT)
        out["launches"][key] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("static", "build", "run", "combine"))
    ap.add_argument("counts", nargs="?")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r4b_glsl_traffic.json"))
    a = ap.parse_args()
    if a.mode == "static":
        st = static()
        print(json.dumps({k: st[k] for k in ("kernel", "valu_per_execution", "valu_total_static",
                                              "isa")}, indent=1))
    elif a.mode == "build":
        build()
    elif a.mode == "run":
        run()
    else:
        combine(a.counts, a.pmc)
