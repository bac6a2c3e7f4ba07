"""Where the voxel kernel's VALU instructions go, block by block.

    python tools/voxel_block_profile.py static     # here: static VALU per block of the release ISA
    python tools/voxel_block_profile.py build      # here: an instrumented copy of libsfrt.so
    python tools/voxel_block_profile.py run        # GPU: per-wave executions of each block (JSON)
    python tools/voxel_block_profile.py combine COUNTS.json [--pmc profiles/<tag>_voxel_traffic.json]

The method of tools/glsl_block_profile.py: each VALU instruction of k_voxel_ordered's release
ISA (the line-table build, checked identical) is assigned to a block by its ISA loop and its
inline chain (llvm-symbolizer --inlining: the innermost of raycast_t / shade_hit / lraycast_t and
its line), an instrumented copy counts each block's executions per wave (the first active lane
counts), and `combine` multiplies the two and compares the total with the PMC pass.

Blocks (World::Raycast / LRaycast, World.cpp:302-491; csrc/voxel_trace.hip):
  setup        kernel entry, pixel direction, ray setup of raycast_t (before its DDA loop)
  step         one DDA step of the primary ray: three divisions, the axis choice, the advance,
               the cell lookup, the loop test (World.cpp:322-350, 380-385)
  billboard    one iteration of the billboard loop (World.cpp:353-378)
  shade        the hit block outside the light loop: texel, lighting start, store (:385-412, :450)
  light_test   one light of the hit block's light loop up to the per-wave skip (the squared
               distance, :425)
  light        the rest of a light the wave does not skip, outside its shadow ray (:426-449)
  shadow_setup one shadow ray's setup (LRaycast before its loop)
  shadow_step  one step of a shadow ray (World.cpp:467-489)
  rare         the plain-division instantiations (a wave with an axis-parallel ray), the tile
               sorter and keep_branch fallbacks: counted separately, excluded from the total
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
SRC = os.path.join(PKG, "csrc", "voxel_trace.hip")
BASE = os.path.join(PKG, "build_voxprof")
OUT = os.path.join(BASE, "pkg")
KERNEL = "_ZN4sfrt12_GLOBAL__N_115k_voxel_orderedENS_8VoxFrameEii"
COUNTED = ["step", "billboard", "shade", "light_test", "shadow_setup", "shadow_step", "light"]
ONCE = ["setup"]
LLVM = "/opt/rocm/lib/llvm/bin"
sys.path.insert(0, os.path.join(ROOT, "tools"))
import glsl_block_profile as gbp  # noqa: E402  (compile flags, assembly block parser)

ANCHORS = {  # one line each in voxel_trace.hip
    "main_loop": "for (uint32_t i = 0; dist < f.view_distance && i < f.maxiter; i++) {",
    "billboard_first": "V3 bp = pos;",
    "billboard_last": "dnext = DI < f.ndyn ? f.dyn[DI].dist : __builtin_nanf(\"\");\n      }",
    "light_loop": "for (int j = 0; j < f.nlights; j++) {",
    "shadow_loop": "for (uint32_t i = 0; i < maxIter && dist < maxDist; i++) {",
    "light_skip": "if (!__builtin_amdgcn_ballot_w64(ddf < L.dd_skip)) continue;",
}


def anchor_lines():
    text = open(SRC).read()
    out = {}
    for k, a in ANCHORS.items():
        if text.count(a) != 1:
            raise SystemExit(f"anchor {k!r} found {text.count(a)} times in {SRC}")
        out[k] = text[:text.index(a)].count("\n") + 1 + a.count("\n")
    return out


def compile_device(extra, out, kind):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950"] + gbp.FLAGS + extra +
                   ["-x", "hip", "--offload-device-only", "--no-gpu-bundle-output", kind, "-o", out,
                    "csrc/voxel_trace.hip"], cwd=PKG, check=True, stderr=subprocess.DEVNULL)
    return out


def inline_chains(co):
    """(mnemonic, [(function, line), ... innermost first]) for every instruction of the kernel."""
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
        chain = []
        for k in range(0, len(fr) - 1, 2):
            parts = fr[k + 1].split(":")
            chain.append((fr[k], int(parts[-2]) if len(parts) >= 3 and parts[-2].isdigit() else 0))
        out.append((mn, chain))
    return out


def static():
    isa = os.path.join(PKG, "build", "isa")
    plain = compile_device([], os.path.join(isa, "voxel_trace_plain.s"), "-S")
    lined = compile_device(["-gline-tables-only"], os.path.join(isa, "voxel_trace_lines.s"), "-S")
    co = compile_device(["-gline-tables-only"], os.path.join(isa, "voxel_trace_lines.co"), "-c")
    import isa_compare
    (a, am), (b, bm) = isa_compare.kernels(plain), isa_compare.kernels(lined)
    if a.get(KERNEL) != b.get(KERNEL) or am.get(KERNEL) != bm.get(KERNEL):
        raise SystemExit("the line-table build's k_voxel_ordered ISA differs from the release build's")
    A = anchor_lines()
    gbp.KERNEL = KERNEL
    blocks = gbp.parse_blocks(gbp.kernel_lines(lined))
    chains = inline_chains(co)
    if [mn for mn, _ in chains] != [mn for bl in blocks for mn in bl["insts"]]:
        raise SystemExit("the code object's instruction sequence differs from the assembly's")
    it = iter(chains)
    for bl in blocks:
        bl["chains"] = [next(it)[1] for _ in bl["insts"]]

    def frame(chain, name):
        for fn, line in chain:
            if fn.startswith(name):
                return fn, line
        return None, None

    # the loops of the reciprocal instantiations, from the anchor lines' blocks
    def loop_of(fname, key):
        hs = set()
        for bl in blocks:
            for ch in bl["chains"]:
                fn, line = frame(ch, fname)
                if fn == fname and line == A[key] and bl["header"]:
                    hs.add(bl["header"])
        if not hs:
            raise SystemExit(f"no loop block holds {fname}:{A[key]} ({key})")
        return hs

    parent = {bl["name"]: bl["parent"] for bl in blocks if bl["header"] == bl["name"]}

    def ancestors(h):
        out = set()
        h = parent.get(h)
        while h:
            out.add(h)
            h = parent.get(h)
        return out

    def innermost(hs):  # a loop test evaluated in an enclosing loop's preheader names that loop too
        return {h for h in hs if not any(h in ancestors(o) for o in hs if o != h)}

    main_h = innermost(loop_of("raycast_t<true>", "main_loop"))
    light_h = innermost(loop_of("shade_hit<true>", "light_loop"))
    shadow_h = innermost(loop_of("lraycast_t<true>", "shadow_loop"))

    def inside(h, heads):  # block header h is one of heads or nested in one
        while h:
            if h in heads:
                return True
            h = parent.get(h)
        return False

    def region(bl, ch):
        names = [fn for fn, _ in ch]
        if bl["rare"] or any(n.endswith("<false>") for n in names) or \
                any(n.startswith("sort_tiles") for n in names):
            return "rare"
        h = bl["header"]
        if "lraycast_t<true>" in names:
            return "shadow_step" if inside(h, shadow_h) else "shadow_setup"
        if "shade_hit<true>" in names:
            if not inside(h, light_h):
                return "shade"
            _, line = frame(ch, "shade_hit<true>")
            return "light_test" if line <= A["light_skip"] else "light"
        fn, line = frame(ch, "raycast_t<true>")
        if fn and inside(h, main_h):
            return "billboard" if A["billboard_first"] <= line <= A["billboard_last"] else "step"
        return "setup"

    per, per_block = {}, []
    for bl in blocks:
        v = {}
        for mn, ch in zip(bl["insts"], bl["chains"]):
            if mn.startswith("v_"):
                r = region(bl, ch)
                per[r] = per.get(r, 0) + 1
                v[r] = v.get(r, 0) + 1
        per_block.append({"name": bl["name"], "header": bl["header"], "valu": v})
    return {"kernel": KERNEL, "valu_per_execution": per, "valu_total_static": sum(per.values()),
            "blocks": per_block,
            "isa": "release flags + -gline-tables-only (ISA checked identical); each VALU "
                   "instruction assigned by its ISA loop and its inline chain (llvm-symbolizer)"}


PATCHES = [
    ("__device__ __forceinline__ uint32_t pack(",
     "__device__ unsigned long long g_vblock_cnt[7];\n"
     "__device__ unsigned long long g_vblock_waves;\n"
     "__device__ uint32_t g_cnt_slot_dummy;\n"
     "__device__ __forceinline__ uint32_t first_lane_here() {\n"
     "  const uint64_t e = __builtin_amdgcn_read_exec();\n"
     "  return (uint32_t)((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(e));\n"
     "}\n"
     "__device__ __forceinline__ uint32_t pack("),
    # lraycast_t: one shadow ray per call (setup) and its steps
    ("                           uint32_t& work) {\n  float dist = 0.0f;\n",
     "                           uint32_t& work, uint32_t* cnt) {\n  cnt[4] += first_lane_here();\n"
     "  float dist = 0.0f;\n"),
    ("  for (uint32_t i = 0; i < maxIter && dist < maxDist; i++) {\n    work++;\n",
     "  for (uint32_t i = 0; i < maxIter && dist < maxDist; i++) {\n    work++;\n"
     "    cnt[5] += first_lane_here();\n"),
]


def build():
    """The instrumented copy: counters threaded through by a per-lane array passed down."""
    if os.path.exists(BASE):
        shutil.rmtree(BASE)
    os.makedirs(OUT)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(BASE, "include"))
    shutil.copy(os.path.join(PKG, "Makefile"), OUT)
    shutil.copytree(os.path.join(PKG, "csrc"), os.path.join(OUT, "csrc"))
    p = os.path.join(OUT, "csrc", "voxel_trace.hip")
    s = open(p).read()
    for old, new in PATCHES:
        if s.count(old) != 1:
            raise SystemExit(f"patch anchor not found once: {old[:60]!r}")
        s = s.replace(old, new)
    # thread `cnt` through the call chain: work is already passed everywhere; add cnt beside it
    s = s.replace("uint32_t& work) {", "uint32_t& work, uint32_t* cnt) {")
    s = s.replace("uint32_t& work, uint32_t* cnt, uint32_t* cnt) {", "uint32_t& work, uint32_t* cnt) {")
    s = re.sub(r"(lraycast(?:_t<(?:true|false)>)?\(f, pos, [^;]*?), work\)", r"\1, work, cnt)", s)
    s = re.sub(r"(shade_hit<RECIP>\([^;]*?), work\)", r"\1, work, cnt)", s)
    s = re.sub(r"(raycast_t<(?:true|false)>\(f, dir, yscale, atan_dir), work\)", r"\1, work, cnt)", s)
    s = s.replace("float atan_dir, uint32_t& work) {", "float atan_dir, uint32_t& work, uint32_t* cnt) {")
    for old, new in [
        ("  for (uint32_t i = 0; dist < f.view_distance && i < f.maxiter; i++) {\n    work++;\n",
         "  for (uint32_t i = 0; dist < f.view_distance && i < f.maxiter; i++) {\n    work++;\n"
         "    cnt[0] += first_lane_here();\n"),
        ("      const VoxDyn& d = f.dyn[DI];\n",
         "      const VoxDyn& d = f.dyn[DI];\n      cnt[1] += first_lane_here();\n"),
        ("  uint32_t c;\n  if (id < 0) {", "  cnt[2] += first_lane_here();\n  uint32_t c;\n  if (id < 0) {"),
        ("    const VoxLight L = light_at(f.lights, j);\n",
         "    const VoxLight L = light_at(f.lights, j);\n    cnt[3] += first_lane_here();\n"),
        ("    if (!__builtin_amdgcn_ballot_w64(ddf < L.dd_skip)) continue;\n",
         "    if (!__builtin_amdgcn_ballot_w64(ddf < L.dd_skip)) continue;\n"
         "    cnt[6] += first_lane_here();\n"),
        ("  uint32_t work = 0;\n  const int i = f.xstart", "  uint32_t work = 0;\n"
         "  uint32_t cnt[7] = {0, 0, 0, 0, 0, 0, 0};\n  const int i = f.xstart"),
        ("f.col[3 * i + 2], work);", "f.col[3 * i + 2], work, cnt);"),
        ("  if (f.tile_cost) {\n    // the tile's slowest ray",
         "  for (int q = 0; q < 7; q++) {\n    uint32_t v = cnt[q];\n"
         "    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);\n"
         "    if (lane == 0) atomicAdd(&g_vblock_cnt[q], (unsigned long long)v);\n  }\n"
         "  if (lane == 0) atomicAdd(&g_vblock_waves, 1ull);\n"
         "  if (f.tile_cost) {\n    // the tile's slowest ray"),
        ("}  // namespace\n\nlong long voxel_tile_key(",
         "}  // namespace\n\n"
         "extern \"C\" __attribute__((visibility(\"default\"))) int sfrt_voxel_block_counts("
         "unsigned long long* out, int reset) {\n"
         "  if (hipDeviceSynchronize() != hipSuccess) return -1;\n"
         "  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vblock_cnt), 7 * 8) != hipSuccess) return -1;\n"
         "  if (hipMemcpyFromSymbol(out + 7, HIP_SYMBOL(g_vblock_waves), 8) != hipSuccess) return -1;\n"
         "  if (reset) {\n    unsigned long long z[8] = {};\n"
         "    if (hipMemcpyToSymbol(HIP_SYMBOL(g_vblock_cnt), z, 7 * 8) != hipSuccess) return -1;\n"
         "    if (hipMemcpyToSymbol(HIP_SYMBOL(g_vblock_waves), z, 8) != hipSuccess) return -1;\n"
         "  }\n  return 0;\n}\n\nlong long voxel_tile_key("),
    ]:
        if s.count(old) != 1:
            raise SystemExit(f"patch anchor not found once: {old[:60]!r}")
        s = s.replace(old, new)
    open(p, "w").write(s)
    subprocess.run(["make", "-s", "-j", "8", "-C", OUT, "EXTRA=-DSFRT_VOXEL_BLOCK_PROFILE"], check=True)
    print(os.path.join(OUT, "libsfrt.so"))


def run():
    os.environ["SFRT_LIB"] = os.path.join(OUT, "libsfrt.so")
    sys.path.insert(0, PKG)
    import torch
    import voxel_scenes as vs
    import sfrt
    L = sfrt.lib()
    L.sfrt_voxel_block_counts.argtypes = [ctypes.c_void_p, ctypes.c_int]
    v = sfrt.VoxelWorld(0)
    tex, dyn = vs.load_textures()
    v.load_assets(tex, dyn, vs.COLORS)
    out = (ctypes.c_ulonglong * 8)()
    res = {}
    for w, h in ((1920, 1080), (3840, 2160)):
        v.set_scene(vs.default_world((15.5, 1.9, 15.5), 0.0, 0.0), w, h)
        buf = torch.empty(h, w * 4, dtype=torch.uint8, device="cuda")
        v.render_band(buf.data_ptr(), w * 4, 0, h, 0)
        L.sfrt_voxel_block_counts(out, 1)
        frames = 3
        for _ in range(frames):
            v.render_band(buf.data_ptr(), w * 4, 0, h, 0)
        v.check()
        L.sfrt_voxel_block_counts(out, 1)
        c = list(out)
        waves = c[7]
        res[str(w * h)] = {"frame": f"{w}x{h}", "waves": waves // frames,
                           "per_wave": {k: round(c[q] / waves, 3) for q, k in enumerate(COUNTED)}}
    v.close()
    print(json.dumps({"tool": "tools/voxel_block_profile.py run",
                      "note": "block executions per wave (first active lane counts; instrumented "
                              "copy of the kernel, default world, pose (15.5,1.9,15.5)/(0,0))",
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
               "valu_per_wave": {k: round(x, 1) for k, x in valu.items()},
               "share": {k: round(x / tot, 4) for k, x in valu.items()},
               "predicted_valu_per_wave": round(tot, 1),
               "rare_valu_static": st["valu_per_execution"].get("rare", 0)}
        if pmc:
            t = pmc.get("per_launch_pixels", pmc.get("per_grid_threads", {})).get(key)
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
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r4q_voxel_traffic.json"))
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
