"""Exact instruction counts by basic block for the three frame kernels (VALU, SALU, SMEM, ...).

    python tools/isa_block_profile.py build  KERNEL   # here: instrumented libsfrt.so copy
    python tools/isa_block_profile.py run    KERNEL   # GPU: block executions per launch (JSON)
    python tools/isa_block_profile.py report KERNEL COUNTS.json [--pmc profiles/<tag>_traffic.json]

KERNEL is one of: sphere (k_trace_window_r<4>, the headline), voxel (k_voxel_ordered), glsl
(k_glsl_ordered).

Method.  The release kernel's assembly (hipcc -S of the product source, release flags plus
-gline-tables-only, which only adds .loc directives: the kernel's instruction text is checked
identical to the plain release build's) is split into its basic blocks (every `.LBBn_m:` label
and `; %bb.n:` marker).  An instrumented copy of that same assembly gets, at the top of every
block, a scalar increment of the block's counter -- lane b % 64 of spare VGPR b / 64, read and
written with v_readlane / v_writelane, which ignore EXEC, so a block counts once per wave
execution whatever lanes are active; SCC is saved and restored around the add -- and, before
s_endpgm, one global atomic add per counter VGPR into a device array.  Nothing else of the kernel
changes: the original instructions, their order and their registers are the release build's,
so the control flow and every block's executions are the release kernel's.  The tool assembles
and links that copy with the commands hipcc itself runs (-###), builds libsfrt.so around it
(flavour "ab", never a product library), and `run` renders the bench workloads through it.

`report` multiplies each block's executions by its static instruction counts (from the
unmodified assembly) and prints, per launch size, the predicted VALU / SALU / SMEM / VMEM / LDS /
branch instructions per wave next to the PMC pass's SQ_INSTS_* / SQ_WAVES, and a VALU and SALU
attribution by source region (each instruction's region from its inline chain,
llvm-symbolizer --inlining on the code object of the unmodified assembly, and the ISA loop it
sits in).  Unlike round 4's tools/voxel_block_profile.py and glsl_block_profile.py (source-level counters
that charge a region's whole static code to every execution, 1.29x and 1.036x over PMC in round
4) the totals here are exact by construction: they should equal PMC to the counters' noise.
"""
import argparse
import ctypes
import json
import os
import re
import shlex
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sfml-software-raytracer_amd")
LLVM = "/opt/rocm/lib/llvm/bin"
FLAGS = ["-DSFRT_BUILD_FLAVOUR=\"ab\"", "-O3", "-fno-slp-vectorize", "-std=c++17", "-fPIC",
         "-fvisibility=hidden", "-ffp-contract=off", "-fno-fast-math", "-I../include", "-Icsrc"]
RELEASE_FLAGS = [f.replace('"ab"', '"release"') for f in FLAGS]
COUNTERS = "g_sfrt_bbprof"
MAX_BLOCKS = 64 * 12

KERNELS = {
    "sphere": {"src": "sphere_trace.hip", "obj": "sphere_trace.o",
               "symbol": "_ZN4sfrt12_GLOBAL__N_116k_trace_window_rILi4EEEvNS_10InlineArgsE"},
    # k_voxel_ordered<false>: the launch without tile costs (the voxel default)
    "voxel": {"src": "voxel_trace.hip", "obj": "voxel_trace.o",
              "symbol": "_ZN4sfrt12_GLOBAL__N_115k_voxel_orderedILb0EEEvNS_8VoxFrameEii"},
    "glsl": {"src": "glsl_trace.hip", "obj": "glsl_trace.o",
             "symbol": "_ZN4sfrt12_GLOBAL__N_114k_glsl_orderedENS_9GlslFrameEi"},
}


VARIANT = {"tag": "", "defines": []}  # --variant TAG -DNAME=V ...: an A/B build's counts


def base(kind):
    return os.path.join(PKG, f"build_bbprof_{kind}" + (f"_{VARIANT['tag']}" if VARIANT["tag"] else ""))


# ------------------------------------------------------------------------------------------
# assembly parsing

def function_range(lines, symbol):
    st = next(i for i, l in enumerate(lines) if l.startswith(symbol + ":"))
    en = next(i for i in range(st, len(lines)) if re.match(r"^\.Lfunc_end\d+:", lines[i]))
    return st, en


def is_inst(line):
    t = line.strip()
    return bool(t) and not t.startswith((".", ";")) and not t.endswith(":")


def parse_blocks(lines, symbol):
    """Basic blocks of `symbol` in order: dict(start = index of the first line after the block's
    label, name, header, parent, insts = [(line index, instruction text)], rare)."""
    st, en = function_range(lines, symbol)
    blocks, cur = [], None
    for i in range(st + 1, en):
        line = lines[i]
        m = re.match(r"^(\.LBB\d+_\d+):(.*)", line) or re.match(r"^; (%bb\.\d+):(.*)", line)
        if m:
            cur = {"name": m.group(1), "start": i + 1, "header": None, "parent": None,
                   "insts": [], "rare": False}
            blocks.append(cur)
            tail = m.group(2)
        else:
            if cur is None:
                if not is_inst(line):
                    continue
                cur = {"name": "entry", "start": i, "header": None, "parent": None,
                       "insts": [], "rare": False}
                blocks.append(cur)
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
        if t == "; keep_branch":
            cur["rare"] = True  # keep_branch() (sfrt_device.h): its asm comment marks a rare path
        if is_inst(line):
            cur["insts"].append((i, t.split(";")[0].strip()))
    return [b for b in blocks if b["insts"] or b["name"] != "entry"]


def klass(mn):
    if mn.startswith("v_"):
        return "valu"
    if mn.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime", "s_dcache")):
        return "smem"
    if mn.startswith(("s_branch", "s_cbranch", "s_setpc", "s_swappc")):
        return "branch"
    if mn.startswith(("s_waitcnt", "s_nop", "s_endpgm", "s_barrier", "s_sleep", "s_setprio",
                      "s_sendmsg", "s_trap", "s_sched", "s_delay")):
        return "other"
    if mn.startswith("s_"):
        return "salu"
    if mn.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if mn.startswith("ds_"):
        return "lds"
    return "other"


def descriptor(lines, symbol):
    st = next(i for i, l in enumerate(lines) if l.strip() == f".amdhsa_kernel {symbol}")
    en = next(i for i in range(st, len(lines)) if l_strip(lines[i]) == ".end_amdhsa_kernel")
    out = {}
    for i in range(st, en):
        m = re.match(r"\s*\.amdhsa_(next_free_vgpr|next_free_sgpr|accum_offset)\s+(\d+)", lines[i])
        if m:
            out[m.group(1)] = (i, int(m.group(2)))
    return out


def l_strip(s):
    return s.strip()


def kernel_text(lines, symbol):
    """The kernel's instructions, directives and comments dropped (the ISA-identity check)."""
    st, en = function_range(lines, symbol)
    return [l.split(";")[0].strip() for l in lines[st + 1:en] if is_inst(l)]


# ------------------------------------------------------------------------------------------
# instrumentation

def instrument(lines, symbol):
    """The instrumented assembly (list of lines) and the block table."""
    blocks = parse_blocks(lines, symbol)
    nb = len(blocks)
    if nb > MAX_BLOCKS:
        raise SystemExit(f"{nb} blocks > {MAX_BLOCKS}")
    d = descriptor(lines, symbol)
    (iv, nv), (is_, ns), (ia, acc) = d["next_free_vgpr"], d["next_free_sgpr"], d["accum_offset"]
    if acc < nv:
        raise SystemExit("AGPRs in use: not supported")
    ncv = (nb + 63) // 64
    vc = [nv + k for k in range(ncv)]
    s_t, s_s = ns, ns + 1
    if s_s > 101:
        raise SystemExit("no spare SGPRs")
    ins = {}  # line index -> lines to insert before it
    for b, bl in enumerate(blocks):
        v, lane = vc[b // 64], b % 64
        code = [f"\ts_cselect_b32 s{s_s}, -1, 0",
                f"\tv_readlane_b32 s{s_t}, v{v}, {lane}",
                "\ts_nop 4",
                f"\ts_add_u32 s{s_t}, s{s_t}, 1",
                f"\tv_writelane_b32 v{v}, s{s_t}, {lane}",
                "\ts_nop 4",
                f"\ts_cmp_lg_u32 s{s_s}, 0"]
        if b == 0:
            code = [f"\tv_mov_b32_e32 v{x}, 0" for x in vc] + ["\ts_nop 4"] + code
        ins.setdefault(bl["start"], []).extend(code)
    st, en = function_range(lines, symbol)
    for i in range(st + 1, en):
        if lines[i].strip().startswith("s_endpgm"):
            flush = ["\ts_mov_b64 exec, -1",
                     "\tv_mbcnt_lo_u32_b32 v0, -1, 0",
                     "\tv_mbcnt_hi_u32_b32 v0, -1, v0",
                     "\tv_lshlrev_b32_e32 v0, 2, v0",
                     "\ts_getpc_b64 s[0:1]",
                     f"\ts_add_u32 s0, s0, {COUNTERS}@rel32@lo+4",
                     f"\ts_addc_u32 s1, s1, {COUNTERS}@rel32@hi+12",
                     "\ts_nop 4"]
            flush += [f"\tglobal_atomic_add v0, v{x}, s[0:1] offset:{256 * k}"
                      for k, x in enumerate(vc)]
            flush += ["\ts_waitcnt vmcnt(0)"]
            ins.setdefault(i, []).extend(flush)
    out = []
    for i, l in enumerate(lines):
        if i in ins:
            out.extend(ins[i])
        if i == iv:
            l = re.sub(r"\d+$", str(nv + ncv), l)
        elif i == is_:
            l = re.sub(r"\d+$", str(ns + 2), l)
        elif i == ia:
            l = re.sub(r"\d+$", str((nv + ncv + 3) // 4 * 4), l)
        out.append(l)
    # the metadata's register counts (informational; kept consistent with the descriptor)
    txt = "\n".join(out)
    return txt, blocks


def patch_source(src_text):
    """The counter array and its host reader, appended to the copy of the kernel source (the
    kernels' ISA is checked unchanged by this)."""
    return src_text + f"""

// ---- isa_block_profile.py instrumentation (copy only) ----
__device__ unsigned int {COUNTERS}[{MAX_BLOCKS}];
extern "C" __attribute__((visibility("default"))) int sfrt_bbprof_read(unsigned int* out, int reset) {{
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL({COUNTERS}), sizeof {COUNTERS}) != hipSuccess) return -1;
  if (reset) {{
    static unsigned int z[{MAX_BLOCKS}];
    if (hipMemcpyToSymbol(HIP_SYMBOL({COUNTERS}), z, sizeof z) != hipSuccess) return -1;
  }}
  return 0;
}}
"""


def hipcc_commands(src, out_obj, extra, cwd):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950"] + FLAGS + extra + \
          ["-x", "hip", "-c", src, "-o", out_obj, "-save-temps=obj", "-###"]
    p = subprocess.run(cmd, capture_output=True, text=True, check=True, cwd=cwd)
    return [shlex.split(l) for l in p.stderr.splitlines() if l.startswith(' "')]


def device_asm_step(c):
    return "-S" in c and "-cc1" in c and "-triple" in c and \
        c[c.index("-triple") + 1] == "amdgcn-amd-amdhsa"


def build(kind):
    k = KERNELS[kind]
    B = base(kind)
    if os.path.exists(B):
        shutil.rmtree(B)
    out = os.path.join(B, "pkg")
    os.makedirs(out)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(B, "include"))
    shutil.copy(os.path.join(PKG, "Makefile"), out)
    shutil.copytree(os.path.join(PKG, "csrc"), os.path.join(out, "csrc"))
    srcp = os.path.join(out, "csrc", k["src"])
    text = patch_source(open(srcp).read())
    open(srcp, "w").write(text)
    obj = os.path.join(out, "build", k["obj"])
    os.makedirs(os.path.dirname(obj))
    # the plain release kernel, for the identity check
    rel = os.path.join(B, "release.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950"] + RELEASE_FLAGS +
                   VARIANT["defines"] + ["-x", "hip", "--offload-device-only", "--no-gpu-bundle-output", "-S", "-o", rel,
                    os.path.join(PKG, "csrc", k["src"])], cwd=PKG, check=True,
                   stderr=subprocess.DEVNULL)
    cmds = hipcc_commands(os.path.join("csrc", k["src"]), obj,
                          ["-gline-tables-only"] + VARIANT["defines"], out)
    info = None
    for c in cmds:
        subprocess.run(c, cwd=out, check=True)
        if device_asm_step(c):
            asm = c[c.index("-o") + 1]
            asm = asm if os.path.isabs(asm) else os.path.join(out, asm)
            lines = open(asm).read().split("\n")
            if kernel_text(lines, k["symbol"]) != kernel_text(open(rel).read().split("\n"),
                                                              k["symbol"]):
                raise SystemExit("the patched line-table copy's kernel ISA differs from the "
                                 "release build's")
            shutil.copy(asm, os.path.join(B, "orig.s"))
            txt, blocks = instrument(lines, k["symbol"])
            open(asm, "w").write(txt)
            info = {"kernel": k["symbol"], "blocks": len(blocks)}
    if info is None:
        raise SystemExit("no device assembly step in hipcc's pipeline")
    # the unmodified assembly as a code object, for the inline chains of `report`
    co = assemble(os.path.join(B, "orig.s"), os.path.join(B, "orig"))
    info["code_object"] = os.path.relpath(co, ROOT)
    subprocess.run(["make", "-s", "-j", "8", "-C", out,
                    "EXTRA=-DSFRT_BBPROF " + " ".join(VARIANT["defines"])], check=True)
    json.dump(info, open(os.path.join(B, "info.json"), "w"))
    print(os.path.join(out, "libsfrt.so"), info)


def assemble(asm, stem):
    o, co = stem + ".o", stem + ".co"
    subprocess.run([LLVM + "/clang", "-cc1as", "-triple", "amdgcn-amd-amdhsa", "-filetype", "obj",
                    "-target-cpu", "gfx950", "-mrelocation-model", "pic", "-o", o, asm], check=True)
    subprocess.run([LLVM + "/ld.lld", "-shared", "-o", co, o], check=True)
    return co


# ------------------------------------------------------------------------------------------
# GPU run: the bench workloads through the instrumented library

def run(kind, frames=3):
    os.environ["SFRT_LIB"] = os.path.join(base(kind), "pkg", "libsfrt.so")
    sys.path.insert(0, PKG)
    import numpy as np
    import torch
    import sfrt
    L = sfrt.lib()
    L.sfrt_bbprof_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    info = json.load(open(os.path.join(base(kind), "info.json")))
    nb = info["blocks"]
    cnt = np.zeros(MAX_BLOCKS, np.uint32)
    res = {}

    def measure(key, label, draw):
        draw()
        draw()
        draw()  # steady state: the ordered launches use the order of two frames back
        torch.cuda.synchronize()
        L.sfrt_bbprof_read(cnt.ctypes.data, 1)
        for _ in range(frames):
            draw()
        torch.cuda.synchronize()
        if L.sfrt_bbprof_read(cnt.ctypes.data, 1) != 0:
            raise SystemExit("counter read failed")
        c = cnt[:nb].astype(np.float64) / frames
        res[key] = {"frame": label, "block_executions_per_launch": [round(x, 3) for x in c]}

    if kind == "voxel":
        import voxel_scenes as vs
        v = sfrt.VoxelWorld(0)
        tex, dyn = vs.load_textures()
        v.load_assets(tex, dyn, vs.COLORS)
        for w, h in ((1920, 1080), (3840, 2160)):
            v.set_scene(vs.default_world((15.5, 1.9, 15.5), 0.0, 0.0), w, h)
            buf = torch.empty(h, w * 4, dtype=torch.uint8, device="cuda")
            measure(str(w * h), f"{w}x{h}",
                    lambda: v.render_band(buf.data_ptr(), w * 4, 0, h, 0))
        v.check()
        v.close()
    elif kind == "glsl":
        import glsl_scenes as gs
        import scenes
        s = sfrt.GlslShader(0)
        s.set_ground(*scenes.load_floor())
        for w, h in ((1920, 1080), (3840, 2160)):
            s.set_uniforms(gs.default_uniforms(w, h))
            buf = torch.empty(h, w * 4, dtype=torch.uint8, device="cuda")
            measure(str(w * h + 64), f"{w}x{h} (ordered: + the sorter workgroup)",
                    lambda: s.draw(buf.data_ptr(), w, h, w * 4, 0, h, 0))
        s.check()
        s.close()
    else:
        import scenes
        wd = sfrt.World(0)
        wd.load_texture(*scenes.load_floor())
        w, h = 3840, 2160
        wd.set_scene(scenes.lcg64(), w, h)
        buf = torch.empty(h, w * 4, dtype=torch.uint8, device="cuda")
        measure(str(w * h + 256), f"{w}x{h} lcg64 pose (0,0), adaptive order (+ the sorter)",
                lambda: wd.render_band(buf.data_ptr(), w * 4, 0, h, 0))
        wd.check()
        wd.close()
    print(json.dumps({"tool": "tools/isa_block_profile.py run", "kernel": info["kernel"],
                      "blocks": nb, "frames": frames, "launches": res}))


# ------------------------------------------------------------------------------------------
# report

def chains(co, symbol, n_expected):
    dis = subprocess.run([LLVM + "/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                         capture_output=True, text=True).stdout.splitlines()
    st = next(i for i, l in enumerate(dis) if l.endswith(f"<{symbol}>:"))
    insts = []
    for l in dis[st + 1:]:
        if l.strip() == "" or l.endswith(">:"):
            if insts:
                break
            continue
        m = re.match(r"\s+(\S+).*//\s+([0-9A-Fa-f]+):", l)
        if m:
            insts.append((m.group(1), int(m.group(2), 16)))
    insts = insts[:n_expected]
    sym = subprocess.run([LLVM + "/llvm-symbolizer", "--obj=" + co, "--inlining",
                          "--functions=short"], input="".join(f"0x{a:x}\n" for _, a in insts),
                         check=True, capture_output=True, text=True).stdout
    frames = [f.strip().splitlines() for f in sym.strip().split("\n\n")]
    out = []
    for (mn, _), fr in zip(insts, frames):
        ch = []
        for k in range(0, len(fr) - 1, 2):
            parts = fr[k + 1].split(":")
            ch.append((fr[k], os.path.basename(parts[0]),
                       int(parts[-2]) if len(parts) >= 3 and parts[-2].isdigit() else 0))
        out.append((mn, ch))
    return out


def src_anchor(kind, text):
    """Line of `text` in the build's own copy of the kernel source (its line tables' lines)."""
    src = open(os.path.join(base(kind), "pkg", "csrc", KERNELS[kind]["src"])).read()
    if src.count(text) != 1:
        raise SystemExit(f"anchor {text!r} found {src.count(text)} times")
    return src[:src.index(text)].count("\n") + 1 + text.count("\n")


class Loops:
    def __init__(self, blocks):
        self.parent = {b["name"]: b["parent"] for b in blocks if b["header"] == b["name"]}

    def inside(self, h, heads):
        while h:
            if h in heads:
                return True
            h = self.parent.get(h)
        return False

    def innermost(self, hs):
        def anc(h):
            out, h = set(), self.parent.get(h)
            while h:
                out.add(h)
                h = self.parent.get(h)
            return out
        return {h for h in hs if not any(h in anc(o) for o in hs if o != h)}


def frame_of(ch, prefix):
    for fn, f, line in ch:
        if fn.startswith(prefix):
            return fn, line
    return None, None


def loops_with(blocks, fname, line):
    return {b["header"] for b in blocks for ch in b["chains"]
            if b["header"] and frame_of(ch, fname) == (fname, line)}


def regions_voxel(blocks):
    A = {k: src_anchor("voxel", v) for k, v in {
        "main_loop": "float tryDist = dist + raySpeed;",
        "billboard_first": "V3 bp = pos;",
        "billboard_last": "dnext = DI < f.ndyn ? f.dyn[DI].dist : __builtin_nanf(\"\");\n        }",
        "light_loop": "const VoxLight L = light_at(lp, 0);",
        "shadow_loop": "raySpeed += 0.002f;",
        "light_skip": "if (!__builtin_amdgcn_ballot_w64(ddf < L.dd_skip)) continue;",
    }.items()}
    lp = Loops(blocks)
    main_h = lp.innermost(loops_with(blocks, "raycast_t<true>", A["main_loop"]))
    light_h = lp.innermost(loops_with(blocks, "shade_hit<true>", A["light_loop"]))
    shadow_h = lp.innermost(loops_with(blocks, "lraycast_t<true>", A["shadow_loop"]))
    if not (main_h and light_h and shadow_h):
        raise SystemExit(f"voxel loops not found: {main_h} {light_h} {shadow_h}")

    def region(b, ch):
        names = [fn for fn, _, _ in ch]
        if b["rare"] or any(n.startswith(("raycast_t<false>", "lraycast_t<false>")) for n in names):
            return "rare_plain_division"
        if any(n.startswith("sort_tiles") for n in names):
            return "sorter"
        h = b["header"]
        if "lraycast_t<true>" in names:
            return "shadow_step" if lp.inside(h, shadow_h) else "shadow_setup"
        if "shade_hit<true>" in names:
            if not lp.inside(h, light_h):
                return "shade"
            _, line = frame_of(ch, "shade_hit<true>")
            return "light_test" if line <= A["light_skip"] else "light"
        if lp.inside(h, light_h):
            return "light"  # lraycast()'s ballot (the shadow ray's division choice)
        fn, line = frame_of(ch, "raycast_t<true>")
        if fn and lp.inside(h, main_h):
            return "billboard" if A["billboard_first"] <= line <= A["billboard_last"] else "step"
        if fn:
            return "ray_setup_and_exit"
        return "kernel_entry_store"
    return region


def regions_glsl(blocks):
    """The regions of round 4's source-level GLSL tool: by the ISA loop and the line of fragment()."""
    A = {k: src_anchor("glsl", v) for k, v in {
        "wall_loop": "const bool inside = s <= w.s_in;",
        "wall_inside_first": "moved |= inside_mask;",
        "wall_inside_last": "total = total + tosurf;",
        "march_loop": "ball_dist += smooth + 0.01f;",
        "ball_loop": "const bool dominated = ssf >= bnd * bnd;",
        "ball_body_first": "const float ss = (ox * ox + oy * oy) + oz * oz;  // the shader's",
        "ball_body_last": "thr = fmaxf(fmaxf(smooth + 0.5f, shortest), 0.5f) * kThrMul + kThrAdd;\n      };",
        "ball_first_first": "if (nballs > 0) {",
        "ball_first_last": "thr = 1e30f;",
        "light_loop": "const float tlx = L.x - px, tly = L.y - py, tlz = L.z - pz;",
        "shadow_loop": "const float cosang = (-tnx * P.ux + -tny * P.uy) + -tnz * P.uz;",
        "shadow_body_first": "float sangle = sfrt_math::acosf(cosang);",
        "shadow_body_last": "shadow *= gclamp(sangle / P.sanglet",
        "texture": "// ---- wall or ball",
        "lighting": "// ---- lighting",
    }.items()}
    lp = Loops(blocks)

    def frag_line(ch):
        """The line of fragment() (or of a lambda inside it) the instruction belongs to."""
        for fn, f, ln in ch:
            if f == "glsl_trace.hip" and (fn.startswith("fragment") or fn.startswith("operator()")):
                return fn, ln
        return None, None

    def loops_at(line):
        return lp.innermost({b["header"] for b in blocks for ch in b["chains"]
                             if b["header"] and frag_line(ch)[1] == line})
    L = {k: loops_at(A[k]) for k in ("wall_loop", "march_loop", "ball_loop", "light_loop",
                                      "shadow_loop")}
    for k, v in L.items():
        if not v:
            raise SystemExit(f"glsl loop {k} not found")

    def region(b, ch):
        names = [fn for fn, _, _ in ch]
        if any(n.startswith("sort_tiles") for n in names):
            return "sorter"
        if any(n.startswith("wall_mask") for n in names):
            return "wall_cull"
        fn, line = frag_line(ch)
        if b["rare"]:
            return "rare"
        h = b["header"]
        inr = lambda a, z: line is not None and A[a] <= line <= A[z]
        if lp.inside(h, L["ball_loop"]):
            return "ball_body" if inr("ball_body_first", "ball_body_last") else "ball_test"
        if lp.inside(h, L["march_loop"]):
            # the step's first ball (specialized, or the lambda's body inlined for it)
            if inr("ball_first_first", "ball_first_last") or inr("ball_body_first", "ball_body_last"):
                return "ball_first"
            return "march_step"
        if lp.inside(h, L["wall_loop"]):
            return "wall_inside" if inr("wall_inside_first", "wall_inside_last") else "wall_test"
        if lp.inside(h, L["shadow_loop"]):
            return "shadow_body" if inr("shadow_body_first", "shadow_body_last") else "shadow_test"
        if lp.inside(h, L["light_loop"]):
            return "light"
        if fn is None or line is None or line < A["texture"]:
            return "setup"
        return "texture" if line < A["lighting"] else "colour_store"
    return region


def regions_sphere(blocks):
    """k_trace_window_r<4>: by helper function on the inline chain, else by the line of
    trace_tile_window_r (or of one of its lambdas) the instruction belongs to."""
    A = {k: src_anchor("sphere", v) for k, v in {
        "fn_first": "const int lane = threadIdx.x & 63;\n  P probe;",
        "windowed": "const bool windowed = f.cull && l0 > 0.0f;",
        "entry_lambda": "auto entry = [&](uint32_t e)",
        "advance_first": "auto advance = [&](const float (&L)[R]) {",
        "visit_first": "auto visit = [&](float cx, float cy, float cz",
        "visit_all_first": "auto visit_all = [&](float (&L)[R]) {",
        "slots_first": "if (kSlotsR > 0 && !full && __builtin_popcountll(m) <= kSlotsR) {",
        "slots_loop": "for (q = 0; q < kSlotsR; q++) visit(",
        "window_first": "uint32_t th = 0u;  // +0",
        "window_last": "m & __builtin_amdgcn_ballot_w64(lo < thi) & __builtin_amdgcn_ballot_w64(hi > tlo);",
        "visits_first": "if (win) {",
        "visits_last": "} while (more);",
        "full_loop": "for (; any_marching() && trips < kMaxIterations; ++trips) {",
        "tail_first": "if (trips >= kMaxIterations && any_marching() && lane == 0)",
        "fn_last": "probe.tile_end(px_out(0), lane_s, valid(0), trips, slot, m);",
    }.items() if k != "slots_loop"}
    helpers = [("sort_tiles", "sorter"), ("shade_texel", "shade"), ("shade_rgba", "shade"),
               ("primary_dir", "ray_setup"), ("tile_cone", "cull"), ("cull_window", "cull"),
               ("dist2", "visit_test"), ("pass_body_r", "pass_body"), ("zero_steps", "step_control")]

    def region(b, ch):
        for fn, f, line in ch:
            for h, r in helpers:
                if fn.startswith(h):
                    return r
        line = None
        for fn, f, ln in ch:
            if f == "sphere_trace.hip" and A["fn_first"] <= ln <= A["fn_last"]:
                line = ln
                break
        if line is None:
            return None  # no line (compiler-made): the region of its neighbours
        if line < A["windowed"]:
            return "ray_setup"
        if line < A["entry_lambda"]:
            return "cull"
        if A["advance_first"] <= line < A["visit_first"]:
            return "advance"
        if A["visit_all_first"] <= line < A["visit_all_first"] + 6:
            return "full_list"
        if A["window_first"] <= line <= A["window_last"]:
            return "window_upkeep"
        if A["visits_first"] <= line <= A["visits_last"]:
            return "visit_loop"
        if A["slots_first"] <= line < A["window_first"] - 4 and line < A["slots_first"] + 20:
            return "slots_setup" if line < A["slots_first"] + 20 - 2 else "step_control"
        if line >= A["tail_first"]:
            return "shade"
        if A["full_loop"] <= line < A["tail_first"]:
            return "full_list"
        return "step_control"
    return region


REGIONS = {"voxel": regions_voxel, "glsl": regions_glsl, "sphere": regions_sphere}


def report(kind, counts_path, pmc_path):
    B = base(kind)
    sym = KERNELS[kind]["symbol"]
    lines = open(os.path.join(B, "orig.s")).read().split("\n")
    blocks = parse_blocks(lines, sym)
    seq = [t.split()[0] for b in blocks for _, t in b["insts"]]
    ch = chains(os.path.join(B, "orig.co"), sym, len(seq))
    norm = lambda m: m[:-4] if m.endswith(("_e32", "_e64")) else m  # inline asm omits the suffix
    if [norm(mn) for mn, _ in ch] != [norm(m) for m in seq]:
        raise SystemExit("the code object's instruction sequence differs from the assembly's")
    it = iter(ch)
    for b in blocks:
        b["chains"] = [next(it)[1] for _ in b["insts"]]
    region = REGIONS[kind](blocks) if kind in REGIONS else (lambda b, c: "all")
    counts = json.load(open(counts_path))
    pmc = json.load(open(pmc_path)) if pmc_path else None
    out = {"tool": "tools/isa_block_profile.py report", "kernel": sym,
           "counts": os.path.relpath(counts_path, ROOT), "launches": {}}
    for key, ent in counts["launches"].items():
        ex = ent["block_executions_per_launch"]
        if len(ex) != len(blocks):
            raise SystemExit("counts for a different block table")
        tot, reg = {}, {}
        for b, n in zip(blocks, ex):
            rs = [region(b, c) for c in b["chains"]]
            # an instruction without a source line takes the region of the nearest one before
            # it in its block (else after it)
            known = [r for r in rs if r is not None]
            prev = known[0] if known else "unattributed"
            for i, r in enumerate(rs):
                if r is None:
                    rs[i] = prev
                else:
                    prev = r
            for (_, t), r in zip(b["insts"], rs):
                k = klass(t.split()[0])
                tot[k] = tot.get(k, 0.0) + n
                if k in ("valu", "salu"):
                    reg.setdefault(k, {})
                    reg[k][r] = reg[k].get(r, 0.0) + n
        row = {"frame": ent["frame"], "predicted_per_launch": {k: round(v) for k, v in tot.items()}}
        if pmc:
            t = pmc.get("per_launch_pixels", pmc.get("per_grid_threads", {})).get(key)
            if t:
                waves = t["SQ_WAVES"]
                row["pmc_source"] = os.path.relpath(pmc_path, ROOT)
                row["pmc_waves"] = waves
                cmp = {}
                for k, c in (("valu", "SQ_INSTS_VALU"), ("salu", "SQ_INSTS_SALU"),
                             ("smem", "SQ_INSTS_SMEM"), ("vmem", "SQ_INSTS_VMEM_RD"),
                             ("lds", "SQ_INSTS_LDS")):
                    if c in t and t[c]:
                        cmp[k] = {"pmc": round(t[c]), "predicted": round(tot.get(k, 0)),
                                  "predicted_over_pmc": round(tot.get(k, 0) / t[c], 4)}
                if "SQ_INSTS_SALU" in t:
                    cmp["salu+branch"] = {"predicted_over_pmc": round(
                        (tot.get("salu", 0) + tot.get("branch", 0)) / t["SQ_INSTS_SALU"], 4)}
                row["vs_pmc"] = cmp
                row["per_wave"] = {k: round(v / waves, 1) for k, v in tot.items()}
        for k, d in reg.items():
            s = sum(d.values())
            row[f"{k}_by_region"] = {r: {"per_launch": round(v), "share": round(v / s, 4)}
                                     for r, v in sorted(d.items(), key=lambda x: -x[1])}
        out["launches"][key] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("build", "run", "report"))
    ap.add_argument("kernel", choices=sorted(KERNELS))
    ap.add_argument("counts", nargs="?")
    ap.add_argument("--pmc", default=None)
    ap.add_argument("--variant", default="", help="A/B build: its own directory tag")
    ap.add_argument("-D", dest="defines", action="append", default=[],
                    help="NAME=V defines of the A/B build")
    a = ap.parse_args()
    VARIANT["tag"] = a.variant
    VARIANT["defines"] = ["-D" + d for d in a.defines]
    if a.mode == "build":
        build(a.kernel)
    elif a.mode == "run":
        run(a.kernel)
    else:
        report(a.kernel, a.counts, a.pmc)
