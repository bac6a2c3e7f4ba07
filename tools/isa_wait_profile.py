"""Where a frame kernel's waves wait: shader cycles spent in each s_waitcnt, by source region.

    python tools/isa_wait_profile.py build  KERNEL   # here: timed libsfrt.so copy (+ block build)
    python tools/isa_wait_profile.py run    KERNEL   # GPU: cycles per wait site per launch (JSON)
    python tools/isa_wait_profile.py report KERNEL WAITS.json BBCOUNTS.json [--pmc TRAFFIC.json]

KERNEL as in tools/isa_block_profile.py (sphere = k_trace_window_r<4>, the headline).

Method.  The release kernel's assembly, split into basic blocks exactly as
tools/isa_block_profile.py does (its functions are reused), gets around every `s_waitcnt` outside
the tile sorter and the rare paths an `s_memtime` before and after it; the difference of the two
shader-clock stamps is added to the site's accumulator -- lane k % 64 of spare VGPR k / 64, read
and written with v_readlane / v_writelane (EXEC-independent, SCC saved and restored) -- and the
accumulators are added to a device array at s_endpgm.  Each site therefore costs one extra
`s_waitcnt lgkmcnt(0)` after the second stamp, outside the interval it measures, and an
`lgkmcnt(0)` site also waits for the first stamp's own return: its interval is at least that
stamp's latency (the calibration lanes measure it, at the wave's start and end, as a stamp pair
around an `lgkmcnt(0)` with nothing else outstanding).  A site with `lgkmcnt(k)`, k > 0, waits
for lgkmcnt(k + 1) instead (the stamp is the youngest scalar request; such sites only ever count
in-order requests).  Lanes 0-4: the wave's lifetime (end stamp minus entry stamp), the
calibration pair at the end and at the start, the number of waves, and the drain of the wave's
last stores before s_endpgm (which the release kernel's s_endpgm waits for implicitly).  At most 4 spare VGPRs
are used (the headline kernel has 60: 64 keep 8 waves per SIMD), so at most 251 sites.  Each wave
adds its lanes into the copy of its CU (XCC_ID and HW_ID), not into one array for the whole chip:
32,400 waves' atomics on the same two cache lines had tripled the kernel's time and queued its
own loads behind them.

`report` divides each site's cycles by its executions (the block counts of the same tree's
tools/isa_block_profile.py build) and sums cycles by the source regions of
tools/isa_block_profile.py, next to the wave lifetime and, with --pmc, the PMC pass's
SQ_WAIT_ANY / SQ_WAVE_CYCLES of the same launch.  Diagnostic only: the timed copy is never a
product library (flavour "ab").
"""
import argparse
import json
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_block_profile as ibp  # noqa: E402

TAG = "waits"
RESERVED = 5  # lanes: lifetime, calibration at the end and at the start, waves, end drain
MAX_VGPRS = 4
COPIES = 1024  # one accumulator copy per CU: XCC_ID (3 bits) and HW_ID's cu / sh / se (7 bits)
LANES = 64 * MAX_VGPRS


def excluded(chain_list, rare):
    return rare or any(fn.startswith("sort_tiles") for ch in chain_list for fn, _, _ in ch)


def select_sites(lines, symbol, co):
    """[(line index, block index, waitcnt text)] of the timed sites, and the skipped ones."""
    blocks = ibp.parse_blocks(lines, symbol)
    seq = [t.split()[0] for b in blocks for _, t in b["insts"]]
    ch = ibp.chains(co, symbol, len(seq))
    it = iter(ch)
    sites, skipped = [], 0
    for bi, b in enumerate(blocks):
        for (i, t) in b["insts"]:
            c = next(it)[1]
            if not t.startswith("s_waitcnt"):
                continue
            if excluded([c], b["rare"]):
                skipped += 1
                continue
            sites.append((i, bi, t))
    return blocks, sites, skipped


def instrument(lines, symbol, sites):
    d = ibp.descriptor(lines, symbol)
    (iv, nv), (is_, ns), (ia, acc) = d["next_free_vgpr"], d["next_free_sgpr"], d["accum_offset"]
    if acc < nv:
        raise SystemExit("AGPRs in use: not supported")
    nl = RESERVED + len(sites)
    ncv = (nl + 63) // 64
    if ncv > MAX_VGPRS:
        raise SystemExit(f"{len(sites)} sites need {ncv} VGPRs > {MAX_VGPRS}")
    vc = [nv + k for k in range(ncv)]
    s0 = (ns + 1) & ~1  # even: the stamp pairs
    sA, sB, sT, sU, sS = s0, s0 + 2, s0 + 4, s0 + 5, s0 + 6
    if sS > 101:
        raise SystemExit("no spare SGPRs")

    def acc_add(lane, val):
        v, l = vc[lane // 64], lane % 64
        return [f"\tv_readlane_b32 s{sU}, v{v}, {l}", "\ts_nop 4",
                f"\ts_add_u32 s{sU}, s{sU}, {val}",
                f"\tv_writelane_b32 v{v}, s{sU}, {l}", "\ts_nop 4"]

    def stamp_pair(lane):  # A; lgkmcnt(0); B; lgkmcnt(0); lane += B - A
        return [f"\ts_memtime s[{sA}:{sA + 1}]", "\ts_waitcnt lgkmcnt(0)",
                f"\ts_memtime s[{sB}:{sB + 1}]", "\ts_waitcnt lgkmcnt(0)",
                f"\ts_sub_u32 s{sT}, s{sB}, s{sA}"] + acc_add(lane, f"s{sT}")

    ins_before, replace = {}, {}
    st, en = ibp.function_range(lines, symbol)
    first = next(i for i in range(st + 1, en) if ibp.is_inst(lines[i]))
    ins_before[first] = ([f"\tv_mov_b32_e32 v{x}, 0" for x in vc] + ["\ts_nop 4"] +
                         [f"\ts_cselect_b32 s{sS}, -1, 0"] + stamp_pair(2) +
                         # lane 0 starts at minus the entry stamp
                         [f"\ts_memtime s[{sA}:{sA + 1}]", "\ts_waitcnt lgkmcnt(0)",
                          f"\ts_sub_u32 s{sT}, 0, s{sA}"] + acc_add(0, f"s{sT}") +
                         [f"\ts_cmp_lg_u32 s{sS}, 0"])
    for k, (i, _, t) in enumerate(sites):
        lane = RESERVED + k
        m = re.search(r"lgkmcnt\((\d+)\)", t)
        w = t
        if m and int(m.group(1)) > 0:
            n = int(m.group(1)) + 1
            if n > 15:
                raise SystemExit(f"{t}: lgkmcnt beyond 15")
            w = t[:m.start()] + f"lgkmcnt({n})" + t[m.end():]
        replace[i] = ([f"\ts_memtime s[{sA}:{sA + 1}]", "\t" + w,
                       f"\ts_memtime s[{sB}:{sB + 1}]", "\ts_waitcnt lgkmcnt(0)",
                       f"\ts_cselect_b32 s{sS}, -1, 0",
                       f"\ts_sub_u32 s{sT}, s{sB}, s{sA}"] + acc_add(lane, f"s{sT}") +
                      [f"\ts_cmp_lg_u32 s{sS}, 0"])
    for i in range(st + 1, en):
        if lines[i].strip().startswith("s_endpgm"):
            # the drain of the wave's last stores (s_endpgm's implicit wait in the release
            # kernel), timed like a site into lane 4
            end = [f"\ts_memtime s[{sA}:{sA + 1}]", "\ts_waitcnt vmcnt(0) lgkmcnt(0)",
                   f"\ts_memtime s[{sB}:{sB + 1}]", "\ts_waitcnt lgkmcnt(0)",
                   f"\ts_sub_u32 s{sT}, s{sB}, s{sA}"] + acc_add(4, f"s{sT}") + stamp_pair(1) + \
                  [f"\ts_memtime s[{sA}:{sA + 1}]", "\ts_waitcnt lgkmcnt(0)"] + \
                  acc_add(0, f"s{sA}") + acc_add(3, "1")
            flush = ["\ts_mov_b64 exec, -1",
                     "\tv_mbcnt_lo_u32_b32 v0, -1, 0",
                     "\tv_mbcnt_hi_u32_b32 v0, -1, v0",
                     "\tv_lshlrev_b32_e32 v0, 2, v0",
                     # the CU's copy: (XCC_ID << 7 | HW_ID[14:8]) * LANES * 4 bytes
                     f"\ts_getreg_b32 s{sT}, hwreg(HW_REG_XCC_ID, 0, 3)",
                     f"\ts_getreg_b32 s{sU}, hwreg(HW_REG_HW_ID, 8, 7)",
                     f"\ts_lshl_b32 s{sT}, s{sT}, 7",
                     f"\ts_or_b32 s{sT}, s{sT}, s{sU}",
                     f"\ts_mul_i32 s{sT}, s{sT}, {LANES * 4}",
                     f"\tv_add_u32_e32 v0, s{sT}, v0",
                     "\ts_getpc_b64 s[0:1]",
                     f"\ts_add_u32 s0, s0, {ibp.COUNTERS}@rel32@lo+4",
                     f"\ts_addc_u32 s1, s1, {ibp.COUNTERS}@rel32@hi+12",
                     "\ts_nop 4"]
            flush += [f"\tglobal_atomic_add v0, v{x}, s[0:1] offset:{256 * k}"
                      for k, x in enumerate(vc)]
            flush += ["\ts_waitcnt vmcnt(0)"]
            ins_before.setdefault(i, []).extend(end + flush)
    out = []
    for i, l in enumerate(lines):
        if i in ins_before:
            out.extend(ins_before[i])
        if i in replace:
            out.extend(replace[i])
            continue
        if i == iv:
            l = re.sub(r"\d+$", str(nv + ncv), l)
        elif i == is_:
            l = re.sub(r"\d+$", str(sS + 1), l)
        elif i == ia:
            l = re.sub(r"\d+$", str((nv + ncv + 3) // 4 * 4), l)
        out.append(l)
    return "\n".join(out), nl


def patch_source(src_text):
    """The per-CU accumulator copies and a reader summing them (sfrt_bbprof_read's signature,
    so tools/isa_block_profile.py run reads them)."""
    return src_text + f"""

// ---- isa_wait_profile.py instrumentation (copy only) ----
__device__ unsigned int {ibp.COUNTERS}[{COPIES * LANES}];
extern "C" __attribute__((visibility("default"))) int sfrt_bbprof_read(unsigned int* out, int reset) {{
  static unsigned int h[{COPIES * LANES}];
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL({ibp.COUNTERS}), sizeof h) != hipSuccess) return -1;
  for (int l = 0; l < {LANES}; l++) {{  // 64-bit sums as (low, high) words
    unsigned long long t = 0;
    for (int c = 0; c < {COPIES}; c++) t += h[c * {LANES} + l];
    out[2 * l] = (unsigned int)t;
    out[2 * l + 1] = (unsigned int)(t >> 32);
  }}
  if (reset) {{
    for (auto& x : h) x = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL({ibp.COUNTERS}), h, sizeof h) != hipSuccess) return -1;
  }}
  return 0;
}}
"""


def build(kind):
    """The timed copy, through isa_block_profile.build's pipeline with this instrumentation."""
    ibp.VARIANT["tag"] = TAG
    k = ibp.KERNELS[kind]
    state = {}

    def timed(lines, symbol):
        B = ibp.base(kind)
        orig = os.path.join(B, "orig_for_sites.s")
        open(orig, "w").write("\n".join(lines))
        co = ibp.assemble(orig, os.path.join(B, "orig_for_sites"))
        blocks, sites, skipped = select_sites(lines, symbol, co)
        txt, nl = instrument(lines, symbol, sites)
        state.update(sites=[{"line": i, "block": b, "text": t} for i, b, t in sites],
                     skipped=skipped, lanes=nl)
        return txt, [None] * (2 * nl)  # isa_block_profile.build records len(): two words a lane

    saved = ibp.instrument, ibp.patch_source
    ibp.instrument, ibp.patch_source = timed, patch_source
    try:
        ibp.build(kind)
    finally:
        ibp.instrument, ibp.patch_source = saved
    info_p = os.path.join(ibp.base(kind), "info.json")
    info = json.load(open(info_p))
    info.update(state)
    json.dump(info, open(info_p, "w"))
    print(f"{len(state['sites'])} timed sites, {state['skipped']} skipped (sorter, rare paths)")


def run(kind):
    ibp.VARIANT["tag"] = TAG
    ibp.run(kind)


def report(kind, waits_path, counts_path, pmc_path):
    ibp.VARIANT["tag"] = TAG
    B = ibp.base(kind)
    info = json.load(open(os.path.join(B, "info.json")))
    sym = ibp.KERNELS[kind]["symbol"]
    lines = open(os.path.join(B, "orig.s")).read().split("\n")
    blocks = ibp.parse_blocks(lines, sym)
    seq = [t.split()[0] for b in blocks for _, t in b["insts"]]
    ch = ibp.chains(os.path.join(B, "orig.co"), sym, len(seq))
    it = iter(ch)
    for b in blocks:
        b["chains"] = [next(it)[1] for _ in b["insts"]]
    region = ibp.REGIONS[kind](blocks)
    line_region = {}
    for b in blocks:
        rs = [region(b, c) for c in b["chains"]]
        known = [r for r in rs if r is not None]
        prev = known[0] if known else "unattributed"
        for (i, _), r in zip(b["insts"], rs):
            prev = r if r is not None else prev
            line_region[i] = prev
    waits = json.load(open(waits_path))
    counts = json.load(open(counts_path))
    pmc = json.load(open(pmc_path)) if pmc_path else None
    out = {"tool": "tools/isa_wait_profile.py report", "kernel": sym,
           "waits": os.path.relpath(waits_path, ibp.ROOT),
           "counts": os.path.relpath(counts_path, ibp.ROOT), "launches": {}}
    for key, ent in waits["launches"].items():
        w = ent["block_executions_per_launch"]  # (low, high) words of each lane's sum
        lanes = [w[2 * i] + w[2 * i + 1] * 4294967296.0 for i in range(len(w) // 2)]
        ex = counts["launches"][key]["block_executions_per_launch"]
        if len(ex) != len(blocks):
            raise SystemExit("block counts for a different block table")
        waves = lanes[3]
        life, cal_end, cal_start = lanes[0], lanes[1] / waves, lanes[2] / waves
        by_region, sites = {}, []
        total = 0.0
        for k, s in enumerate(info["sites"]):
            cyc = lanes[RESERVED + k]
            n = ex[s["block"]]
            total += cyc
            r = line_region.get(s["line"], "unattributed")
            d = by_region.setdefault(r, {"cycles_per_launch": 0.0, "executions_per_launch": 0.0})
            d["cycles_per_launch"] += cyc
            d["executions_per_launch"] += n
            sites.append({"site": s["text"], "line": s["line"], "region": r,
                          "executions_per_launch": round(n, 1),
                          "cycles_per_execution": round(cyc / n, 1) if n else None,
                          "share_of_lifetime": round(cyc / life, 5)})
        for r, d in by_region.items():
            d["share_of_lifetime"] = round(d["cycles_per_launch"] / life, 5)
            d["cycles_per_execution"] = round(d["cycles_per_launch"] / d["executions_per_launch"], 1) \
                if d["executions_per_launch"] else None
            d["cycles_per_launch"] = round(d["cycles_per_launch"])
            d["executions_per_launch"] = round(d["executions_per_launch"], 1)
        row = {"frame": ent["frame"], "waves": round(waves, 1),
               "end_store_drain_cycles_mean": round(lanes[4] / waves, 1),
               "end_store_drain_share_of_lifetime": round(lanes[4] / life, 5),
               "wave_lifetime_cycles_mean": round(life / waves, 1),
               "stamp_pair_cycles_start": round(cal_start, 1),
               "stamp_pair_cycles_end": round(cal_end, 1),
               "timed_wait_share_of_lifetime": round(total / life, 5),
               "by_region": dict(sorted(by_region.items(), key=lambda x: -x[1]["cycles_per_launch"])),
               "top_sites": sorted(sites, key=lambda x: -x["share_of_lifetime"])[:25]}
        if pmc:
            t = pmc.get("per_launch_pixels", {}).get(key)
            if t and "SQ_WAIT_ANY" in t:
                row["pmc_SQ_WAIT_ANY_over_SQ_WAVE_CYCLES"] = round(t["SQ_WAIT_ANY"] / t["SQ_WAVE_CYCLES"], 5)
                row["pmc_source"] = os.path.relpath(pmc_path, ibp.ROOT)
        out["launches"][key] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("build", "run", "report"))
    ap.add_argument("kernel", choices=sorted(ibp.KERNELS))
    ap.add_argument("waits", nargs="?")
    ap.add_argument("counts", nargs="?")
    ap.add_argument("--pmc", default=None)
    a = ap.parse_args()
    if a.mode == "build":
        build(a.kernel)
    elif a.mode == "run":
        run(a.kernel)
    else:
        report(a.kernel, a.waits, a.counts, a.pmc)
