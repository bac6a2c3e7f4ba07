"""tools/isa_block_profile.py on the CPU: the instrumented copy of a kernel's assembly assembles,
keeps every original instruction in order, and counts each basic block exactly once per entry.

The GPU side (`run`) is what the round-5 attributions in profiles/r5*_blocks.json come from; here
the parts that need no GPU: block parsing, the instrumentation text, and the report arithmetic.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_block_profile as ibp  # noqa: E402


@pytest.fixture(scope="module")
def voxel_asm(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("ibp") / "voxel.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950"] + ibp.RELEASE_FLAGS +
                   ["-x", "hip", "--offload-device-only", "--no-gpu-bundle-output", "-S", "-o", out,
                    os.path.join("csrc", "voxel_trace.hip")], cwd=ibp.PKG, check=True,
                   stderr=subprocess.DEVNULL)
    return out


def test_blocks_cover_the_kernel(voxel_asm):
    lines = open(voxel_asm).read().split("\n")
    sym = ibp.KERNELS["voxel"]["symbol"]
    blocks = ibp.parse_blocks(lines, sym)
    text = ibp.kernel_text(lines, sym)
    assert sum(len(b["insts"]) for b in blocks) == len(text)
    assert [t for b in blocks for _, t in b["insts"]] == text
    assert any(b["header"] for b in blocks)  # loops found
    assert blocks[0]["insts"][0][1].startswith("s_")


def test_instrumented_copy_assembles_and_keeps_the_kernel(voxel_asm, tmp_path):
    lines = open(voxel_asm).read().split("\n")
    sym = ibp.KERNELS["voxel"]["symbol"]
    txt, blocks = ibp.instrument(lines, sym)
    inst = txt.split("\n")
    # one counter increment per block, the original instructions unchanged and in order
    assert sum(1 for ln in inst if ln.strip().startswith("v_writelane_b32")) == len(blocks)
    added = ("v_readlane_b32", "v_writelane_b32", "s_cselect_b32", "s_add_u32", "s_cmp_lg_u32",
             "s_nop", "v_mov_b32_e32", "s_mov_b64", "v_mbcnt_lo_u32_b32", "v_mbcnt_hi_u32_b32",
             "v_lshlrev_b32_e32", "s_getpc_b64", "s_addc_u32", "global_atomic_add", "s_waitcnt")
    orig = ibp.kernel_text(lines, sym)
    new = ibp.kernel_text(inst, sym)
    it = iter(new)
    for t in orig:  # orig is a subsequence of new; every extra line is one of ours
        for n in it:
            if n == t:
                break
            assert n.split()[0] in added, n
        else:
            raise AssertionError(f"instruction {t!r} lost")
    # the counter array the flush adds into is declared by the source patch; assemble against it
    src = txt + f"\n\t.globl\t{ibp.COUNTERS}\n\t.type\t{ibp.COUNTERS},@object\n" \
                f"\t.bss\n{ibp.COUNTERS}:\n\t.zero\t{4 * ibp.MAX_BLOCKS}\n"
    asm = tmp_path / "inst.s"
    asm.write_text(src)
    subprocess.run([ibp.LLVM + "/clang", "-cc1as", "-triple", "amdgcn-amd-amdhsa", "-filetype",
                    "obj", "-target-cpu", "gfx950", "-mrelocation-model", "pic", "-o",
                    str(tmp_path / "inst.o"), str(asm)], check=True)


def test_report_arithmetic_is_static_counts_times_executions(voxel_asm):
    lines = open(voxel_asm).read().split("\n")
    blocks = ibp.parse_blocks(lines, ibp.KERNELS["voxel"]["symbol"])
    ex = [float(k % 3) for k in range(len(blocks))]
    tot = {}
    for b, n in zip(blocks, ex):
        for _, t in b["insts"]:
            k = ibp.klass(t.split()[0])
            tot[k] = tot.get(k, 0.0) + n
    valu = sum(n * sum(1 for _, t in b["insts"] if t.startswith("v_")) for b, n in zip(blocks, ex))
    assert tot["valu"] == valu and tot["salu"] > 0 and tot["smem"] > 0
    assert ibp.klass("s_cbranch_execz") == "branch" and ibp.klass("s_waitcnt") == "other"
    assert ibp.klass("buffer_load_ubyte") == "vmem" and ibp.klass("s_load_dwordx4") == "smem"
    json.dumps(tot)
