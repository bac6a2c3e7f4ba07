"""tools/isa_wait_profile.py on the CPU: the timed copy of a kernel's assembly brackets every timed
s_waitcnt with two s_memtime stamps, keeps every original instruction in order, stays within the
spare registers, and assembles.

The GPU side (`run`) is what profiles/r6f_*_waits.json come from ("Round 6").
"""
import os
import re
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_block_profile as ibp  # noqa: E402
import isa_wait_profile as iwp  # noqa: E402


@pytest.fixture(scope="module")
def voxel_build(tmp_path_factory):
    """The voxel kernel's release assembly with line tables (the sorter's sites are told apart by
    their inline chains) and its code object."""
    d = tmp_path_factory.mktemp("iwp")
    asm = str(d / "voxel.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950"] + ibp.RELEASE_FLAGS +
                   ["-gline-tables-only", "-x", "hip", "--offload-device-only", "--no-gpu-bundle-output",
                    "-S", "-o", asm, os.path.join("csrc", "voxel_trace.hip")], cwd=ibp.PKG, check=True,
                   stderr=subprocess.DEVNULL)
    co = ibp.assemble(asm, str(d / "voxel"))
    return asm, co


def test_timed_copy_brackets_every_site_and_keeps_the_kernel(voxel_build, tmp_path):
    asm, co = voxel_build
    lines = open(asm).read().split("\n")
    sym = ibp.KERNELS["voxel"]["symbol"]
    blocks, sites, skipped = iwp.select_sites(lines, sym, co)
    assert sites and skipped > 0  # the sorter's waits are left out
    assert all(t.startswith("s_waitcnt") for _, _, t in sites)
    txt, lanes = iwp.instrument(lines, sym, sites)
    assert lanes == iwp.RESERVED + len(sites)
    new = txt.split("\n")
    # each timed site: s_memtime, the (adjusted) wait, s_memtime, s_waitcnt lgkmcnt(0)
    stamps = [i for i, ln in enumerate(new) if ln.strip().startswith("s_memtime")]
    assert len(stamps) >= 2 * len(sites)
    for _, _, t in sites:
        m = re.search(r"lgkmcnt\((\d+)\)", t)
        want = t if not (m and int(m.group(1)) > 0) else \
            t[:m.start()] + f"lgkmcnt({int(m.group(1)) + 1})" + t[m.end():]
        assert any(new[i].strip() == want and new[i - 1].strip().startswith("s_memtime") and
                   new[i + 1].strip().startswith("s_memtime") for i in range(1, len(new) - 1)), t
    # the original instructions survive in order; every extra line is one of the tool's
    added = ("s_memtime", "s_waitcnt", "v_readlane_b32", "v_writelane_b32", "s_cselect_b32",
             "s_add_u32", "s_sub_u32", "s_cmp_lg_u32", "s_nop", "v_mov_b32_e32", "s_mov_b64",
             "v_mbcnt_lo_u32_b32", "v_mbcnt_hi_u32_b32", "v_lshlrev_b32_e32", "s_getreg_b32",
             "s_lshl_b32", "s_or_b32", "s_mul_i32", "v_add_u32_e32", "s_getpc_b64", "s_addc_u32",
             "global_atomic_add")
    timed = {i for i, _, _ in sites}
    orig = [t for i, t in ((i, t) for b in blocks for i, t in b["insts"]) if i not in timed]
    it = iter(ibp.kernel_text(new, sym))
    for t in orig:
        for n in it:
            if n == t:
                break
            assert n.split()[0] in added, n
        else:
            raise AssertionError(f"instruction {t!r} lost")
    # within the spare registers: the descriptor's VGPR count stays at 64 or below (8 waves/SIMD)
    d = iwp.ibp.descriptor(new, sym)
    assert d["next_free_vgpr"][1] <= 64 and d["next_free_sgpr"][1] <= 102
    src = txt + f"\n\t.globl\t{ibp.COUNTERS}\n\t.type\t{ibp.COUNTERS},@object\n" \
                f"\t.bss\n{ibp.COUNTERS}:\n\t.zero\t{4 * iwp.COPIES * iwp.LANES}\n"
    p = tmp_path / "timed.s"
    p.write_text(src)
    subprocess.run([ibp.LLVM + "/clang", "-cc1as", "-triple", "amdgcn-amd-amdhsa", "-filetype",
                    "obj", "-target-cpu", "gfx950", "-mrelocation-model", "pic", "-o",
                    str(tmp_path / "timed.o"), str(p)], check=True)


def test_patch_source_reads_64_bit_sums():
    src = iwp.patch_source("")
    assert f"[{iwp.COPIES * iwp.LANES}]" in src and "out[2 * l + 1]" in src
