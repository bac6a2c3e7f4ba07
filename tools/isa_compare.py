"""Compare two builds' gfx950 ISA kernel by kernel (the release instantiation must not change
when code moves around it, e.g. the diagnostic probes behind sfrt_probe.h's NoProbe).

    python tools/isa_compare.py OLD.s NEW.s

Per kernel: VGPR / SGPR counts, scratch bytes and the instruction stream with labels, comments
and branch-target names stripped.  Exit 1 if any kernel differs.
"""
import re
import sys


def kernels(path):
    out, cur, meta = {}, None, {}
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m and not line.startswith("\t"):
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is None:
            continue
        if line.startswith("\t.end_amdhsa_kernel") or re.match(r"^\.Lfunc_end", line):
            cur = None
            continue
        s = line.split(";")[0].strip()
        if not s or s.endswith(":") or s.startswith("."):
            continue
        s = re.sub(r"\.LBB\d+_\d+", "L", s)
        out[cur].append(s)
    for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", open(path).read(), re.S):
        body = m.group(2)
        g = {k: re.search(rf"\.amdhsa_{k}\s+(\d+)", body) for k in
             ("next_free_vgpr", "next_free_sgpr", "private_segment_fixed_size", "accum_offset")}
        meta[m.group(1)] = {k: int(v.group(1)) for k, v in g.items() if v}
    return out, meta


def main():
    a, am = kernels(sys.argv[1])
    b, bm = kernels(sys.argv[2])
    bad = 0
    for k in sorted(set(a) | set(b)):
        if k not in a or k not in b:
            print(f"{'only old' if k in a else 'only new'}: {k}")
            bad += 1
            continue
        same = a[k] == b[k] and am.get(k) == bm.get(k)
        valu = sum(1 for s in b[k] if s.startswith("v_"))
        print(f"{'same' if same else 'DIFF'} {k[:70]:70s} insts {len(a[k])}->{len(b[k])} "
              f"v_ {valu} regs {am.get(k)} -> {bm.get(k)}")
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
