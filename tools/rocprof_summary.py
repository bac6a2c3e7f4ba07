"""Summarise rocprofv3 CSV output of bench.py runs into profiles/.

    python tools/rocprof_summary.py --trace DIR --fetch DIR --write DIR --tag r1 [--sq DIR ...]
                                    [--kernel k_trace|k_glsl|k_voxel] [--out profiles]

Writes
  profiles/<tag>_kernel_stats_by_grid.csv  per (kernel, grid size): calls, avg/min/max ns
  profiles/<tag>_traffic.json              HBM bytes per launch of the trace kernels,
                                           keyed by pixels per launch (grid threads x
                                           pixels per thread),
                                           from separate --pmc FETCH_SIZE / WRITE_SIZE passes,
                                           and SQ_INSTS_VALU / SQ_WAVES per launch (--sq)
HBM bytes follow MI355X_MICROARCH.md "HBM": counters are in KiB; on gfx950
FETCH_SIZE reads half the bytes of wide streaming reads, so the read side is
doubled (an upper bound for the narrow gathers here); WRITE_SIZE is exact for
the dword-per-lane stores.  bench.py copies the per-launch traffic of its
workload into roofline.traffic.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def pixels_per_thread(kernel_name: str) -> int:
    """Pixels one work-item writes: R for k_trace_window_r<R> / k_trace_window_list<R>
    (round 1: k_trace_window_r<SLOTS, R, ...>), else 1."""
    m = re.search(r"k_trace_window_(?:r|list)<\s*(\d+)\s*>", kernel_name) or \
        re.search(r"k_trace_window_r<\s*\d+\s*,\s*(\d+)", kernel_name)
    return int(m.group(1)) if m else 1


def launch_key(kernel_name: str, grid: int) -> str:
    """Pixels per launch; the n > 64 culled-list kernel's launches get a "list:" prefix so
    that they never mix with the n <= 64 kernel's at the same frame size."""
    px = grid * pixels_per_thread(kernel_name)
    return f"list:{px}" if "k_trace_window_list" in kernel_name else str(px)


def rows(d, name):
    (path,) = glob.glob(os.path.join(d, "**", f"*{name}.csv"), recursive=True)
    return list(csv.DictReader(open(path)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--sq", nargs="*", default=[],
                    help="--pmc passes with SQ_* counters (SQ_INSTS_VALU / SQ_WAVES, stall counters)")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--kernel", default="k_trace", help="kernel-name substring (k_trace, k_glsl, k_voxel)")
    ap.add_argument("--out", default="profiles")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)

    per = collections.defaultdict(list)
    for r in rows(a.trace, "kernel_trace"):
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        per[(r["Kernel_Name"], grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    with open(os.path.join(a.out, f"{a.tag}_kernel_stats_by_grid.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "GridThreads", "Calls", "AverageNs", "MinNs", "MaxNs"])
        for (name, grid), v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, grid, len(v), round(sum(v) / len(v), 1), min(v), max(v)])

    traffic = {}
    for d, counter in ((a.fetch, "FETCH_SIZE"), (a.write, "WRITE_SIZE")):
        acc = collections.defaultdict(list)
        for r in rows(d, "counter_collection"):
            if a.kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                acc[launch_key(r["Kernel_Name"], int(r["Grid_Size"]))].append(
                    float(r["Counter_Value"]) * 1024.0)
        for grid, v in acc.items():
            traffic.setdefault(str(grid), {})[counter] = sum(v) / len(v)
    for sq_dir in a.sq:
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in rows(sq_dir, "counter_collection"):
            if a.kernel in r["Kernel_Name"]:
                acc[launch_key(r["Kernel_Name"], int(r["Grid_Size"]))][r["Counter_Name"]].append(
                    float(r["Counter_Value"]))
        for grid, cs in acc.items():
            for c, v in cs.items():
                traffic.setdefault(str(grid), {})[c] = sum(v) / len(v)
    for g, t in traffic.items():
        t["hbm_bytes_per_launch"] = 2.0 * t.get("FETCH_SIZE", 0.0) + t.get("WRITE_SIZE", 0.0)
        t["algorithmic_bytes_per_launch"] = 4.0 * int(g.split(":")[-1])
    with open(os.path.join(a.out, f"{a.tag}_traffic.json"), "w") as f:
        json.dump({"note": __doc__.split("Writes")[0].strip(), "kernel": a.kernel,
                   "per_launch_pixels": traffic}, f, indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
