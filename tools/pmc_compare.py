"""Per-launch PMC counters of the 4K headline frame for several libraries (A/B builds), from
rocprofv3 --pmc runs of tools/frame_loop.py (tools/gpu/ab_pmc.sh):
    python tools/pmc_compare.py gpurun_out/<tag>/pmc_0 gpurun_out/<tag>/pmc_1 ...
Prints, per directory, the mean of each counter over the k_trace launches of the largest grid,
and lane-instructions per ray for the SQ_INSTS_* counters."""
import collections
import csv
import glob
import os
import sys

RAYS = 3840 * 2160


def main():
    for d in sys.argv[1:]:
        (path,) = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(path)):
            if "k_trace" in r["Kernel_Name"]:
                acc[int(r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        grid = max(acc)
        out = {c: sum(v) / len(v) for c, v in acc[grid].items()}
        per_ray = {c: round(v * 64 / RAYS, 1) for c, v in out.items() if c.startswith("SQ_INSTS")}
        print(d, "grid", grid, {c: round(v) for c, v in out.items()}, "per ray", per_ray)


if __name__ == "__main__":
    main()
