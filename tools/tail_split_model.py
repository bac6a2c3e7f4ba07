"""Model: would rendering the cheapest tiles of the ordered 4K frame as two 16x8 half tiles
(R = 2) shorten the kernel's ramp-down?  Greedy list scheduling on 8192 wave slots of the
measured per-tile durations (tools/tile_timeline.py --dump, R = 4 and forced R = 2 runs of the
-DSFRT_EXP=16 build), longest first, the last N tiles replaced by their two halves.
    python tools/tail_split_model.py gpurun_out/tl
"""
import sys
import numpy as np, heapq
d4 = np.load(sys.argv[1] + "/static_r4.npz"); d2 = np.load(sys.argv[1] + "/static_r2.npz")
dur4 = (d4["t1"] - d4["t0"]) / 1e3  # us, tile grid order (270 x 120)
dur2 = ((d2["t1"] - d2["t0"]) / 1e3).reshape(270, 240)
halves = np.stack([dur2[:, 0::2].ravel(), dur2[:, 1::2].ravel()], 1)  # per 32x8 tile
print("R4 sum/8192", dur4.sum() / 8192, "R2 sum/8192", dur2.sum() / 8192)
def sim(items, slots=8192, gap=0.0):
    h = [0.0] * slots
    heapq.heapify(h)
    end = 0.0
    for d in items:
        t = heapq.heappop(h)
        f = t + gap + d
        end = max(end, f)
        heapq.heappush(h, f)
    return end
order = np.argsort(-dur4, kind="stable")
for gap in (0.0, 1.0, 2.0, 3.0):
    print("gap", gap, "all R4 LPT", round(sim(dur4[order], gap=gap), 1))
gap = 2.0
for n2 in (0, 2048, 4096, 8192, 12288, 16384):
    head = dur4[order[:len(order) - n2]]
    tail = halves[order[len(order) - n2:]].ravel() if n2 else np.array([])
    items = np.concatenate([head, tail])
    print("split last", n2, "tiles:", round(sim(items, gap=gap), 1), "work +", round((tail.sum() - dur4[order[len(order)-n2:]].sum()) / 8192, 2) if n2 else 0)
