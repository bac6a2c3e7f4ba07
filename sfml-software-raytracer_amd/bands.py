"""Row bands of one frame over the GPUs of a node, gathered to rank 0.

Pixels are independent (SphereWorld.cpp:94-110 reads nothing but the camera,
the scene and (i, j)), so a frame splits into contiguous row bands, one per
rank; each rank renders its band with GLOBAL row indices (sfrt_world_render_band),
and the bands travel to rank 0 over RCCL -- the path's one exchange step.

Two things shape the partition on MI355X:

* rank 0's own band never crosses a link, every other band does.  A 4K
  band renders at ~48 Grays/s (0.021 ns per pixel) but crosses one xGMI link
  at 4 B per pixel (~0.06 ns per pixel at ~65 GB/s one way), so with equal
  bands every rank but 0 idles on its link.  ``root_weighted_spans`` gives
  rank 0 ``factor`` times the rows of each other rank;
* the link/render ratio depends on the node (link generation, RCCL channel
  count, clocks, the scene).  ``tune_spans`` times the real pipeline for a
  few factors during warm-up and keeps the fastest (every rank takes the same
  decision from the same all-reduced times).  Factor 1 is the plain equal
  split with one RCCL gather.

``BandPipeline`` double-buffers bands and frames so that the transfer of
frame k overlaps the render of frame k + 1.  With ``packed`` (bands of a world whose
textures are alpha-binary, sfrt.World.alpha_binary) every band but rank 0's crosses
the link in libsfrt's packed format (3.125 B per pixel instead of 4; include/sfrt.h
"Band transfer packing") and rank 0 unpacks it into the frame on a stream of its own.
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.distributed as dist

ALIGN = 8  # rows per kernel tile: bands that start on a tile row waste no lanes

# Root factors tried by tune_spans (1.0 = equal bands).
DEFAULT_FACTORS = (1.0, 1.5, 2.0, 2.5, 3.0, 4.0)


def band_of(rank: int, world: int, height: int) -> tuple[int, int]:
    """Equal split: rank r renders rows [r*H/n, (r+1)*H/n)."""
    r0 = rank * height // world
    return r0, (rank + 1) * height // world - r0


def equal_spans(height: int, world: int) -> list[tuple[int, int]]:
    return [band_of(r, world, height) for r in range(world)]


def root_weighted_spans(height: int, world: int, factor: float,
                        align: int = ALIGN) -> list[tuple[int, int]]:
    """(row0, rows) per rank: rank 0 renders about `factor` times the rows of every
    other rank (their bands are equal and `align`-row multiples).  factor == 1, or a
    frame too short to weight, gives the equal split."""
    if world == 1:
        return [(0, height)]
    if factor == 1.0:
        return equal_spans(height, world)
    other = int(height / (world - 1 + factor))
    other -= other % align
    if other <= 0 or other * (world - 1) >= height:
        return equal_spans(height, world)
    first = height - (world - 1) * other
    return [(0, first)] + [(first + (r - 1) * other, other) for r in range(1, world)]


def cost_weighted_spans(row_cost, world: int, factor: float = 1.0,
                        align: int = ALIGN) -> list[tuple[int, int]]:
    """(row0, rows) per rank from per-row work (SURVEY 8e "Balance": cost-weighted band
    edges): rank 0 gets `factor` shares of the frame's total cost, every other rank one
    share.  Edges sit on `align`-row boundaries (or the last row); each is the boundary
    whose cost prefix is closest to its target, never before the previous edge.  The
    C ABI's sfrt_multi_cost_bands computes the same partition (same double sums in row
    order, same ties).  Costs that are negative, non-finite or all zero fall back to
    root_weighted_spans."""
    height = len(row_cost)
    at, pre = [], []
    total, ok = 0.0, True
    for j in range(height + 1):
        if j % align == 0 or j == height:
            at.append(j)
            pre.append(total)
        if j < height:
            c = float(row_cost[j])
            if not (c >= 0.0) or c == float("inf"):
                ok = False
            total += c
    if world == 1 or not ok or not total > 0.0:
        return root_weighted_spans(height, world, factor, align)
    factor = float(np.float32(factor))  # the C ABI takes a binary32 factor
    denom = (world - 1) + factor
    edges, i = [0], 0
    for r in range(1, world):
        target = total * (factor + (r - 1)) / denom
        k = i
        while k + 1 < len(at) and pre[k] < target:
            k += 1
        if k > i and pre[k] - target > target - pre[k - 1]:
            k -= 1
        i = k
        edges.append(at[i])
    edges.append(height)
    return [(edges[r], edges[r + 1] - edges[r]) for r in range(world)]


def check_spans(spans, height: int) -> None:
    """Bands must tile [0, height) in rank order (rank 0 first)."""
    row = 0
    for r0, n in spans:
        if r0 != row or n < 0:
            raise ValueError(f"bands {spans} do not tile {height} rows")
        row += n
    if row != height:
        raise ValueError(f"bands {spans} do not tile {height} rows")


class _HostStagedWork:
    """A point-to-point transfer staged through host memory (see stage_p2p_through_host).
    wait() blocks on the host transfer, then a receive copies into its device tensor on the
    caller's current stream -- the stream-side order NCCL's Work.wait() gives: work queued on
    that stream afterwards sees the bytes."""

    def __init__(self, work, host, dst=None):
        self.work, self.host, self.dst = work, host, dst

    def wait(self):
        if self.work is None:
            return
        self.work.wait()
        self.work = None
        if self.dst is not None:
            self.dst.copy_(self.host)
            self.dst = None


def _host_staged_batch_isend_irecv(ops):
    works = []
    for op in ops:
        if op.op is dist.isend:
            host = op.tensor.to("cpu")  # waits for the current stream's work (the render)
            works.append(_HostStagedWork(dist.isend(host, op.peer, tag=op.tag), host))
        else:
            host = torch.empty(op.tensor.shape, dtype=op.tensor.dtype)
            works.append(_HostStagedWork(dist.irecv(host, op.peer, tag=op.tag), host, op.tensor))
    return works


_P2P = {"staged": False}


def stage_p2p_through_host(on: bool = True) -> None:
    """TEST ONLY (bench.py --rehearse): BandPipeline's point-to-point transfers of device
    bands go through host copies, for a gloo process group whose ranks share one GPU (RCCL
    refuses two ranks on one device, and gloo's send/recv take host buffers).  The gather of
    equal bands and the all-reduces keep their device tensors (gloo's HIP paths)."""
    _P2P["staged"] = bool(on)


def batch_isend_irecv(ops):
    """dist.batch_isend_irecv, or its host-staged stand-in after stage_p2p_through_host()."""
    if _P2P["staged"]:
        return _host_staged_batch_isend_irecv(ops)
    return dist.batch_isend_irecv(ops)


class BandPipeline:
    """Row-band frames with the transfer to rank 0 overlapped with rendering.

    Every rank owns `depth` band buffers; rank 0 also owns `depth` whole
    frames.  Frame k renders into band k % depth and its transfer into frame
    k % depth is queued asynchronously (RCCL runs it on its own stream after
    the render that produced the band), so frame k+1 renders while frame k
    crosses xGMI.  Reusing a buffer first waits (stream-side on RCCL) for the
    transfer that last read it.  Equal bands use one gather collective;
    unequal bands one batch of point-to-point transfers straight into the
    frame's row slices.  With one rank the band IS the frame and nothing is
    exchanged."""

    def __init__(self, rank: int, world_size: int, height: int, pitch: int, device,
                 depth: int = 2, spans=None, local_depth: int = 1, packed: bool = False):
        self.rank, self.world_size, self.height = rank, world_size, height
        self.spans = list(spans) if spans is not None else equal_spans(height, world_size)
        check_spans(self.spans, height)
        if len(self.spans) != world_size:
            raise ValueError("one band per rank")
        self.equal = len({n for _, n in self.spans}) == 1
        # one rank: `local_depth` whole frames (several frames in flight on as many streams)
        self.depth = depth if world_size > 1 else local_depth
        self.row0, self.rows = self.spans[rank]
        self.frames, self.views = [], []
        if world_size == 1:
            self.frames = [torch.empty(height, pitch, dtype=torch.uint8, device=device)
                           for _ in range(self.depth)]
            self.bands = self.frames
        else:
            if rank == 0:
                for _ in range(self.depth):
                    fr = torch.empty(height, pitch, dtype=torch.uint8, device=device)
                    self.frames.append(fr)
                    self.views.append([fr[r0:r0 + n] for r0, n in self.spans])
            if rank == 0 and not self.equal:
                # rank 0 renders straight into its rows of the frame (no copy)
                self.bands = [v[0] for v in self.views]
            else:
                self.bands = [torch.empty(self.rows, pitch, dtype=torch.uint8, device=device)
                              for _ in range(self.depth)]
        self.pending = [[] for _ in range(self.depth)]
        self.packed = bool(packed) and world_size > 1
        if self.packed:
            self._init_packed(pitch, device)

    def _init_packed(self, pitch: int, device) -> None:
        """Packed transfers: every non-root rank packs its band (sfrt_band_pack) into a
        per-slot buffer and sends it point-to-point; rank 0 renders straight into its rows
        of the frame, receives each band into a per-slot staging buffer and unpacks it into
        the frame on `unpack_stream` (ordered after the receives, not after rank 0's
        render of the next frame).  Needs a HIP device and pitch = width * 4."""
        import sfrt
        self._sfrt = sfrt
        if pitch % 4:
            raise ValueError("packed bands need whole RGBA8 rows")
        self.pixels = [n * (pitch // 4) for _, n in self.spans]
        nbytes = [sfrt.band_packed_bytes(p) for p in self.pixels]
        if self.rank == 0:
            self.bands = [v[0] for v in self.views]
            self.stage = [[torch.empty(nbytes[r], dtype=torch.uint8, device=device)
                           if r > 0 and self.pixels[r] else None for r in range(self.world_size)]
                          for _ in range(self.depth)]
            self.unpack_stream = torch.cuda.Stream(device=device)
            self.unpacked = [torch.cuda.Event() for _ in range(self.depth)]
            self.unpack_pending = [False] * self.depth
        else:
            self.packbuf = [torch.empty(max(nbytes[self.rank], 8), dtype=torch.uint8, device=device)
                            for _ in range(self.depth)]

    def acquire(self, k: int):
        """The band buffer for frame k, once the transfer that last read it is done."""
        b = k % self.depth
        for work in self.pending[b]:
            work.wait()
        self.pending[b] = []
        if self.packed and self.rank == 0 and self.unpack_pending[b]:
            # frame slot b and its staging buffers: free once the last unpacks are done
            torch.cuda.current_stream().wait_event(self.unpacked[b])
            self.unpack_pending[b] = False
        return self.bands[b]

    def submit(self, k: int) -> None:
        """Queue frame k's transfer (after everything already queued on the current stream)."""
        if self.world_size == 1:
            return
        b = k % self.depth
        band = self.bands[b]
        views = self.views[b] if self.rank == 0 else None
        if self.packed:
            return self._submit_packed(b, band, views)
        if self.equal:
            self.pending[b] = [dist.gather(band, views, dst=0, async_op=True)]
        elif self.rank == 0:
            ops = [dist.P2POp(dist.irecv, views[r], r) for r in range(1, self.world_size)
                   if self.spans[r][1] > 0]
            self.pending[b] = batch_isend_irecv(ops) if ops else []
        elif self.rows > 0:
            self.pending[b] = batch_isend_irecv([dist.P2POp(dist.isend, band, 0)])

    def _submit_packed(self, b: int, band, views) -> None:
        sf = self._sfrt
        if self.rank > 0:
            if self.rows > 0:
                sf.band_pack(band.data_ptr(), self.pixels[self.rank], self.packbuf[b].data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
                self.pending[b] = batch_isend_irecv(
                    [dist.P2POp(dist.isend, self.packbuf[b], 0)])
            return
        srcs = [r for r in range(1, self.world_size) if self.pixels[r]]
        if not srcs:
            return
        works = batch_isend_irecv([dist.P2POp(dist.irecv, self.stage[b][r], r) for r in srcs])
        with torch.cuda.stream(self.unpack_stream):
            for work in works:
                work.wait()  # the unpack stream waits for the receives
            for r in srcs:
                sf.band_unpack(self.stage[b][r].data_ptr(), self.pixels[r], views[r].data_ptr(),
                               self.unpack_stream.cuda_stream)
            self.unpacked[b].record(self.unpack_stream)
        self.unpack_pending[b] = True

    def drain(self) -> None:
        for b in range(self.depth):
            for work in self.pending[b]:
                work.wait()
            self.pending[b] = []
            if self.packed and self.rank == 0 and self.unpack_pending[b]:
                torch.cuda.current_stream().wait_event(self.unpacked[b])
                self.unpack_pending[b] = False

    def frame(self, k: int):
        """Rank 0's assembled frame k (valid after drain() or the next acquire of its slot)."""
        return self.frames[k % self.depth] if self.frames else None


def max_over_ranks(x: float, device="cpu") -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def run_frames(pipe: BandPipeline, render, frames: int, sync=lambda: None) -> float:
    """Render + transfer `frames` frames through `pipe`; wall seconds between two
    barriers (this rank's view).  render(band_tensor, row0, rows) queues one band."""
    if dist.is_initialized():
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(frames):
        band = pipe.acquire(k)
        render(band, pipe.row0, pipe.rows)
        pipe.submit(k)
    pipe.drain()
    sync()
    if dist.is_initialized():
        dist.barrier()
    return time.perf_counter() - t0


def tune_spans(render, rank: int, world_size: int, height: int, pitch: int, device,
               factors=DEFAULT_FACTORS, frames: int = 8, warm: int = 2,
               sync=lambda: None, reduce_device="cpu", row_cost=None, packed=(False,)):
    """Pick the partition whose pipelined frames run fastest on this node.

    Candidates: root_weighted_spans for every factor and, given the frame's per-row work
    `row_cost` (sfrt_world_row_costs, the same on every rank), cost_weighted_spans for
    every factor, each with every transfer format in `packed` (False: RGBA8 bands, True:
    packed bands).  Every candidate runs `warm` + `frames` real frames through a
    BandPipeline; the time that counts is the max over ranks (all-reduced, so every
    rank sees the same numbers and takes the same decision).  Returns (spans, pick,
    {label: ms per frame}) with pick = {"root_factor": f, "weights": "rows" | "cost",
    "packed": bool} and labels "f" / "cost:f", prefixed "packed:" for packed bands."""
    if world_size == 1:
        return [(0, height)], {"root_factor": 1.0, "weights": "rows", "packed": False}, {}
    parts = [(f"{f}", {"root_factor": f, "weights": "rows"}, root_weighted_spans(height, world_size, f))
             for f in factors]
    if row_cost is not None:
        parts += [(f"cost:{f}", {"root_factor": f, "weights": "cost"},
                   cost_weighted_spans(row_cost, world_size, f)) for f in factors]
    cands = [(("packed:" if pk else "") + label, dict(pick, packed=bool(pk)), spans)
             for pk in packed for label, pick, spans in parts]
    table, best = {}, None
    tried = set()
    for label, pick, spans in cands:
        key = (tuple(spans), pick["packed"])
        if key in tried:
            continue
        tried.add(key)
        pipe = BandPipeline(rank, world_size, height, pitch, device, spans=spans,
                            packed=pick["packed"])
        run_frames(pipe, render, warm, sync)
        wall = max_over_ranks(run_frames(pipe, render, frames, sync), reduce_device)
        del pipe
        ms = wall / frames * 1e3
        table[label] = round(ms, 4)
        if best is None or ms < best[0]:
            best = (ms, pick, spans)
    return best[2], best[1], table
