"""Benchmark: Mrays/s of the sphere-cave frame fill on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step is one full frame: every rank fills its row band of a 3840 x (2160*N)
RGBA8 frame in HBM through libsfrt.so (64-sphere cave, BASELINE config 3),
then for N > 1 the bands travel to rank 0 over RCCL (one gather for equal
bands, grouped point-to-point transfers otherwise), the transfer of frame k
overlapping the render of frame k+1 (double-buffered bands/frames).  The
band heights are tuned during the untimed warm-up (bands.tune_spans: rank 0,
whose band never crosses a link, may take more rows).  Per-GPU work is fixed
on average as N grows ("weak" scaling); rays use the global row index, so the
gathered frame is byte-identical to a single-GPU render of the same frame.
value = all rays of the K frames / (max over ranks of the timed wall time).
One frame at a time on one stream; at N = 1 the `*_2_in_flight` lines under "also" render
frames alternately on two HIP streams into two buffers, frame k+1 starting while frame k's
last tiles drain (the throughput of a double-buffered display or offline loop).
Before the W warm-up frames, --settle seconds of untimed frames let the chip
reach its steady clock (it ramps over the first few hundred frames).

Also reported under "also", each line with its own settle (--also-settle), warm-up
(--also-warmup) and timed frames (--also-steps, independent of --steps so that a short
headline run still times every line over enough frames): the 7680x4320 frame row-tiled
over the N ranks (BASELINE config 4; N = 1, 2, 4, 8) and the 16384x16384 frame at N = 1
and 8 (config 5), strong scaling with the overlapped gather; at N = 1 the 1920x1080
10-sphere frame (config 2) and variants of the headline; at N > 1 "c_abi_multi", the
single-process C-ABI path (sfrt_multi_render over devices 0..N-1, RCCL) timed by rank 0
while the other ranks wait on a host barrier.  And the kernel's HBM roofline from HIP
events on the launch stream (around every 8th timed frame: a pair per frame
would put marker packets between all frames of the wall-clock measurement),
and the CPU baseline: the oracle (CPU restatement, oracle/) rendering one
whole 4K frame on the host cores, compared byte for byte with the GPU frame.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sfml-software-raytracer_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bands as bands_mod  # noqa: E402
import scenes  # noqa: E402
import sfrt  # noqa: E402
from bands import (BandPipeline, band_of, equal_spans,  # noqa: E402,F401
                   max_over_ranks as _max_over_ranks, tune_spans)

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# VALU issue peak: 256 CUs x 4 SIMD32 x one wave64 instruction per 2 clocks at
# 2.4 GHz = 1.229e12 wave-instructions/s (x 64 lanes = the 157.3 TFLOPS FP32
# figure counted as FMA = 2).
VALU_PEAK_WAVE_INSTS = 256 * 4 * 0.5 * 2.4e9
# What a plain stream of independent v_add_f32 reaches on this chip at 8 waves/SIMD: 0.438
# wave64 instructions per SIMD-clock (tools/native/pk_rate_check.hip), at the 2.33 GHz shader
# clock measured across the headline kernel's tiles (s_memtime over s_memrealtime, the
# -DSFRT_EXP=1040 build): profiles/r3y_valu_rate_check.txt, r3y_timeline/tile_timeline_4k_clock.txt.
VALU_STREAM_CEILING = 256 * 4 * 0.438 * 2.33e9
BYTES_PER_RAY = 4            # RGBA8 store; texture + sphere table are cache-resident
WIDTH, ROWS_PER_GPU = 3840, 2160


def measured_traffic(pixels: int, kernel: str = "k_trace"):
    """Per-launch HBM bytes and VALU instruction counts of this workload from the
    newest profiles/*_traffic.json of `kernel` (tools/rocprof_summary.py over separate
    rocprofv3 --pmc passes of this same workload), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        doc = json.load(open(path))
        if doc.get("kernel", "k_trace") != kernel:
            continue
        table = doc.get("per_launch_pixels", doc.get("per_grid_threads", {}))
        # the sphere kernel's steady-state launch has the tile-order sorter workgroup (+64 x R
        # pixels, R = 4, 3, 2 or 1 pixels per lane)
        # (the GLSL renderer's ordered launch likewise, since round 4: one sorter workgroup of 64)
        for extra in ((256, 192, 128, 64, 0) if kernel == "k_trace" else
                      (64, 0) if kernel == "k_glsl" else (0,)):
            ent = table.get(str(pixels + extra))
            if ent:
                return ent, os.path.relpath(path, ROOT)
    return None, None


EVENT_EVERY = 8  # frames per HIP-event-timed frame in time_frames

GOLDEN_PATH = os.path.join(ROOT, "tests", "golden", "golden.json")
_GOLDEN = {}


def golden_sha256(section: str, key):
    """SHA-256 of a committed golden frame (tests/golden/golden.json, generated by
    tests/golden/make_golden.py), or None.  Data, not the oracle: bench.py never runs it
    outside cpu_baseline."""
    if key is None:
        return None
    if not _GOLDEN:
        _GOLDEN["doc"] = json.load(open(GOLDEN_PATH)) if os.path.exists(GOLDEN_PATH) else {}
    return _GOLDEN["doc"].get(section, {}).get(key, {}).get("sha256")


def verify_frame(frame, section: str, key) -> dict:
    """A timed line's last frame against its golden frame: SHA-256 (hashlib) of the device
    frame's bytes copied to the host.  {"golden": "section/key", "bit_identical": bool}, or
    the digest alone where no golden frame exists for the workload."""
    host = np.ascontiguousarray(frame.cpu().numpy()).reshape(-1)
    digest = hashlib.sha256(host.data).hexdigest()
    want = golden_sha256(section, key)
    if want is None:
        return {"golden": None, "sha256": digest}
    return {"golden": f"{section}/{key}", "bit_identical": digest == want}


def event_pair_ms(stream, n: int = 64) -> float:
    """Median elapsed time of an empty HIP-event pair on `stream`: the marker overhead that
    each sampled (start, end) pair adds to the kernel it brackets (subtracted from kernel_ms,
    so that it agrees with the rocprofv3 kernel trace and never exceeds the wall time per
    frame)."""
    pairs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
             for _ in range(n)]
    for a, b in pairs:
        a.record(stream)
        b.record(stream)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in pairs]))


# Two frames in flight (the `*_2_in_flight` lines under also, N = 1): frames alternate
# between the launch stream and a second stream, each into its own buffer, so frame k+1
# starts while frame k's last tiles drain -- each stream has its own tile-order chain in
# libsfrt (sfrt_sched.h TileChains).  The headline stays one frame at a time: its kernel_ms is then each launch's
# own time, as the rocprof trace and the roofline use it (with two in flight every launch
# shares the chip with the next and its duration says nothing about throughput).
SECOND_STREAM = []


def frame_streams(stream, in_flight: int):
    if in_flight == 1:
        return [stream]
    if not SECOND_STREAM:
        SECOND_STREAM.append(torch.cuda.Stream())
    return [stream, SECOND_STREAM[0]]


def time_frames(world, pipe: BandPipeline, pitch, steps, warmup, stream, per_frame=None,
                in_flight: int = 1):
    """Warmup, then `steps` timed frames through the pipeline, frame k on
    streams[k % in_flight] (pipe.depth >= in_flight buffers in turn).  Returns (wall
    seconds, kernel ms per launch from HIP events around every EVENT_EVERY-th render on its
    launch stream, minus the empty event pair's own elapsed time).
    per_frame(k), if given, runs before frame k is queued (a moving camera)."""
    streams = frame_streams(stream, in_flight)
    if pipe.depth < len(streams):
        raise ValueError("one frame buffer per stream in flight")
    for k in range(warmup):
        if per_frame:
            per_frame(k)
        world.render_band(pipe.acquire(k).data_ptr(), pitch, pipe.row0, pipe.rows,
                          streams[k % len(streams)].cuda_stream)
        pipe.submit(k)
    pipe.drain()
    torch.cuda.synchronize()
    for s in streams:
        world.check(s.cuda_stream)
    # HIP events around every EVENT_EVERY-th frame only: an event is a marker
    # packet in the stream, and one pair per frame would add its own gap to
    # every frame of the wall-clock measurement.
    sampled = [k for k in range(steps) if k % EVENT_EVERY == 0]
    starts = {k: torch.cuda.Event(enable_timing=True) for k in sampled}
    ends = {k: torch.cuda.Event(enable_timing=True) for k in sampled}
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        if per_frame:
            per_frame(warmup + k)
        band = pipe.acquire(k)
        sk = streams[k % len(streams)]  # frame k's buffer is pipe.acquire(k): k % depth
        if k in starts:
            starts[k].record(sk)
        world.render_band(band.data_ptr(), pitch, pipe.row0, pipe.rows, sk.cuda_stream)
        if k in ends:
            ends[k].record(sk)
        pipe.submit(k)
    pipe.drain()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    wall = time.perf_counter() - t0
    for s in streams:
        world.check(s.cuda_stream)
    raw = sum(starts[k].elapsed_time(ends[k]) for k in sampled) / len(sampled)
    kernel_ms = max(0.0, raw - event_pair_ms(stream))
    return wall, kernel_ms


def max_over_ranks(x: float) -> float:
    return _max_over_ranks(x, "cuda")


def settle(world, pitch, row0, rows, stream, seconds: float) -> None:
    """Untimed frames until `seconds` have passed: the chip ramps its clock over the
    first few hundred frames after idling, and the timed frames should
    see the steady state a continuously rendering display or offline job runs at.  Run
    before every timed line (the host-side setup between lines lets the clock drop)."""
    if seconds <= 0 or rows <= 0:
        return
    buf = torch.empty(rows, pitch, dtype=torch.uint8, device="cuda")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(16):
            world.render_band(buf.data_ptr(), pitch, row0, rows, stream.cuda_stream)
        torch.cuda.synchronize()
    del buf


def frame_row_costs(world, rank, world_size, height, pitch, stream, device="cuda"):
    """The frame's per-row work (sfrt_world_row_costs) on every rank: each rank renders its
    equal band once in the adaptive tile order, and the bands' costs are summed over ranks
    into one full-height vector (SURVEY 8e "Balance": cost-weighted band edges)."""
    r0, n = band_of(rank, world_size, height)
    # the last element counts ranks whose costs failed: every rank still joins the
    # all-reduce, and the tuner then falls back to row-weighted bands on every rank
    full = torch.zeros(height + 1, dtype=torch.float64, device=device)
    try:
        buf = torch.empty(max(n, 1), pitch, dtype=torch.uint8, device=device)
        world.render_band(buf.data_ptr(), pitch, r0, n, stream.cuda_stream)
        c0, cost = world.row_costs()
        if (c0, cost.size) != (r0, n):
            raise RuntimeError(f"row costs cover rows {c0}+{cost.size}, the band is {r0}+{n}")
        full[c0:c0 + cost.size] = torch.from_numpy(cost.astype(np.float64)).to(device)
        del buf
    except Exception as e:  # noqa: BLE001 -- reported, never fatal to the run
        print(f"rank {rank}: row costs unavailable ({e}); row-weighted bands only",
              file=sys.stderr, flush=True)
        full[height] = 1.0
    dist.all_reduce(full)
    if float(full[height].item()) > 0:
        return None
    return full[:height].cpu().numpy().astype(np.float32)


def tuned_pipeline(world, rank, world_size, height, pitch, stream, band_mode="tuned"):
    """Row bands for this node: tune_spans times root-weighted and cost-weighted partitions,
    with RGBA8 and packed band transfers, on real frames (untimed warm-up) and keeps the
    fastest; N = 1 is one whole band.  band_mode "equal": the plain equal split (one gather
    per frame), untuned."""
    if band_mode == "equal" or world_size == 1:
        spans = equal_spans(height, world_size)
        pipe = BandPipeline(rank, world_size, height, pitch, "cuda", spans=spans)
        return pipe, {"rows_per_rank": [n for _, n in spans], "root_factor": 1.0,
                      "weights": "rows", "transfer": "rgba8",
                      **({"tuning": "off (--bands equal)"} if world_size > 1 else {})}

    def render(band, row0, rows):
        world.render_band(band.data_ptr(), pitch, row0, rows, stream.cuda_stream)
    row_cost = frame_row_costs(world, rank, world_size, height, pitch, stream) \
        if world_size > 1 else None
    # packed band transfers (3.125 B per pixel over the links) are a candidate when every
    # texel's alpha is 0 or 255 (Floor.png's are; the same textures on every rank)
    formats = (False, True) if world_size > 1 and world.alpha_binary() else (False,)
    spans, pick, table = tune_spans(render, rank, world_size, height, pitch, "cuda",
                                    sync=torch.cuda.synchronize, reduce_device="cuda",
                                    row_cost=row_cost, packed=formats)
    pipe = BandPipeline(rank, world_size, height, pitch, "cuda", spans=spans,
                        packed=pick["packed"])
    info = {"rows_per_rank": [n for _, n in spans], "root_factor": pick["root_factor"],
            "weights": pick["weights"], "transfer": "packed" if pick["packed"] else "rgba8"}
    if table:
        info["tuning_ms_per_frame"] = table
    return pipe, info


def hbm_frac(rays: int, kernel_ms: float) -> float:
    """The HBM roofline fraction of one launch: 4 algorithmic bytes per ray / kernel time."""
    return round(BYTES_PER_RAY * rays / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6) if kernel_ms > 0 else 0.0


def host_delivery(local_rank, floor, scene, width, height, frames, want):
    """the end-to-end rate with the frame copied into a host `sf::Uint8*` buffer
    (PCIe included), reported beside the HBM-resident `value`, never as it.  "pipelined":
    sfrt_world_submit_frame / wait_frame into two pinned frames (render k+1 overlaps the
    copy of k); "sync": sfrt_world_update_image into a pageable buffer, one frame at a time.
    Static camera, the headline scene; `want` is the device frame the host frames must equal."""
    w = sfrt.World(local_rank)
    w.load_texture(*floor)
    w.set_scene(scene, width, height)
    res = {}
    bufs = [sfrt.HostFrame(width * height * 4) for _ in range(2)]
    for n in (8, frames):  # warm-up, then timed
        pending = []
        t0 = time.perf_counter()
        for k in range(n):
            pending.append(w.submit_frame(bufs[k % 2]))
            if len(pending) == 2:
                w.wait_frame(pending.pop(0))
        for t in pending:
            w.wait_frame(t)
        dt = time.perf_counter() - t0
    same = all(np.array_equal(b.array, want) for b in bufs)
    res["pipelined_pinned"] = {"Mrays_per_s": round(width * height * frames / dt / 1e6, 2),
                               "fps": round(frames / dt, 2),
                               "GB_per_s_to_host": round(width * height * 4 * frames / dt / 1e9, 2),
                               "bit_identical_to_device_frame": same}
    for b in bufs:
        b.free()
    out = np.zeros(width * height * 4, np.uint8)
    for n in (4, max(4, frames // 4)):
        t0 = time.perf_counter()
        for _ in range(n):
            w.update_image(out)
        dt = time.perf_counter() - t0
    res["sync_pageable"] = {"Mrays_per_s": round(width * height * n / dt / 1e6, 2),
                            "fps": round(n / dt, 2),
                            "GB_per_s_to_host": round(width * height * 4 * n / dt / 1e9, 2),
                            "bit_identical_to_device_frame": bool(np.array_equal(out, want))}
    w.close()
    return res


def measure_frame(world, scene, width, height, rank, world_size, steps, warmup, stream,
                  settle_s=0.0, band_mode="tuned"):
    """One extra BASELINE frame size, row-tiled over all ranks (+ overlapped transfer); rank 0
    checks the last gathered frame against the golden frame of the workload."""
    world.set_scene(scene, width, height)
    pipe, bands = tuned_pipeline(world, rank, world_size, height, width * 4, stream, band_mode)
    settle(world, width * 4, pipe.row0, pipe.rows, stream, settle_s)
    wall, kms = time_frames(world, pipe, width * 4, steps, warmup, stream)
    wall = max_over_ranks(wall)
    rays0 = width * pipe.rows
    check = verify_frame(pipe.frame(steps - 1), "frames",
                         scenes.golden_key(width, height, scene.name)) if rank == 0 else None
    del pipe
    return {"n_gpus": world_size, "Mrays_per_s": round(width * height * steps / wall / 1e6, 2),
            "fps": round(steps / wall, 2), "ms_per_frame": round(wall / steps * 1e3, 4),
            "kernel_ms_rank0_band": round(kms, 4),
            # a small band (1080p over 8 ranks: 135 rows) can time at or below the event pair's
            # own gap: hbm_frac() reports 0 there instead of dividing by it
            "hbm_frac_rank0_kernel": hbm_frac(rays0, kms),
            "bands": bands, **(check or {})}


# BASELINE.json configs 4 and 5 (the 8K and 16384^2 frames also on one GPU: the
# strong-scaling anchors of the N > 1 lines): frame size by GPU count.
# The north star reports Mrays/s at 1080p / 4K / 8K at 1, 2, 4 and 8 GPUs: at N > 1 the
# 1080p (full scene) and 4K frames are split over the ranks too (at N = 1 they are the
# headline and the 1920x1080_default10 line).
EXTRA_FRAMES = {1: [(7680, 4320, "lcg64"), (16384, 16384, "lcg64"), (16384, 16384, "default10")],
                2: [(1920, 1080, "default10"), (3840, 2160, "lcg64"), (7680, 4320, "lcg64")],
                4: [(1920, 1080, "default10"), (3840, 2160, "lcg64"), (7680, 4320, "lcg64")],
                8: [(1920, 1080, "default10"), (3840, 2160, "lcg64"), (7680, 4320, "lcg64"),
                    (16384, 16384, "lcg64")]}


def host_cpu_info() -> dict:
    """Host CPUs as this process sees them: nproc (the affinity mask), os.cpu_count() (the
    machine) and the cgroup CPU quota when one is set (the GPU box's share)."""
    info = {"nproc": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count()}
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            info["cgroup_cpu_quota"] = round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        pass
    return info


def cpu_baseline(scene, width, height, floor, gpu_frame):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU restatement, timed as the baseline
    cpus = host_cpu_info()
    # T = nproc threads -- capped at the cgroup CPU quota where one is set (the GPU
    # box: nproc 256, quota 16), since more threads than the quota only time-slice
    threads = cpus["nproc"]
    if "cgroup_cpu_quota" in cpus:
        threads = max(1, min(threads, int(cpus["cgroup_cpu_quota"])))
    o = oracle.Oracle.from_scene(scene, width, height, *floor)
    reps = 3  # ~1.5 s on 16 threads: ~25 s of CPU work (the contract's 10-30 s sample)
    t0 = time.perf_counter()
    for _ in range(reps):
        frame = o.render(threads)
    dt = (time.perf_counter() - t0) / reps
    same = bool(np.array_equal(frame, gpu_frame))
    # One thread on every 16th row (the reference's UpdateImage(img, 0, 16, 0, 1)).
    sub = np.zeros(width * height * 4, dtype=np.uint8)
    t1 = time.perf_counter()
    o.update_image(sub, 0, 16, 0, 1)
    dt1 = time.perf_counter() - t1
    rows1 = (height + 15) // 16
    same1 = bool(np.array_equal(sub.reshape(height, -1)[::16], gpu_frame.reshape(height, -1)[::16]))
    # T = nproc literally, beside the quota-capped figure: one frame
    at_nproc = None
    if threads != cpus["nproc"]:
        t2 = time.perf_counter()
        o.render(cpus["nproc"])
        dt2 = time.perf_counter() - t2
        at_nproc = {"value": round(width * height / dt2 / 1e6, 3), "unit": "Mrays/s",
                    "threads": cpus["nproc"], "sample": f"one full frame, {dt2:.2f} s"}
    return {"value": round(width * height / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads,
            "kind": "port",
            "sample": f"{reps} full {width}x{height} frames of the same scene (mean), "
                      f"oracle/sphereworld_oracle.c (-O2, no FMA), {threads} threads with the "
                      f"reference's row interleave (Source.cpp:21), {dt:.2f} s per frame",
            "host_cpus": cpus,
            "frame_bit_identical_to_gpu": same,
            "single_thread": {"value": round(width * rows1 / dt1 / 1e6, 3), "unit": "Mrays/s",
                              "cores": 1, "sample": f"rows j % 16 == 0 ({rows1} rows), {dt1:.2f} s",
                              "bit_identical_to_gpu": same1},
            "at_nproc_threads": at_nproc}


def c_abi_multi(devices, floor, frames, steps, warmup, settle_s):
    """The single-process caller's multi-GPU path (Source.cpp:47-52 fills ONE sf::Image):
    sfrt_multi_render over `devices` -- one world per device, row bands rendered in parallel,
    gathered on devices[0] by RCCL (distinct devices) or peer copies (a device listed twice),
    packed to 3.125 B per pixel for the alpha-binary textures.  Rank 0 times it after the
    torch.distributed lines while the other ranks wait on a host barrier.  For every frame
    size: equal, root-weighted and cost-weighted bands x packed / RGBA8 transfers, each after
    its own settle and warm-up; the last frame of every candidate must equal a one-GPU frame."""
    n = len(devices)
    m = sfrt.Multi(devices, sfrt.SFRT_MULTI_AUTO)
    m.load_texture(*floor)
    dev0 = torch.device("cuda", devices[0])
    stream = torch.cuda.Stream(device=dev0)
    out = {"devices": list(devices),
           "transport": {sfrt.SFRT_MULTI_RCCL: "rccl", sfrt.SFRT_MULTI_PEER: "peer"}[m.transport]}
    if m.transport == sfrt.SFRT_MULTI_RCCL:
        # real RCCL only: a test transport is selected by an explicit call this script never makes
        out["rccl_library"] = sfrt.multi_transport_library()
        if out["rccl_library"].startswith("test:"):
            raise RuntimeError(f"c_abi_multi: test transport {out['rccl_library']} in use")
    for fw, fh, sname in frames:
        scene = scenes.lcg64() if sname == "lcg64" else scenes.SCENES[sname]()
        m.set_scene(scene, fw, fh)
        with sfrt.World(devices[0]) as ref:
            ref.load_texture(*floor)
            ref.set_scene(scene, fw, fh)
            want = torch.empty(fh, fw * 4, dtype=torch.uint8, device=dev0)
            ref.render_band(want.data_ptr(), fw * 4, 0, fh, stream.cuda_stream)
            ref.check(stream.cuda_stream)
        # every candidate's frame must equal `want`, and `want` the golden frame
        want_check = verify_frame(want, "frames", scenes.golden_key(fw, fh, sname))
        bufs = [torch.empty(fh, fw * 4, dtype=torch.uint8, device=dev0) for _ in range(2)]
        table = {}
        best = None
        for weights, f in (("rows", 1.0), ("rows", 2.0), ("rows", 3.0), ("cost", 1.0), ("cost", 2.0)):
            for fmt in (sfrt.SFRT_TRANSFER_AUTO, sfrt.SFRT_TRANSFER_RGBA):
                m.set_transfer(fmt)
                m.set_bands(None)
                if weights == "rows" and f != 1.0:
                    m.set_bands([r for _, r in sfrt.multi_bands(fh, n, f)])
                elif weights == "cost":
                    m.render(bufs[0].data_ptr(), fw * 4, stream.cuda_stream)  # records the costs
                    m.check()
                    m.balance(f)

                def frame(k):
                    m.render(bufs[k % 2].data_ptr(), fw * 4, stream.cuda_stream)
                t0 = time.perf_counter()
                k = 0
                while time.perf_counter() - t0 < settle_s or k < warmup:
                    frame(k)
                    k += 1
                    if k % 8 == 0:
                        m.check()
                m.check()
                torch.cuda.synchronize(dev0)
                t0 = time.perf_counter()
                for k in range(steps):
                    frame(k)
                m.check()
                torch.cuda.synchronize(dev0)
                wall = time.perf_counter() - t0
                same = bool(torch.equal(bufs[(steps - 1) % 2], want))
                packed = m.transfer()[1]
                key = f"{weights}:{f}/{'packed' if packed else 'rgba8'}"
                ms = wall / steps * 1e3
                table[key] = {"ms_per_frame": round(ms, 4), "bit_identical": same}
                if not same:
                    raise RuntimeError(f"c_abi_multi {fw}x{fh} {key}: frame differs from one GPU")
                if best is None or ms < best[1]:
                    best = (key, ms)
        out[f"{fw}x{fh}_{sname}"] = {
            "n_gpus": n, "Mrays_per_s": round(fw * fh / (best[1] * 1e-3) / 1e6, 2),
            "fps": round(1e3 / best[1], 2), "ms_per_frame": round(best[1], 4), "bands": best[0],
            "candidates": table, **want_check}
        del bufs, want
    m.close()
    return out


C_ABI_CHILD_TIMEOUT_S = 300


def c_abi_multi_isolated(devices, steps, warmup, settle_s):
    """c_abi_multi in a child process (bench.py --c-abi-child), so that a hang or a failure of
    the single-process RCCL path costs its own line only, never the headline JSON line: the
    child's result, or {"error": ...} on a non-zero exit, a bad frame or the time limit."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--c-abi-child", ",".join(map(str, devices)),
           "--also-steps", str(steps), "--also-warmup", str(warmup), "--also-settle", str(settle_s)]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                        "ROLE_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    try:
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=C_ABI_CHILD_TIMEOUT_S)
    except subprocess.TimeoutExpired:
        return {"devices": list(devices), "error": f"timed out after {C_ABI_CHILD_TIMEOUT_S} s"}
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        tail = (p.stderr or p.stdout).strip().splitlines()[-3:]
        return {"devices": list(devices), "error": f"exit {p.returncode}: " + " | ".join(tail)}
    return json.loads(lines[-1])


def c_abi_child(devices_arg: str, steps: int, warmup: int, settle_s: float) -> None:
    """bench.py --c-abi-child D0,D1,...: one c_abi_multi run, its result as one JSON line."""
    devs = [int(d) for d in devices_arg.split(",") if d.strip()]
    frames = [(7680, 4320, "lcg64")] + ([(16384, 16384, "lcg64")] if len(devs) >= 8 else [])
    try:
        out = c_abi_multi(devs, scenes.load_floor(), frames, steps, warmup, settle_s)
    except RuntimeError as e:  # a frame that differs from the one-GPU frame
        out = {"devices": devs, "error": str(e)}
    print(json.dumps(out), flush=True)


class GlslBands:
    """GlslShader.draw behind the render_band / check interface the timing helpers use
    (rayShader.frag per render-target pixel)."""

    def __init__(self, shader, width: int, height: int):
        self.shader, self.width, self.height = shader, width, height

    def render_band(self, dev_ptr, pitch, row0, rows, stream=0):
        self.shader.draw(dev_ptr, self.width, self.height, pitch, row0, rows, stream)

    def check(self, stream=0):
        self.shader.check(stream)


def valu_fraction(pixels: int, kernel: str, kernel_ms: float):
    """The launch's VALU issue rate from the newest committed PMC pass of `kernel` at this
    launch size (profiles/*_traffic.json) over this run's kernel time."""
    meas, src = measured_traffic(pixels, kernel)
    if not meas or "SQ_INSTS_VALU" not in meas or kernel_ms <= 0:
        return None
    rate = meas["SQ_INSTS_VALU"] / (kernel_ms * 1e-3)
    out = {"frac": round(rate / VALU_PEAK_WAVE_INSTS, 4),
           "frac_of_stream_ceiling": round(rate / VALU_STREAM_CEILING, 4),
           "valu_insts_per_launch": round(meas["SQ_INSTS_VALU"]), "source": src}
    if "hbm_bytes_per_launch" in meas:
        out["traffic_bytes_per_launch"] = round(meas["hbm_bytes_per_launch"])
    return out


SUPERVISOR_TIME_LIMIT_S = 1500
PG_TIMEOUT_S = 300


def _partial_write(path, result) -> None:
    """Rank 0's line so far (bench.py --partial-out): the supervisor prints it, with the
    failure under "error", if this process dies or hangs before printing the full line."""
    if not path or result is None:
        return
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(result, f)
    os.replace(tmp, path)


PARTIAL_EXIT = 4  # supervise(): the line carries a measured headline but is incomplete


def _die_with_parent() -> None:
    """preexec_fn of the supervised child (runs in the child before exec; the supervisor has not
    touched the GPU): SIGKILL when the supervisor exits, whatever ends it."""
    import ctypes
    import signal
    try:
        ctypes.CDLL(None, use_errno=True).prctl(1, int(signal.SIGKILL), 0, 0, 0)  # PR_SET_PDEATHSIG
    except (OSError, AttributeError):
        pass


def supervise(argv, rank: int, world_size: int, time_limit: float) -> int:
    """N > 1 (one process per GPU under torch.distributed.run): this rank's body runs in a child
    process (bench.py --worker), so that an RCCL failure -- communicator init, a collective on
    device bands, a hang in the tuner -- ends in ONE parseable JSON line from rank 0 with an
    "error" field instead of a crash or a hang without output.  The supervisor never touches the
    GPU (the child is the only process that initialises HIP).  It relays the child's output; the
    child runs under a process-group timeout (PG_TIMEOUT_S, so a stuck collective raises) and the
    supervisor's own limit.  If the child fails, hangs past `time_limit` or the supervisor is
    signalled (torch.distributed.run ends every rank when one rank fails), rank 0 prints the line
    the child had reached (--partial-out: the headline once measured, then every also line) with
    "error" = {stage, exit, detail}, or a line with "value": null when the headline was not
    reached.  Exit status (rank 0): 0 for a complete line, 3 for a complete line with a frame that
    differs, PARTIAL_EXIT (4) for a line with a measured headline and "complete": false -- so a
    partial run shows in the status the driver sees, not only in the JSON body -- and 1 for a line
    with no headline; ranks != 0 pass their child's status on.  The signal handlers it installs are
    restored before it returns, and the child is killed if the supervisor dies first
    (PR_SET_PDEATHSIG: the child runs in its own session, out of reach of the group signals
    torch.distributed.run sends).  Reference caller: Source.cpp:47-52."""
    import collections
    import signal
    import subprocess
    import tempfile
    import threading
    partial = None
    if rank == 0:
        fd, partial = tempfile.mkstemp(prefix="bench_partial_", suffix=".json")
        os.close(fd)
        os.unlink(partial)
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + list(argv) + ["--worker"]
    if partial:
        cmd += ["--partial-out", partial]
    child = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                             start_new_session=True, preexec_fn=_die_with_parent)
    seen = {"line": False}
    tail = collections.deque(maxlen=12)

    def relay(src, dst, keep):
        for ln in src:
            if keep:
                tail.append(ln.rstrip())
            elif ln.startswith('{"metric"'):
                seen["line"] = True
            dst.write(ln)
            dst.flush()
    threads = [threading.Thread(target=relay, args=(child.stdout, sys.stdout, False), daemon=True),
               threading.Thread(target=relay, args=(child.stderr, sys.stderr, True), daemon=True)]
    for t in threads:
        t.start()
    why = {"signal": None}

    def stop_child():
        for sig, wait in ((signal.SIGTERM, 10), (signal.SIGKILL, 10)):
            try:
                os.killpg(child.pid, sig)
            except ProcessLookupError:
                return
            try:
                child.wait(timeout=wait)
                return
            except subprocess.TimeoutExpired:
                continue

    def on_signal(signum, _frame):
        why["signal"] = signal.Signals(signum).name
        stop_child()
    previous = {sg: signal.signal(sg, on_signal) for sg in (signal.SIGTERM, signal.SIGINT)}
    try:
        deadline = time.monotonic() + time_limit
        timed_out = False
        while child.poll() is None:
            if time.monotonic() > deadline:
                timed_out = True
                stop_child()
                break
            time.sleep(0.2)
        try:
            rc = child.wait(timeout=30)
        except subprocess.TimeoutExpired:  # not gone even after SIGKILL (stuck in the driver)
            rc = -9
        for t in threads:
            t.join(timeout=5)
    finally:
        for sg, h in previous.items():
            signal.signal(sg, h)
    if rank != 0:
        return rc if rc >= 0 else 1
    line = None
    if partial and os.path.exists(partial):
        try:
            line = json.load(open(partial))
        except (OSError, ValueError):
            line = None
        os.unlink(partial)
    if rc == 0 and seen["line"] and not (timed_out or why["signal"]):
        return 0
    if seen["line"]:  # the full line is out (rc 3: it reports frames that differ)
        if rc != 3:
            print(f"bench supervisor: rank 0 exited {rc} after printing its line", file=sys.stderr)
        return 3 if rc == 3 else 0
    if timed_out:
        cause = f"time limit {time_limit:.0f} s (supervisor)"
    elif why["signal"]:
        cause = f"supervisor received {why['signal']} (another rank failed?)"
    else:
        cause = f"rank 0 body exited {rc}"
    headline = line is not None and line.get("value") is not None
    if line is None:
        line = {"metric": "Mrays/s (primary rays, full RGBA8 frames in HBM)", "value": None,
                "unit": "Mrays/s", "n_gpus": world_size, "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic"}
    line["error"] = {"stage": line.pop("_stage", "before the headline"), "cause": cause,
                     "exit": rc, "detail": list(tail)[-6:]}
    line["complete"] = False
    print(json.dumps(line), flush=True)
    return PARTIAL_EXIT if headline else 1


def injected_failure(args, rank: int, world_size: int, where: str) -> None:
    """TEST ONLY (--inject-failure MODE@WHERE, tests/test_bench_failures.py): rank 1 fails at
    `where` while the other ranks enter a collective: "raise" raises, "exit" ends the process
    abruptly, "hang" blocks until killed.  Never part of a measurement."""
    mode = args.inject_failure.split("@")[0]
    if rank == 1:
        print(f"rank 1: injected failure {args.inject_failure}", file=sys.stderr, flush=True)
        if mode == "raise":
            raise RuntimeError(f"injected failure at {where}")
        if mode == "exit":
            os._exit(7)
        while True:
            time.sleep(1)
    dist.barrier()  # never completes: rank 1 does not join


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--settle", type=float, default=0.3,
                    help="seconds of untimed frames before the warm-up (clock ramp)")
    ap.add_argument("--also-steps", type=int, default=200,
                    help="timed frames of every line under also (at least 20)")
    ap.add_argument("--also-warmup", type=int, default=20, help="warm-up frames of those lines")
    ap.add_argument("--also-settle", type=float, default=0.2,
                    help="seconds of untimed frames before every line under also")
    ap.add_argument("--bands", choices=("tuned", "equal"), default="tuned",
                    help="N > 1 row bands: tuned during the warm-up (default) or the plain "
                         "equal split, one gather per frame")
    ap.add_argument("--c-abi-devices", type=str, default="",
                    help="devices of the sfrt_multi line (default at N > 1: 0..N-1; e.g. 0,0,0,0 "
                         "rehearses it on one GPU with peer copies)")
    ap.add_argument("--c-abi-child", type=str, default="", help=argparse.SUPPRESS)
    ap.add_argument("--rehearse", action="store_true",
                    help="TEST ONLY, never a measurement: every rank on cuda:0 over a gloo "
                         "process group (RCCL refuses two ranks on one device), point-to-point "
                         "band transfers staged through host memory; runs the N > 1 body of "
                         "this script on a one-GPU box (tests/test_bench_rehearsal.py)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the 8K / 16K frames")
    ap.add_argument("--no-f1f2", action="store_true", help="skip the GLSL-mode and voxel lines")
    ap.add_argument("--headline-only", action="store_true",
                    help="only the headline workload (no also lines, no CPU baseline): the command "
                         "whose rocprof kernel trace profiles/*_kernel_stats_by_grid.csv summarises")
    ap.add_argument("--time-limit", type=float, default=SUPERVISOR_TIME_LIMIT_S,
                    help="N > 1: seconds before the supervisor ends a rank's body and rank 0 "
                         "prints the line reached so far with an error field")
    ap.add_argument("--pg-timeout", type=float, default=PG_TIMEOUT_S,
                    help="N > 1: process-group timeout in seconds (a collective stuck longer raises)")
    ap.add_argument("--worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--partial-out", type=str, default="", help=argparse.SUPPRESS)
    ap.add_argument("--inject-failure", type=str, default="",
                    help="TEST ONLY (MODE@WHERE, MODE raise|exit|hang, WHERE init|also): rank 1 "
                         "fails there; the run then ends in rank 0's error line")
    args = ap.parse_args()
    also_steps, also_warmup = max(20, args.also_steps), max(5, args.also_warmup)
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size > 1 and not (args.worker or args.c_abi_child):
        return supervise(sys.argv[1:], rank, world_size, args.time_limit)
    from datetime import timedelta
    pg_timeout = timedelta(seconds=args.pg_timeout)
    if args.inject_failure.endswith("@init"):  # TEST ONLY: no GPU needed
        dist.init_process_group("gloo", timeout=pg_timeout)
        injected_failure(args, rank, world_size, "init")
        return 1

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device (no CPU fallback)")
    if args.c_abi_child:
        c_abi_child(args.c_abi_child, args.also_steps, args.also_warmup, args.also_settle)
        return 0
    if sfrt.build_flavour() != "release":
        raise SystemExit(f"bench.py measures the release library only; {sfrt.LIB_PATH} reports "
                         f"build flavour {sfrt.build_flavour()!r} (unset SFRT_LIB, rebuild)")
    if world_size != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world_size}")
    device = 0 if args.rehearse else local_rank
    torch.cuda.set_device(device)
    host_group = None
    if world_size > 1:
        if args.rehearse:
            dist.init_process_group("gloo", timeout=pg_timeout)
            bands_mod.stage_p2p_through_host()
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank),
                                    timeout=pg_timeout)
        # a host-side barrier for the c_abi_multi line: ranks waiting on an RCCL barrier
        # would keep a kernel spinning on the GPUs rank 0 renders on
        host_group = dist.new_group(backend="gloo",
                                    timeout=timedelta(seconds=C_ABI_CHILD_TIMEOUT_S + 120))

    floor = scenes.load_floor()
    scene = scenes.lcg64()
    height = ROWS_PER_GPU * world_size
    pitch = WIDTH * 4
    # A dedicated stream: the kernels, the HIP events that time them and the
    # RCCL gather (which orders itself after the current stream) all use it.
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    w = sfrt.World(device)
    w.load_texture(*floor)
    w.set_scene(scene, WIDTH, height)

    settle(w, pitch, *band_of(rank, world_size, height), stream, args.settle)
    pipe, bands = tuned_pipeline(w, rank, world_size, height, pitch, stream, args.bands)
    row0, rows = pipe.row0, pipe.rows
    settle(w, pitch, row0, rows, stream, 0.1)  # the tuning's host work let the clock drop
    wall, kernel_ms = time_frames(w, pipe, pitch, args.steps, args.warmup, stream)
    wall = max_over_ranks(wall)
    total_rays = WIDTH * height * args.steps
    value = total_rays / wall / 1e6
    ms_per_step = wall / args.steps * 1e3

    result = None
    if rank == 0:
        rays_per_launch = WIDTH * rows
        achieved = BYTES_PER_RAY * rays_per_launch / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
        result = {
            "metric": "Mrays/s (primary rays, full RGBA8 frames in HBM)",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "fps": round(1e3 / ms_per_step, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: pinned 64-sphere cave (SURVEY 8d config 3), Floor.png texels",
            "config": {"workload": f"{WIDTH}x{height} lcg64 pose(0,0), {world_size} row band(s)"
                                   + (" + RCCL transfer to rank 0 (overlapped, bands "
                                      + ("tuned)" if args.bands == "tuned" else "equal)")
                                      if world_size > 1 else ""),
                       "width": WIDTH, "height": height, "spheres": int(scene.spheres.shape[0]),
                       "camera": "static pose (0,0); moving-camera lines under also",
                       "parallelism": f"row-bands x{world_size}",
                       "frames_in_flight": 1},
            "kernel_ms": round(kernel_ms, 4),
            "bands": bands,
            "library": {"path": os.path.relpath(sfrt.LIB_PATH, ROOT),
                        "build_flavour": sfrt.build_flavour(), "abi_version": sfrt.lib().sfrt_version()},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": None,
                         "note": "algorithmic bytes = 4 B/ray (RGBA8 store) x rays per launch / "
                                 "kernel time (HIP events on the launch stream around every 8th timed frame); the kernel is "
                                 "VALU-issue-bound, see valu_roofline and DESIGN.md"},
        }
        if args.rehearse:
            result["metric"] = "REHEARSAL, not a measurement: " + result["metric"]
            result["rehearsal"] = {
                "backend": "gloo" if world_size > 1 else None, "devices": "every rank on cuda:0",
                "p2p": "staged through host memory (bands.stage_p2p_through_host)",
                "note": "tests/test_bench_rehearsal.py: the N > 1 body of bench.py on a one-GPU "
                        "box; the driver's SCALE run uses RCCL with one GPU per rank"}
        meas, src = measured_traffic(rays_per_launch)
        if meas:
            result["roofline"]["traffic"] = round(meas["hbm_bytes_per_launch"])
            result["roofline"]["traffic_source"] = src
            if "SQ_INSTS_VALU" in meas and kernel_ms > 0:
                rate = meas["SQ_INSTS_VALU"] / (kernel_ms * 1e-3)
                result["valu_roofline"] = {
                    "achieved": round(rate / 1e12, 4), "peak": round(VALU_PEAK_WAVE_INSTS / 1e12, 4),
                    "unit": "T wave64-VALU-instructions/s", "frac": round(rate / VALU_PEAK_WAVE_INSTS, 4),
                    "stream_ceiling": round(VALU_STREAM_CEILING / 1e12, 4),
                    "frac_of_stream_ceiling": round(rate / VALU_STREAM_CEILING, 4),
                    "valu_insts_per_launch": round(meas["SQ_INSTS_VALU"]),
                    "valu_insts_per_ray": round(meas["SQ_INSTS_VALU"] * 64 / rays_per_launch, 1),
                    "source": src}
        # the last timed frame (gathered on rank 0 at N > 1) against the golden frame
        result["frame_check"] = verify_frame(pipe.frame(args.steps - 1), "frames",
                                             scenes.golden_key(WIDTH, height, "lcg64"))
    if world_size > 1 and rank == 0:
        # The last gathered frame must equal a single-GPU render of the whole frame.
        frame = pipe.frame(args.steps - 1)
        single = torch.empty_like(frame)
        w.render_band(single.data_ptr(), pitch, 0, height, stream.cuda_stream)
        w.check(stream.cuda_stream)
        result["gathered_frame_bit_identical"] = bool(torch.equal(single, frame))
        del single
    if rank == 0:
        _partial_write(args.partial_out, dict(result, _stage="after the headline"))
    if args.inject_failure.endswith("@also"):  # TEST ONLY
        injected_failure(args, rank, world_size, "also")
    # Larger frames of the BASELINE configs (strong scaling: the frame is fixed,
    # its rows split over the ranks), measured after the main line.
    extra = {}
    if not (args.no_extra or args.headline_only):
        for fw, fh, sname in EXTRA_FRAMES.get(world_size, []):
            sc_x = scene if sname == "lcg64" else scenes.SCENES[sname]()
            line = measure_frame(w, sc_x, fw, fh, rank, world_size, also_steps, also_warmup,
                                 stream, args.also_settle, args.bands)
            if world_size == 1:  # one band: the kernel is the frame
                line["hbm_frac"] = line.pop("hbm_frac_rank0_kernel")
                line["kernel_ms"] = line.pop("kernel_ms_rank0_band")
            extra[f"{fw}x{fh}_{sname}"] = line
            if rank == 0:
                _partial_write(args.partial_out, dict(result, also=dict(extra),
                                                      _stage=f"after also/{fw}x{fh}_{sname}"))
        w.set_scene(scene, WIDTH, height)
    if rank == 0:
        result["also"] = dict(extra)
        result["also_timing"] = {"steps": also_steps, "warmup": also_warmup,
                                 "settle_s": args.also_settle}
    if args.c_abi_devices:
        c_devs = [int(d) for d in args.c_abi_devices.split(",") if d.strip()]
    elif world_size > 1:
        c_devs = [0] * world_size if args.rehearse else list(range(world_size))
    else:
        c_devs = []
    if c_devs and not (args.no_extra or args.headline_only):
        # the single-process multi-GPU path (C ABI), by rank 0 alone while the others wait
        if rank == 0:
            result["also"]["c_abi_multi"] = c_abi_multi_isolated(c_devs, max(20, also_steps // 4),
                                                                 also_warmup, args.also_settle)
        if host_group is not None:
            dist.barrier(group=host_group)
    if world_size == 1 and not args.headline_only:
        def line(wx, fw, fh, name, per_frame=None, in_flight=1, golden=None, kernel="k_trace",
                 **info):
            """One N = 1 line under also: its own settle, warm-up and timed frames; its last
            frame checked against golden = (section, key) of tests/golden/golden.json."""
            pipe_x = BandPipeline(0, 1, fh, fw * 4, "cuda", local_depth=in_flight)
            settle(wx, fw * 4, 0, fh, stream, args.also_settle)
            wall_x, k_x = time_frames(wx, pipe_x, fw * 4, also_steps, also_warmup, stream,
                                      per_frame=per_frame, in_flight=in_flight)
            rec = {"n_gpus": 1, "Mrays_per_s": round(fw * fh * also_steps / wall_x / 1e6, 2),
                   "fps": round(also_steps / wall_x, 2),
                   "ms_per_frame": round(wall_x / also_steps * 1e3, 4)}
            if in_flight == 1:
                rec.update(kernel_ms=round(k_x, 4), hbm_frac=hbm_frac(fw * fh, k_x))
                if kernel != "k_trace":
                    rec["valu"] = valu_fraction(fw * fh, kernel, k_x)
            else:
                rec.update(kernel_ms_per_launch_overlapping=round(k_x, 4), frames_in_flight=in_flight,
                           streams=in_flight)
            rec.update(info)
            rec.update(verify_frame(pipe_x.frame(also_steps - 1), *(golden or ("frames", None))))
            result["also"][name] = rec
            del pipe_x

        # BASELINE config 2: 1920x1080, 10-sphere scene.
        w2 = sfrt.World(device)
        w2.load_texture(*floor)
        w2.set_scene(scenes.default10(), 1920, 1080)
        line(w2, 1920, 1080, "1920x1080_default10",
             golden=("frames", scenes.golden_key(1920, 1080, "default10")))
        w2.close()
        # BASELINE config 3 with "all textures": every reference texture resident, one
        # per sphere (the per-sphere texture extension; the main line is textures[0]).
        w3 = sfrt.World(device)
        for slot, (rgba, tw, th) in enumerate(scenes.load_all_textures()):
            w3.load_texture(rgba, tw, th, slot=slot)
        w3.set_scene(scene, WIDTH, height)
        w3.set_sphere_textures(scenes.all_texture_slots(scene.spheres.shape[0]))
        line(w3, WIDTH, height, "3840x2160_lcg64_all_textures",
             golden=("all_textures", f"{WIDTH}x{height}_lcg64@0,0"))
        w3.close()
        # The adaptive tile order dispatches each frame's tiles longest-first
        # by recorded march steps.  The same workload with a camera turning every frame, in
        # both orders, and the static camera in plain row-major order.  Only the camera
        # changes per frame (one C-ABI call).  The turn ends at pose (0, 0) on the last timed
        # frame, so that frame is checked against the headline's golden frame.
        last = also_warmup + also_steps - 1
        key4k = ("frames", scenes.golden_key(WIDTH, height, "lcg64"))

        def turn(k):
            w.set_camera(scene.cam_pos, 0.004 * (k - last), 0.0)
        for order, key in ((1, "3840x2160_lcg64_turning"), (0, "3840x2160_lcg64_turning_row_major"),
                           (0, "3840x2160_lcg64_row_major")):
            w.set_scene(scene, WIDTH, height)
            w.set_option(sfrt.SFRT_OPT_TILE_ORDER, order)
            moving = "turning" in key
            line(w, WIDTH, height, key, per_frame=turn if moving else None, golden=key4k,
                 camera="rotation = 0.004 rad x (frame index - last frame's)" if moving
                 else "static pose (0,0)",
                 tile_order="adaptive" if order else "row-major (SFRT_OPT_TILE_ORDER 0)")
        w.set_option(sfrt.SFRT_OPT_TILE_ORDER, 1)
        w.set_scene(scene, WIDTH, height)
        # Beyond the reference's scene sizes: 256 spheres (the n > 64 kernel).
        w5 = sfrt.World(device)
        w5.load_texture(*floor)
        w5.set_scene(scenes.lcg256(), WIDTH, height)
        line(w5, WIDTH, height, "3840x2160_lcg256", spheres=256,
             golden=("frames", scenes.golden_key(WIDTH, height, "lcg256")))
        w5.close()
        # Two frames in flight (see frame_streams): the 4K static and 1080p frames.
        for key, (fw, fh, sc2) in (("3840x2160_lcg64_2_in_flight", (WIDTH, height, scene)),
                                   ("1920x1080_default10_2_in_flight", (1920, 1080, scenes.default10()))):
            w6 = sfrt.World(device)
            w6.load_texture(*floor)
            w6.set_scene(sc2, fw, fh)
            line(w6, fw, fh, key, in_flight=2, golden=("frames", scenes.golden_key(fw, fh, sc2.name)))
            w6.close()
        if not args.no_f1f2:
            # SURVEY 8f rows f1 (GLSL mode, rayShader.frag:63-161) and f2 (voxel World,
            # World.cpp:302-491) under the same rules: settle, warm-up, timed frames, kernel
            # time from HIP events on the launch stream, the last frame against its golden.
            import glsl_scenes
            import voxel_scenes
            sh = sfrt.GlslShader(device)
            sh.set_ground(*floor)
            for fw, fh in ((1920, 1080), (WIDTH, height)):
                sh.set_uniforms(glsl_scenes.default_uniforms(fw, fh))
                line(GlslBands(sh, fw, fh), fw, fh, f"glsl_{fw}x{fh}", kernel="k_glsl",
                     golden=("glsl", f"default@{fw}x{fh}"),
                     scene="constructor scene (srand 0), rot (0,0)", unit="fragments")
            sh.close()
            vw = sfrt.VoxelWorld(device)
            vtex, vdyn = voxel_scenes.load_textures()
            vw.load_assets(vtex, vdyn, voxel_scenes.COLORS)
            pos = (15.5, 1.9, 15.5)
            for fw, fh in ((1920, 1080), (WIDTH, height)):
                vw.set_scene(voxel_scenes.default_world(pos, 0.0, 0.0), fw, fh)
                line(vw, fw, fh, f"voxel_{fw}x{fh}", kernel="k_voxel",
                     golden=("voxel", f"{fw}x{fh}@{pos[0]:g},{pos[1]:g},{pos[2]:g}/0,0"),
                     scene="default world, pose (15.5,1.9,15.5)/(0,0)")
            vw.close()
        torch.cuda.synchronize()
        gpu_frame = pipe.frame(args.steps - 1).cpu().numpy().ravel()
        result["also"]["3840x2160_lcg64_to_host"] = dict(
            host_delivery(device, floor, scene, WIDTH, height, 200, gpu_frame),
            note="PCIe-inclusive (frame copied into a host buffer), not the HBM-resident value")
        if not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(scene, WIDTH, height, floor, gpu_frame)
    rc = 0
    if rank == 0:
        # every frame the line checked must be bit-identical to its golden / one-GPU frame; a line
        # with any that differs is marked invalid and the run exits 3 (after printing it)
        bad = [k for k, v in bit_identity_flags(result) if v is not True]
        result["all_frames_bit_identical"] = not bad
        if bad:
            result["invalid"] = {"frames_differ": bad}
            rc = 3
        print(json.dumps(result), flush=True)
    w.close()
    if world_size > 1:
        dist.barrier()
        dist.destroy_process_group()
    return rc


def bit_identity_flags(obj, path=""):
    """(path, value) of every bit-identity flag in a result line (keys naming bit_identical)."""
    out = []
    if isinstance(obj, dict):
        for k, v in obj.items():
            p = f"{path}/{k}" if path else k
            if "bit_identical" in k and not isinstance(v, (dict, list)):
                out.append((p, v))
            else:
                out += bit_identity_flags(v, p)
    elif isinstance(obj, list):
        for i, v in enumerate(obj):
            out += bit_identity_flags(v, f"{path}[{i}]")
    return out


if __name__ == "__main__":
    sys.exit(main())
