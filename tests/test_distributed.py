"""Multi-rank row bands + gather (bench.py's N > 1 path) on CPU with gloo.

Each rank renders its row band of the frame with the CPU restatement (this is
test infrastructure standing in for the device fill), then the package's
bands.BandPipeline (double-buffered bands, asynchronous gather / point-to-point
transfers to rank 0) assembles the frames on rank 0, which must equal the
single-rank frames byte for byte -- three frames with different camera poses
in flight without draining in between.  world_size 2 and 3, equal and
root-weighted bands; the band tuner agrees across ranks.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world_size, port, width, height, out_path, factor=1.0, staged=False):
    import sys
    for p in (os.path.join(ROOT, "sfml-software-raytracer_amd"), os.path.join(ROOT, "oracle"), ROOT):
        sys.path.insert(0, p)
    import bands
    import oracle
    import scenes
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world_size)
    if staged:  # bench.py --rehearse: point-to-point transfers through host copies
        bands.stage_p2p_through_host()
    tex, tw, th = scenes.load_floor()
    pitch = width * 4
    poses = [(0.4, 0.05), (1.3, -0.2), (2.9, 0.3)]
    oracles = [oracle.Oracle.from_scene(scenes.lcg64().posed(*p), width, height, tex, tw, th)
               for p in poses]
    spans = bands.root_weighted_spans(height, world_size, factor)
    pipe = bands.BandPipeline(rank, world_size, height, pitch, "cpu", spans=spans)
    for k, o in enumerate(oracles):
        band = pipe.acquire(k)
        band.copy_(torch.from_numpy(o.render_band(pipe.row0, pipe.rows).reshape(pipe.rows, pitch)))
        pipe.submit(k)
    pipe.drain()
    if rank == 0:
        ok = [np.array_equal(pipe.frame(k).numpy(), oracles[k].render(2).reshape(height, pitch))
              for k in (1, 2)]
        np.save(out_path, np.array([all(ok)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world_size,height,factor,staged", [
    (2, 90, 1.0, False), (3, 100, 1.0, False), (2, 90, 2.5, False), (3, 100, 1.5, False),
    (3, 100, 1.5, True), (4, 120, 2.0, True)])
def test_row_band_gather_matches_single_rank(tmp_path, world_size, height, factor, staged):
    """staged: the host-staged point-to-point stand-in of bench.py --rehearse
    (bands.stage_p2p_through_host), unequal bands so that every band crosses it."""
    out = str(tmp_path / "ok.npy")
    mp.start_processes(_worker, args=(world_size, _free_port(), 160, height, out, factor, staged),
                       nprocs=world_size, start_method="spawn", join=True)
    assert bool(np.load(out)[0])


def test_band_partition_covers_rows():
    import bands
    for world_size in (1, 2, 3, 4, 8):
        for height in (1, 7, 90, 2160, 4320, 16384, 17280):
            if height < world_size:
                continue
            for factor in (1.0,) + bands.DEFAULT_FACTORS + (0.5, 10.0):
                spans = bands.root_weighted_spans(height, world_size, factor)
                bands.check_spans(spans, height)
                assert len(spans) == world_size
                if spans != bands.equal_spans(height, world_size):
                    # weighted: equal, tile-aligned bands on ranks 1.., rank 0 takes the rest
                    others = {n for _, n in spans[1:]}
                    assert len(others) == 1 and others.pop() % bands.ALIGN == 0
                    assert spans[0][1] >= spans[1][1] or factor < 1.0
    eq = bands.root_weighted_spans(17280, 8, 1.0)
    assert eq == [(r * 2160, 2160) for r in range(8)]
    w = bands.root_weighted_spans(17280, 8, 2.0)
    assert w[1][1] == 1920 and w[0][1] == 17280 - 7 * 1920


def _tune_worker(rank, world_size, port, out_path):
    import sys
    for p in (os.path.join(ROOT, "sfml-software-raytracer_amd"), ROOT):
        sys.path.insert(0, p)
    import time
    import bands
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world_size)
    height, pitch = 64, 16

    def render(band, row0, rows):  # rows [row0, row0+rows) of a synthetic frame
        band.copy_(torch.arange(row0, row0 + rows, dtype=torch.int64).remainder(251)
                   .to(torch.uint8)[:, None].expand(rows, pitch))
        time.sleep(1e-4 * rows if rank == 0 else 1e-5 * rows)

    spans, pick, table = bands.tune_spans(render, rank, world_size, height, pitch, "cpu",
                                          factors=(1.0, 2.0, 3.0), frames=3, warm=1)
    got = torch.tensor([pick["root_factor"]] + [float(n) for _, n in spans], dtype=torch.float64)
    allv = [torch.zeros_like(got) for _ in range(world_size)]
    dist.all_gather(allv, got)
    pipe = bands.BandPipeline(rank, world_size, height, pitch, "cpu", spans=spans)
    bands.run_frames(pipe, render, 2)
    if rank == 0:
        want = torch.arange(height).remainder(251).to(torch.uint8)[:, None].expand(height, pitch)
        same = all(torch.equal(a, allv[0]) for a in allv)
        np.save(out_path, np.array([same, torch.equal(pipe.frame(1), want), len(table) == 3]))
    dist.barrier()
    dist.destroy_process_group()


def test_tune_spans_agrees_across_ranks(tmp_path):
    """Every rank picks the same partition, and the tuned pipeline assembles the frame."""
    out = str(tmp_path / "tune.npy")
    mp.start_processes(_tune_worker, args=(3, _free_port(), out), nprocs=3,
                       start_method="spawn", join=True)
    assert np.load(out).all()


def _row_cost_worker(rank, world_size, port, out_path):
    import sys
    for p in (os.path.join(ROOT, "sfml-software-raytracer_amd"), ROOT):
        sys.path.insert(0, p)
    import types
    import bands
    import bench
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world_size)
    height, pitch = 100, 16
    calls = []

    class FakeWorld:  # stands in for sfrt.World: row j of the frame costs j + 1
        def render_band(self, ptr, p, row0, rows, stream):
            calls.append((row0, rows))

        def row_costs(self):
            row0, rows = calls[-1]
            return row0, np.arange(row0 + 1, row0 + rows + 1, dtype=np.float32)

    cost = bench.frame_row_costs(FakeWorld(), rank, world_size, height, pitch,
                                 types.SimpleNamespace(cuda_stream=0), device="cpu")
    ok = [calls == [bands.band_of(rank, world_size, height)],
          bool(np.array_equal(cost, np.arange(1, height + 1, dtype=np.float32)))]

    class BrokenOnRank1(FakeWorld):  # one rank's costs fail: every rank falls back
        def row_costs(self):
            if rank == 1:
                raise RuntimeError("no ordered fill")
            return super().row_costs()

    ok.append(bench.frame_row_costs(BrokenOnRank1(), rank, world_size, height, pitch,
                                    types.SimpleNamespace(cuda_stream=0), device="cpu") is None)
    spans = bands.cost_weighted_spans(cost, world_size, 1.0)
    got = torch.tensor([float(n) for _, n in spans], dtype=torch.float64)
    allv = [torch.zeros_like(got) for _ in range(world_size)]
    dist.all_gather(allv, got)
    ok.append(all(torch.equal(a, allv[0]) for a in allv))
    if rank == 0:
        np.save(out_path, np.array(ok))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_row_costs_sum_over_ranks(tmp_path):
    """bench.frame_row_costs: every rank renders its equal band once and the ranks' row costs
    add up to the whole frame's vector (the cost-weighted band tuner's input at N > 1)."""
    out = str(tmp_path / "rc.npy")
    mp.start_processes(_row_cost_worker, args=(3, _free_port(), out), nprocs=3,
                       start_method="spawn", join=True)
    assert np.load(out).all()
