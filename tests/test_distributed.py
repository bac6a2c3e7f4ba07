"""Multi-rank row bands + gather (bench.py's N > 1 path) on CPU with gloo.

Each rank renders its row band of the frame with the CPU restatement (this is
test infrastructure standing in for the device fill), then bench.py's own
BandPipeline (double-buffered bands, asynchronous gather / point-to-point
transfers to rank 0) assembles the frames on rank 0, which must equal the
single-rank frames byte for byte -- three frames with different camera poses
in flight without draining in between.  world_size 2 and 3 (uneven bands).
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


def _worker(rank, world_size, port, width, height, out_path):
    import sys
    for p in (os.path.join(ROOT, "sfml-software-raytracer_amd"), os.path.join(ROOT, "oracle"), ROOT):
        sys.path.insert(0, p)
    import bench
    import oracle
    import scenes
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world_size)
    tex, tw, th = scenes.load_floor()
    pitch = width * 4
    poses = [(0.4, 0.05), (1.3, -0.2), (2.9, 0.3)]
    oracles = [oracle.Oracle.from_scene(scenes.lcg64().posed(*p), width, height, tex, tw, th)
               for p in poses]
    pipe = bench.BandPipeline(rank, world_size, height, pitch, "cpu")
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


@pytest.mark.parametrize("world_size,height", [(2, 90), (3, 100)])
def test_row_band_gather_matches_single_rank(tmp_path, world_size, height):
    out = str(tmp_path / "ok.npy")
    mp.start_processes(_worker, args=(world_size, _free_port(), 160, height, out),
                       nprocs=world_size, start_method="spawn", join=True)
    assert bool(np.load(out)[0])


def test_band_partition_covers_rows():
    import bench
    for world_size in (1, 2, 3, 4, 8):
        for height in (1, 7, 2160, 4320, 16384, 17280):
            if height < world_size:
                continue
            spans = [bench.band_of(r, world_size, height) for r in range(world_size)]
            assert spans[0][0] == 0
            assert sum(n for _, n in spans) == height
            for (a, n), (b, _) in zip(spans, spans[1:]):
                assert a + n == b
