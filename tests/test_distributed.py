"""Multi-rank row bands + gather (bench.py's N > 1 path) on CPU with gloo.

Each rank renders its row band of the frame with the CPU restatement (this is
test infrastructure standing in for the device fill), then bench.py's own
band_buffers / dist.gather assemble the frame on rank 0, which must equal the
single-rank frame byte for byte.  world_size 2 and 3 (uneven band sizes).
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
    o = oracle.Oracle.from_scene(scenes.lcg64().posed(0.4, 0.05), width, height, tex, tw, th)
    pitch = width * 4
    buf, frame, gather_list = bench.band_buffers(rank, world_size, height, pitch, "cpu")
    row0, rows = bench.band_of(rank, world_size, height)
    buf.copy_(torch.from_numpy(o.render_band(row0, rows).reshape(rows, pitch)))
    bench.gather_bands(buf, gather_list, rank, world_size, height)
    if rank == 0:
        full = o.render(2).reshape(height, pitch)
        np.save(out_path, np.array([np.array_equal(frame.numpy(), full)]))
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
