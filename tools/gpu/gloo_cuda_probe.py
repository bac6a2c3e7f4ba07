"""Probe: which torch.distributed gloo collectives move HIP device tensors on this image, with
several ranks sharing cuda:0 (RCCL refuses two ranks on one device).  bench.py --rehearse
relies on gather / all_reduce / barrier here; point-to-point transfers are staged through host
memory there (gloo's send/recv take host buffers).

    python tools/gpu/gloo_cuda_probe.py [world_size]
"""
import os
import socket
import sys

import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port):
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    torch.cuda.set_device(0)
    side = torch.cuda.Stream()
    torch.cuda.set_stream(side)
    rows, pitch = 37, 64
    band = torch.full((rows, pitch), rank + 1, dtype=torch.uint8, device="cuda")
    frame = torch.zeros(rows * world, pitch, dtype=torch.uint8, device="cuda") if rank == 0 else None
    views = [frame[r * rows:(r + 1) * rows] for r in range(world)] if rank == 0 else None
    work = dist.gather(band, views, dst=0, async_op=True)
    work.wait()
    if rank == 0:
        want = torch.arange(1, world + 1, dtype=torch.uint8, device="cuda").repeat_interleave(rows)
        ok = bool(torch.equal(frame[:, 0], want)) and bool((frame == frame[:, :1]).all())
        print(f"gather cuda async: {'ok' if ok else 'WRONG'}", flush=True)
    t = torch.tensor([float(rank)], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.ones(5, dtype=torch.float64, device="cuda") * rank
    dist.all_reduce(s)
    if rank == 0:
        print(f"all_reduce cuda max {t.item()} (want {world - 1}), sum {s[0].item()} "
              f"(want {world * (world - 1) / 2})", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    mp.start_processes(worker, args=(n, _free_port()), nprocs=n, start_method="spawn", join=True)
    print("probe done", flush=True)
