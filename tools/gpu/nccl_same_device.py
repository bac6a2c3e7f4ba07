"""Probe: can two torch.distributed ranks share one GPU under RCCL on this image?"""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    t = torch.ones(4, device="cuda") * (rank + 1)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce ok {t.tolist()}", flush=True)
    dist.destroy_process_group()
except Exception as e:  # report and exit cleanly
    print(f"rank {rank}: failed: {type(e).__name__}: {e}", flush=True)
