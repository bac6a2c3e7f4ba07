"""bench.py --gpus N end to end on a one-GPU box: the driver's SCALE command, rehearsed.

The driver launches `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`
on an 8-GPU node, one rank per GPU over RCCL.  RCCL refuses two ranks on one device, so
`--rehearse` (test only; the JSON line says REHEARSAL and is never a measurement) runs the same
N > 1 body with every rank on cuda:0 over a gloo process group: the band tuner over device
tensors (all-reduced timings and row costs), the equal-band `dist.gather` of device bands
(gloo's HIP path, bands.BandPipeline.submit), the point-to-point and packed transfers staged
through host memory, the gathered-frame check against a one-GPU render, the N > 1 also-frames
and the c_abi_multi child over devices [0] * N (peer copies).  Every frame that has a golden
frame must equal it (bench.py verify_frame; tests/golden/golden.json, c2/c3/c4 and w2/w4).
Reference caller: Source.cpp:47-52 (one frame filled by every render thread).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(n, extra, timeout=240):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "bench.py", "--gpus", str(n), "--rehearse", "--steps", "10", "--warmup", "2",
           "--settle", "0", "--also-steps", "20", "--also-warmup", "5", "--also-settle", "0",
           "--no-cpu-baseline"] + extra
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or len(lines) != 1:
        err = p.stderr
        tb = err.find("Traceback (most recent call last)")  # the first rank's own error
        raise AssertionError(f"exit {p.returncode}, {len(lines)} JSON lines\n"
                             + (err[tb:tb + 6000] if tb >= 0 else err[-6000:]))
    return json.loads(lines[0])


# N = 8 is the driver's largest SCALE run and the only one with the 16384^2 lines (BASELINE
# config 5): rehearsing it found a division by a band's zero event time (1080p over 8 ranks)
@pytest.mark.parametrize("n,band_mode", [(2, "equal"), (4, "tuned"), (8, "equal")])
def test_bench_multi_gpu_body_rehearsed(n, band_mode):
    r = _run(n, ["--bands", band_mode])
    assert r["n_gpus"] == n and r["metric"].startswith("REHEARSAL")
    assert r["rehearsal"]["devices"] == "every rank on cuda:0"
    assert r["value"] > 0 and r["steps"] == 10
    assert r["gathered_frame_bit_identical"] is True
    # the weak-scaling frame 3840 x 2160*N against its golden frame (w2_*, w4_*)
    assert r["frame_check"]["golden"] == f"frames/w{n}_3840x{2160 * n}_lcg64@0,0"
    assert r["frame_check"]["bit_identical"] is True
    rows = r["bands"]["rows_per_rank"]
    assert len(rows) == n and sum(rows) == 2160 * n
    if band_mode == "equal":  # one gather of device bands per frame, every line
        assert rows == [2160] * n and r["bands"]["tuning"].startswith("off")
    else:
        assert r["bands"]["tuning_ms_per_frame"]
    also = r["also"]
    lines = [("1920x1080_default10", "frames/c2_1920x1080_default10@0,0"),
             ("3840x2160_lcg64", "frames/c3_3840x2160_lcg64@0,0"),
             ("7680x4320_lcg64", "frames/c4_7680x4320_lcg64@0,0")]
    if n == 8:
        lines.append(("16384x16384_lcg64", "frames/c5_16384x16384_lcg64@0,0"))
    for key, golden in lines:
        line = also[key]
        assert line["n_gpus"] == n and line["Mrays_per_s"] > 0, key
        assert line["golden"] == golden and line["bit_identical"] is True, (key, line)
        if band_mode == "equal":
            assert len(set(line["bands"]["rows_per_rank"])) == 1, (key, line["bands"])
    c = also["c_abi_multi"]
    assert "error" not in c, c
    assert c["devices"] == [0] * n and c["transport"] == "peer"
    frames = [("7680x4320_lcg64", "frames/c4_7680x4320_lcg64@0,0")]
    if n == 8:
        frames.append(("16384x16384_lcg64", "frames/c5_16384x16384_lcg64@0,0"))
    for key, golden in frames:
        ent = c[key]
        assert ent["bit_identical"] is True and ent["golden"] == golden, (key, ent)
        assert all(v["bit_identical"] for v in ent["candidates"].values()), key
