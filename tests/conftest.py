import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "sfml-software-raytracer_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsfrt.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long CPU test (still part of the default suite)")


def poisoned(shape, value: int = 0xA5):
    """A uint8 buffer on cuda:0 filled with `value`, the fill complete on return.  The tests
    render on their own streams (torch pool streams: non-blocking), which nothing orders after
    the fill torch queues on its current stream -- a fill still pending there could overwrite
    a frame rendered on another stream.  Only the current stream is waited for."""
    import torch
    t = torch.full(shape, value, dtype=torch.uint8, device="cuda:0")
    torch.cuda.current_stream().synchronize()
    return t


def host_threads() -> int:
    """CPU threads for the oracle: the container's cores here, at most 16 on the GPU box."""
    return max(1, min(16, os.cpu_count() or 1))


@pytest.fixture(scope="session")
def floor():
    import scenes
    return scenes.load_floor()


@pytest.fixture(scope="session")
def built():
    """Build libsfrt.so and the oracle once per session (no-op when up to date)."""
    import __graft_entry__ as g
    g.build()
    return True
