"""bench.py --gpus N: a failing rank ends the run in ONE parseable JSON line with an "error" field.

The driver's SCALE command (`torch.distributed.run --nproc-per-node N bench.py --gpus N`) is the
first place RCCL runs over real links (reference caller: Source.cpp:47-52, the render threads
filling one frame).  bench.py runs each rank's body in a child process under a supervisor
(bench.supervise) with a process-group timeout; these CPU tests inject the failures that path can
meet -- a collective that raises, a rank that dies, a rank that never joins -- with
`--inject-failure MODE@init` (TEST ONLY: rank 1 fails right after the gloo process group is up,
rank 0 waits in a collective), and check that rank 0 prints exactly one JSON line carrying the
metric, n_gpus, "value": null and an "error", and that the run ends well inside its limits.
"""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(mode, extra=(), timeout=180):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "bench.py", "--gpus", "2", "--inject-failure", f"{mode}@init",
           "--pg-timeout", "8", "--time-limit", "90"] + list(extra)
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    t0 = time.monotonic()
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, lines, time.monotonic() - t0


@pytest.mark.parametrize("mode", ["raise", "exit", "hang"])
def test_failing_rank_gives_one_error_line(mode):
    p, lines, dt = _run(mode)
    assert len(lines) == 1, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    line = json.loads(lines[0])
    assert line["metric"].startswith("Mrays/s") and line["n_gpus"] == 2
    assert line["value"] is None and line["complete"] is False
    err = line["error"]
    assert err["stage"] == "before the headline" and err["cause"], err
    assert p.returncode != 0  # no headline was measured
    assert dt < 150, dt  # the process-group timeout (8 s) or the teardown, not the 90 s limit


def test_supervisor_time_limit_ends_a_hung_run():
    # hang with a process-group timeout longer than the supervisor's limit: the limit ends it
    p, lines, dt = _run("hang", ["--pg-timeout", "600", "--time-limit", "15"])
    assert len(lines) == 1, (p.returncode, p.stderr[-4000:])
    line = json.loads(lines[0])
    assert line["value"] is None and "error" in line
    assert "time limit" in line["error"]["cause"] or "SIGTERM" in line["error"]["cause"]
    assert dt < 120, dt


def test_partial_line_keeps_a_measured_headline(tmp_path):
    """A failure after the headline: rank 0's supervisor prints the line the body had reached
    (bench.py --partial-out), with the error and "complete": false, and exits PARTIAL_EXIT (4,
    distinct from 0, from 1 = no headline and from 3 = frames differ), so the driver's status shows
    the partial run.  The supervisor's signal handlers are restored after it."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    fake = tmp_path / "fake_body.py"
    # a stand-in body: writes a partial line like bench.py's after its headline, then dies
    fake.write_text(
        "import json, os, sys\n"
        "i = sys.argv.index('--partial-out')\n"
        "json.dump({'metric': 'Mrays/s (test)', 'value': 123.0, 'n_gpus': 2,\n"
        "           '_stage': 'after the headline'}, open(sys.argv[i + 1], 'w'))\n"
        "print('body: dying after the headline', file=sys.stderr)\n"
        "os._exit(9)\n")
    import signal
    handlers = {sg: signal.getsignal(sg) for sg in (signal.SIGTERM, signal.SIGINT)}
    old_file = bench.__file__
    bench.__file__ = str(fake)
    try:
        from io import StringIO
        import contextlib
        out = StringIO()
        with contextlib.redirect_stdout(out):
            rc = bench.supervise([], 0, 2, 30)
    finally:
        bench.__file__ = old_file
    lines = [ln for ln in out.getvalue().splitlines() if ln.startswith("{")]
    assert bench.PARTIAL_EXIT not in (0, 1, 3)
    assert rc == bench.PARTIAL_EXIT and len(lines) == 1
    assert {sg: signal.getsignal(sg) for sg in handlers} == handlers
    line = json.loads(lines[0])
    assert line["value"] == 123.0 and line["complete"] is False
    assert line["error"]["stage"] == "after the headline" and line["error"]["exit"] == 9
    assert "dying after the headline" in " ".join(line["error"]["detail"])


def test_bit_identity_flags_found_everywhere():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    res = {"frame_check": {"bit_identical": True}, "gathered_frame_bit_identical": True,
           "also": {"a": {"bit_identical": False}, "c": {"candidates": {"x": {"bit_identical": True}}},
                    "h": {"pipelined_pinned": {"bit_identical_to_device_frame": True}}}}
    flags = dict(bench.bit_identity_flags(res))
    assert flags == {"frame_check/bit_identical": True, "gathered_frame_bit_identical": True,
                     "also/a/bit_identical": False, "also/c/candidates/x/bit_identical": True,
                     "also/h/pipelined_pinned/bit_identical_to_device_frame": True}


def test_supervised_child_dies_with_its_supervisor(tmp_path):
    """the body runs in its own session (start_new_session), out of reach of the group
    signals torch.distributed.run sends; if the supervisor itself is SIGKILLed, the body must not
    live on holding the GPU (PR_SET_PDEATHSIG in bench._die_with_parent)."""
    import signal
    import subprocess
    import sys
    import time
    fake = tmp_path / "sleepy_body.py"
    pidfile = tmp_path / "child.pid"
    fake.write_text("import os, sys, time\n"
                    f"open({str(pidfile)!r}, 'w').write(str(os.getpid()))\n"
                    "time.sleep(120)\n")
    driver = ("import importlib.util, sys\n"
              f"spec = importlib.util.spec_from_file_location('bench_mod', {os.path.join(ROOT, 'bench.py')!r})\n"
              "bench = importlib.util.module_from_spec(spec); spec.loader.exec_module(bench)\n"
              f"bench.__file__ = {str(fake)!r}\n"
              "sys.exit(bench.supervise([], 1, 2, 300))\n")
    sup = subprocess.Popen([sys.executable, "-c", driver])
    try:
        t0 = time.monotonic()
        while not pidfile.exists() or not pidfile.read_text():
            assert time.monotonic() - t0 < 60, "the body never started"
            time.sleep(0.1)
        pid = int(pidfile.read_text())
        os.kill(sup.pid, signal.SIGKILL)
        sup.wait(timeout=30)
        t0 = time.monotonic()
        while True:
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                break
            if time.monotonic() - t0 > 20:
                os.kill(pid, signal.SIGKILL)
                raise AssertionError("the body outlived its SIGKILLed supervisor")
            time.sleep(0.1)
    finally:
        if sup.poll() is None:
            sup.kill()
