"""bench.py's run-bounding machinery on the CPU: the watchdog prints the line assembled so far
(marked incomplete) and leaves with status 0, a finished run prints exactly one line, and a
run with no headline yet leaves with a non-zero status and prints nothing."""
import json
import os
import subprocess
import sys

from conftest import REPO

SNIPPET = r"""
import sys, time
sys.path.insert(0, {repo!r})
import bench
em = bench._Emitter(0, {deadline})
if {with_line}:
    em.line = {{"metric": "m", "value": 1.0}}
em.running = "a slow leg"
if {finish}:
    em.emit()
    em.emit()  # a second emit (e.g. the watchdog racing the end) prints nothing
    em.timer.cancel()
    sys.exit(0)
time.sleep(30)
"""


def _run(deadline, with_line, finish):
    code = SNIPPET.format(repo=REPO, deadline=deadline, with_line=with_line, finish=finish)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"))
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, lines, p.stderr


def test_watchdog_prints_partial_line_and_exits_cleanly():
    rc, lines, err = _run(1.0, True, False)
    assert rc == 0, err
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] == 1.0 and d["incomplete"]["leg"] == "a slow leg"
    assert "watchdog" in err


def test_finished_run_prints_one_line():
    rc, lines, _ = _run(60.0, True, True)
    assert rc == 0 and len(lines) == 1 and "incomplete" not in json.loads(lines[0])


def test_watchdog_before_headline_fails_the_run():
    rc, lines, _ = _run(1.0, False, False)
    assert rc != 0 and lines == []


def test_cpu_baseline_with_two_gloo_processes():
    """The N > 1 CPU baseline (bench.cpu_baseline_dist): two CPU processes under gloo (GPUs
    hidden, as bench's child legs run it) step the reference's per-tensor sequence with its
    per-tensor all_reduce on the tiny tree; rank 0 writes one record with cores = 2."""
    import socket
    import tempfile

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = os.path.join(tempfile.mkdtemp(prefix="dl_cpub_"), "cb.json")
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), os.path.join(REPO, "bench.py"), "--gpus", "2", "--tree",
                        "tiny", "--child-legs", "cpu_baseline", "--child-out", out,
                        "--deadline", "100"], capture_output=True, text=True, timeout=170,
                       env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    with open(out) as f:
        r = json.load(f)
    assert r["cores"] == 2 and r["kind"] == "port" and r["value"] > 0
    assert "2 CPU processes" in r["sample"]
