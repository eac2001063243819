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


def test_mix_ceiling_reads_each_half_against_its_own_probe():
    """bench.with_copy_ceiling: a kernel of R bytes read from s_r buffers and W written to s_w
    is held to t >= R / read_GBs[s_r] + W / write_GBs[s_w]; entries without a byte mix, or a
    failed ceiling leg, pass through unchanged."""
    import sys as _sys

    _sys.path.insert(0, REPO)
    import bench

    ceiling = {"GBs": 6000.0, "read_GBs": {1: 6800.0, 2: 6900.0, 3: 7000.0, 4: 7000.0},
               "write_GBs": {1: 6000.0, 2: 5800.0, 3: 5600.0, 4: 5500.0}}
    # dl_delta_pack_sgd on T125: 12 B/param read from 3 streams, 16 B/param written to 4
    P = 124_475_904
    e = bench.kernel_entry(28 * P, 0.6, rw=(12 * P, 3, 16 * P, 4))
    got = bench.with_copy_ceiling(e, ceiling)
    t = 12 * P / 7000e9 + 16 * P / 5500e9
    assert abs(got["mix_ceiling"] - 28 * P / t / 1e9) < 0.1
    assert abs(got["frac_vs_mix"] - e["achieved"] / (28 * P / t / 1e9)) < 1e-3
    assert got["frac_vs_copy"] == round(e["achieved"] / 6000.0, 4)
    # a kernel that only reads (W = 0) is held to the read probe alone
    r = bench.with_copy_ceiling(bench.kernel_entry(8 * P, 0.2, rw=(8 * P, 2, 0, 1)), ceiling)
    assert r["mix_ceiling"] == 6900.0
    plain = bench.kernel_entry(8 * P, 0.2)
    assert "mix_ceiling" not in bench.with_copy_ceiling(plain, ceiling)
    assert bench.with_copy_ceiling(e, {"ok": False, "error": "x"}) == e
