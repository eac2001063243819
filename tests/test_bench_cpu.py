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
em = bench._Emitter(0, {deadline}, heartbeat_s=0.3)
if {with_line}:
    em.build = lambda: {{"metric": "m", "value": 1.0}}
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
    assert "running a slow leg" in err  # the heartbeat names the running leg


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
    """tools/bench_ab.with_copy_ceiling: a kernel of R bytes read from s_r buffers and W written
    to s_w is held to t >= R / read_GBs[s_r] + W / write_GBs[s_w]; entries without a byte mix,
    or a failed ceiling leg, pass through unchanged."""
    import sys as _sys

    _sys.path.insert(0, REPO)
    import bench
    from tools.bench_ab import with_copy_ceiling

    ceiling = {"GBs": 6000.0, "read_GBs": {1: 6800.0, 2: 6900.0, 3: 7000.0, 4: 7000.0},
               "write_GBs": {1: 6000.0, 2: 5800.0, 3: 5600.0, 4: 5500.0}}
    # dl_delta_pack_sgd on T125: 12 B/param read from 3 streams, 16 B/param written to 4
    P = 124_475_904
    e = bench.kernel_entry(28 * P, 0.6, read_bytes=12 * P, read_streams=3, write_bytes=16 * P,
                           write_streams=4)
    got = with_copy_ceiling(e, ceiling)
    t = 12 * P / 7000e9 + 16 * P / 5500e9
    assert abs(got["mix_ceiling"] - 28 * P / t / 1e9) < 0.1
    assert abs(got["frac_vs_mix"] - e["achieved"] / (28 * P / t / 1e9)) < 1e-3
    assert got["frac_vs_copy"] == round(e["achieved"] / 6000.0, 4)
    r = with_copy_ceiling(bench.kernel_entry(8 * P, 0.2, read_bytes=8 * P, read_streams=2,
                                             write_bytes=0, write_streams=1), ceiling)
    assert r["mix_ceiling"] == 6900.0  # a kernel that only reads is held to the read probe
    plain = bench.kernel_entry(8 * P, 0.2)
    assert "mix_ceiling" not in with_copy_ceiling(plain, ceiling)
    assert with_copy_ceiling(e, {"ok": False, "error": "x"}) == e


def _full_run_records(ws):
    """Every record a bench run at N = ws can produce, at its largest (long strings, error
    records, every leg and parity check present)."""
    import sys as _sys

    _sys.path.insert(0, REPO)
    import bench

    P, P13 = 124_475_904, 1_313_722_368
    roof = bench.kernel_entry(28 * P, 0.6, 3_493_349_683, kernel="dl_delta_pack_sgd",
                              timing="timed loop GPU span / K")
    head = {"tree": "t125", "params": P, "tensors": 148, "padded": P + 4096, "buckets": 2,
            "ms_per_step": 0.6, "value": 830.0, "value_aggregate": 830.0 * ws,
            "loop_gpu_ms_per_step": 0.6, "wire": "f32", "exchange": "sharded",
            "hbm_bytes_per_param": bench.dropin_bpp(ws, "sharded"), "roofline": roof,
            "cold": {"step_ms": 0.62, "value": 800.0, "note": "x" * 200}}
    rec = {"value": 700.0, "value_aggregate": 700.0 * ws, "ms_per_step": 7.5, "params": P13,
           "roofline": dict(roof, note="y" * 500), "kernels": {"a": roof, "b": roof},
           "hbm_bytes_per_param": 22.5, "variant": "z" * 300}
    names = ([f"t125_dropin_{e}" for e in ("replicated", "a2a")] +
             ["t125_engine", "t1.3b_dropin", "t1.3b_dropin_bf16", "t1.3b_int8", "t1.3b_dropin_int8",
              "t125_grad_sync", "t125_two_stages", "xgmi_link_probe", "t1.3b_xgmi_inner",
              "t125_dropin_synced", "dropin_pcie", "t1.3b_bf16"])
    legs = {n: dict(rec) for n in names}
    legs["peer_access_legs"] = {"ok": False, "error": "child exit timeout " + "e" * 400}
    par = {"ok": True, "err": 1.234567891e-7, "tol": 1e-6, "note": "n" * 300}
    parity = {n: dict(par) for n in ("f32", "bf16", "int8", "sharded", "a2a", "dropin_exchanges",
                                     "bf16_t1.3b", "xgmi")}
    cpu = {"value": 2.31, "unit": "GB/s", "cores": ws, "kind": "port", "sample": "s" * 600,
           "host": {"model": "AMD EPYC 9575F 64-Core Processor", "cpu_count": 256}}
    exch = {t: bench.exchange_efficiency(dict(rec, params=p), {"all_reduce": {"busbw_GBs": 300.0}},
                                         ws) for t, p in (("t125", P), ("t1.3b", P13))} if ws > 1 else {}
    meta = {"n_gpus": ws, "steps": 50, "warmup": 3, "workload": "w" * 600}
    return bench, meta, head, cpu, legs, parity, exch


import pytest  # noqa: E402


@pytest.mark.parametrize("ws", [1, 8])
def test_line_is_compact_with_every_leg_present(ws):
    """the stdout line stays <= 4 KB at N = 1 and N = 8 with every leg, parity
    check and exchange figure present (the driver parsed none of round 3's 32 KB line); the
    headline, its roofline and the CPU baseline are always in it."""
    bench, meta, head, cpu, legs, parity, exch = _full_run_records(ws)
    line = bench.assemble_line(meta, head, cpu, legs, parity, exch or None)
    text = json.dumps(line)
    assert len(text) <= bench.LINE_MAX_BYTES, len(text)
    d = json.loads(text)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype",
              "config", "roofline", "cpu_baseline", "value_cold"):
        assert k in d, k
    assert d["roofline"]["frac"] == head["roofline"]["frac"]
    assert d["roofline"]["traffic"] == 3_493_349_683
    assert d["cpu_baseline"]["cores"] == ws and d["cpu_baseline"]["value"] == 2.31
    assert all(set(v) <= {"GBs", "frac", "ms", "Bpp", "ok", "error"}
               for v in d["legs"].values())
    assert all(set(v) == {"ok", "err"} for v in d["parity"].values())
    if ws > 1:
        assert d["exchange_efficiency"]["t1.3b"]["rccl_allreduce_busbw_GBs"] == 300.0
        # the N > 1 line carries the parity the driver's SCALE run needs
        for k in ("f32", "dropin_exchanges"):
            assert d["parity"][k]["ok"] is True and d["parity"][k]["err"] < 1e-6, k
    # nothing had to be dropped for these records
    assert "legs_dropped_from_line" not in d


def test_committed_n8_rehearsal_line_carries_parity_and_exchange_efficiency():
    """The newest committed N = 8 rehearsal line (bench.py with eight ranks at its default
    deadline, profiles/r*_bench_n8_gloo_rehearsal.json) carries parity.f32,
    parity.dropin_exchanges (both ok) and exchange_efficiency -- the figures the driver's
    SCALE run reads -- within the 4 KB line bound."""
    import glob as _glob
    import sys as _sys

    _sys.path.insert(0, REPO)
    import bench

    paths = sorted(_glob.glob(os.path.join(REPO, "profiles", "r*_bench_n8_gloo_rehearsal.json")))
    assert paths
    with open(paths[-1]) as f:
        d = json.load(f)
    assert d["n_gpus"] == 8 and d["dtype"] == "f32"
    for k in ("f32", "dropin_exchanges"):
        assert d["parity"][k]["ok"] is True, k
    assert "t1.3b" in d["exchange_efficiency"]
    assert len(json.dumps(d)) <= bench.LINE_MAX_BYTES


def test_line_drops_side_legs_rather_than_grow():
    bench, meta, head, cpu, legs, parity, exch = _full_run_records(8)
    many = {f"leg_{i}_" + "x" * 60: v for i, v in enumerate(list(legs.values()) * 6)}
    line = bench.assemble_line(meta, head, cpu, many, parity, exch)
    assert len(json.dumps(line)) <= bench.LINE_MAX_BYTES
    assert line["legs_dropped_from_line"] > 0 and line["value"] == 830.0


def test_dropin_hbm_bytes_per_param():
    """The drop-in step's kernel bytes per parameter: one pass 28 at one
    peer; sharded 12 (pack) + 20/n (shard SGD) + 8 (scatter); replicated 12 + 24."""
    import sys as _sys

    _sys.path.insert(0, REPO)
    import bench

    assert bench.dropin_bpp(1, "sharded") == 28
    assert bench.dropin_bpp(8, "sharded") == 20 + 20 / 8
    assert bench.dropin_bpp(2, "replicated") == 36
    assert bench.dropin_bpp(8, "replicated", "bf16") == 32


_WIRING = r"""
import json, os, sys
sys.path.insert(0, {repo!r})
import torch, torch.distributed as dist
import bench
from diloco_amd import comm
comm.DP_BACKEND = "gloo"   # what setup_dist sets under DILOCO_BENCH_BACKEND=gloo
dist.init_process_group("gloo")   # setup_dist's default group at WORLD_SIZE > 1
dev = torch.device("cuda", 0)     # only a device object: new_group needs no GPU
g = bench.dp_group(dev)
t = torch.tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t, group=g)
rec = dict(default=dist.get_backend(), dp=dist.get_backend(g), dp_size=dist.get_world_size(g),
           distinct=g is not dist.group.WORLD, cached=bench.dp_group(dev) is g,
           one_comm=bench.training_comm() is bench.training_comm(),
           cpu_is_stage_group=bench.dp_group(torch.device("cpu"))
           is bench.training_comm().world.curr_stage_group, sum=t.item())
if dist.get_rank() == 0:
    print("REC" + json.dumps(rec), flush=True)
dist.barrier()
dist.destroy_process_group()
"""


def test_bench_dp_group_is_train_py_subgroup_over_gloo_default():
    """bench.py at N > 1 builds src/train.py's process groups: a gloo default group
    (src/world.py:32-33) and, for device tensors, DPSync's DP subgroup created over it
    (use_local_synchronization=True); one TrainingComm per run (src/train.py:291). Two CPU
    processes under torchrun with the DP backend set to gloo, as the one-box rehearsal does."""
    import socket
    import tempfile

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    path = os.path.join(tempfile.mkdtemp(prefix="dl_wiring_"), "w.py")
    with open(path, "w") as f:
        f.write(_WIRING.format(repo=REPO))
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), path], capture_output=True, text=True, timeout=170, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("REC")][0][3:])
    assert rec == dict(default="gloo", dp="gloo", dp_size=2, distinct=True, cached=True,
                       one_comm=True, cpu_is_stage_group=True, sum=3.0), rec
