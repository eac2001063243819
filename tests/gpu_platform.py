"""What the multi-process GPU tests record about the GPU they share: free HBM, the
KFD processes and user-mode queues on this box's GPU, and their queue-eviction time.

/sys/class/kfd/kfd/proc lists every process on the host that has the KFD device open, keyed
by host pid; each has a stats_<gpu_id> directory per GPU it uses, with evicted_ms (time its
queues spent evicted, counted in jiffies), and queues/<id>/type (0 compute, 1 SDMA, 4 SDMA
over xGMI). The box's GPU is ours alone, so every process with a stats entry for its gpu_id
(the topology node with SIMDs this container sees) is one of ours. Read-only; absent files
read as nothing."""
import glob
import os


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return ""


def our_gpu_ids():
    out = []
    for d in glob.glob("/sys/class/kfd/kfd/topology/nodes/*"):
        props = dict(ln.split(None, 1) for ln in _read(os.path.join(d, "properties")).splitlines()
                     if " " in ln)
        if int(props.get("simd_count", "0") or 0) > 0:
            out.append(_read(os.path.join(d, "gpu_id")))
    return [g for g in out if g]


def cp_queue_slots():
    """Hardware compute queue slots the KFD scheduler maps user queues to (num_cp_queues)."""
    for d in glob.glob("/sys/class/kfd/kfd/topology/nodes/*"):
        props = dict(ln.split(None, 1) for ln in _read(os.path.join(d, "properties")).splitlines()
                     if " " in ln)
        if int(props.get("simd_count", "0") or 0) > 0:
            return int(props.get("num_cp_queues", "0") or 0)
    return 0


def gpu_state():
    """{free_gb, procs (with the GPU open), procs_with_queues (in the scheduler's runlist),
    compute_queues, sdma_queues, evicted_ms, cp_queue_slots} for this box's GPU."""
    import torch

    gids = set(our_gpu_ids())
    procs = with_queues = cq = sq = ev = 0
    for d in glob.glob("/sys/class/kfd/kfd/proc/*"):
        mine = [g for g in gids if os.path.isdir(os.path.join(d, f"stats_{g}"))]
        if not mine:
            continue
        procs += 1
        with_queues += bool(glob.glob(os.path.join(d, "queues", "*")))
        for g in mine:
            try:
                ev += int(_read(os.path.join(d, f"stats_{g}", "evicted_ms")) or 0)
            except ValueError:
                pass
        for q in glob.glob(os.path.join(d, "queues", "*")):
            t = _read(os.path.join(q, "type"))
            cq += t == "0"
            sq += t in ("1", "4")
    free = torch.cuda.mem_get_info()[0] / 2**30 if torch.cuda.is_available() else 0.0
    return {"free_gb": round(free, 1), "procs": procs, "procs_with_queues": with_queues,
            "compute_queues": cq, "sdma_queues": sq,
            "evicted_ms": ev, "cp_queue_slots": cp_queue_slots()}
