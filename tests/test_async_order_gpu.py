"""The outer model's asynchronous exchange order, tested deterministically on one GPU.

Behind the reference's calls the fused outer model issues every bucket's collective from
sync_gradients without waiting (async_op=True) and OuterSGD.step waits bucket by bucket
(src/comm.py:120-123 restructured). The contract with a stream-ordered backend --
ProcessGroupNCCL's: the collective runs on its own stream after an event recorded on the
caller's stream, and Work.wait() makes the caller's stream wait for the collective's end --
is what RCCL at N > 1 relies on. On one GPU no real backend has all of it: RCCL refuses two
ranks on one device, and gloo, though it issues asynchronously and orders its staging copy
behind the caller's stream (tools/gloo_sync_probe.py: the issuing call returns in ~17 ms while
a 300 ms producer runs; that side is tested across two processes in
tests/test_dropin_gpu.py::test_collectives_behind_a_slow_producer), holds the host in
Work.wait() until the collective is done instead of ordering the stream only. So here a
second DP rank is
emulated in-process by a backend with exactly that stream contract and made deliberately
slow: each collective waits for the caller's stream, spins 150 ms on its own stream
(dl_spin), then adds rank 1's contribution -- rank 1's deltas, θ and momentum from the
reference's own two-rank fixture (tests/golden/micro_n2.npz) -- while a 150 ms spin also holds
the packs back on the caller's stream (a slow producer). Rank 0's θ, momentum, averaged .grad
and inner parameters must equal the fixture bit for bit, for the replicated exchange
(all_reduce) and the sharded one (reduce_scatter -> shard SGD -> all_gather of θ; momentum and
.grad gathered on read). Two controls break one side each and must come out wrong:
  no_wait          Work.wait() returns without ordering the caller's stream (consumer side)
  unordered_start  the collective does not wait for the caller's stream (producer side)"""
import numpy as np
import pytest
import torch

from conftest import load_npz, spin, split

pytestmark = pytest.mark.gpu
SLOW_MS = 150


class _Work:
    def __init__(self, ev, honour):
        self.ev, self.honour = ev, honour

    def wait(self):
        if self.honour:
            torch.cuda.current_stream().wait_event(self.ev)
        return True

    def is_completed(self):
        return self.ev.query()


class PeerEmulator:
    """torch.distributed as the mirror sees it, for a DP group of two whose rank 1 is emulated:
    every collective is stream-ordered and slow, and adds / fills rank 1's share."""

    def __init__(self, real, mirror, peer, mode="ordered"):
        self._real, self.m, self.peer, self.mode = real, mirror, peer, mode
        self.side = torch.cuda.Stream()
        self.calls = 0

    def __getattr__(self, name):  # ReduceOp, ProcessGroup, is_initialized, ...
        return getattr(self._real, name)

    def get_rank(self, group=None):
        return 0

    def get_world_size(self, group=None):
        return 2

    def _offset(self, t, arena):
        return (t.data_ptr() - arena.data_ptr()) // t.element_size()

    def _run(self, body):
        self.calls += 1
        ev_in = torch.cuda.Event()
        ev_in.record(torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            if self.mode != "unordered_start":
                self.side.wait_event(ev_in)
                spin(SLOW_MS)
            body()
            ev_out = torch.cuda.Event()
            ev_out.record(self.side)
        return _Work(ev_out, self.mode != "no_wait")

    def all_reduce(self, t, op=None, group=None, async_op=False):
        o = self._offset(t, self.m.d_wire)
        w = self._run(lambda: t.add_(self.peer["wire"][o:o + t.numel()]))
        return w if async_op else w.wait()

    def reduce_scatter_tensor(self, out, inp, op=None, group=None, async_op=False):
        # rank 0's half of the bucket: its own deltas (out is that half of inp) + rank 1's
        o = self._offset(out, self.m.d_wire)
        w = self._run(lambda: out.add_(self.peer["wire"][o:o + out.numel()]))
        return w if async_op else w.wait()

    def all_gather_into_tensor(self, out, inp, group=None, async_op=False):
        # rank 1's half: its values of the arena the output lies in
        for name, arena in (("theta", self.m.d_theta), ("mom", self.m.d_mom),
                            ("wsum", self.m.d_wire)):
            if arena is not None and arena.data_ptr() <= out.data_ptr() < (
                    arena.data_ptr() + arena.numel() * 4):
                break
        o = self._offset(out, arena)
        h = out.numel() // 2
        src = self.peer[name][o + h:o + out.numel()]
        w = self._run(lambda: out[h:].copy_(src))
        return w if async_op else w.wait()


def _packed(m, flat, numels):
    a = torch.zeros(m.tree.total, dtype=torch.float32, device="cuda:0")
    for o, x in zip(m.offs, split(flat, numels)):
        a[o:o + x.size] = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    return a


@pytest.mark.parametrize("exchange", ["replicated", "sharded"])
@pytest.mark.parametrize("mode", ["ordered", "no_wait", "unordered_start"])
def test_exchange_order_with_a_slow_stream_ordered_peer(exchange, mode, monkeypatch):
    from types import SimpleNamespace

    import torch.distributed as dist

    from diloco_amd import mirror as mirror_mod
    from diloco_amd import synth
    from diloco_amd.trees import get_tree
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)

    monkeypatch.setenv("DILOCO_OUTER_BUCKET_ELEMS", "4096")
    monkeypatch.setenv("WORLD_SIZE", "2")  # buckets planned to split two ways
    g = load_npz("micro_n2.npz")
    spec = get_tree("micro")
    numels = spec.numels()
    shapes = [s for _, s in spec.params()]
    theta0 = synth.outer_tree(numels, spec.init_spec())
    inner = torch.nn.Module()
    inner.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.from_numpy(v.copy()).view(s))
                                       for v, s in zip(theta0, shapes)]).to("cuda:0")
    outer = get_outer_model(inner, "device", exchange=exchange)
    opt = get_optimizer(outer, SimpleNamespace(type="SGD", lr=0.7, momentum=0.9, nesterov=True))
    m = outer._diloco_mirror
    assert m.tree.n_buckets > 2
    emu = PeerEmulator(dist, m, {}, mode)
    monkeypatch.setattr(mirror_mod, "dist", emu)
    ok = True
    for s in (1, 2):
        prev = [p.detach().cpu().numpy().reshape(-1).copy() for p in outer.parameters()]
        with torch.no_grad():
            for p, v in zip(inner.parameters(), synth.inner_tree(prev, s, 0)):
                p.copy_(torch.from_numpy(v).view(p.shape))
        # rank 1 of the reference's two-rank run: its delta, and its θ / momentum after the step
        emu.peer.update(wire=_packed(m, g[f"delta_s{s}_rlast"], numels),
                        wsum=_packed(m, 2 * g[f"avg_s{s}"], numels),  # Σ = 2·avg exactly
                        theta=_packed(m, g[f"theta_s{s}"], numels),
                        mom=_packed(m, g[f"buf_s{s}"], numels))
        compute_pseudo_gradient(inner, outer)
        spin(SLOW_MS)  # a slow producer: every bucket's pack waits behind it
        m.all_reduce(None, 2)  # what TrainingComm.sync_gradients makes at two peers
        assert m._works is not None and len(m._works) == m.tree.n_buckets
        opt.step()
        sync_inner_model(outer, inner)
        got = {k: np.concatenate([t.detach().cpu().numpy().reshape(-1) for t in ts]) for k, ts in (
            ("theta", list(outer.parameters())), ("inner", list(inner.parameters())),
            ("buf", [opt.state[p]["momentum_buffer"] for p in outer.parameters()]),
            ("avg", [p.grad for p in outer.parameters()]))}
        want = {"theta": g[f"theta_s{s}"], "inner": g[f"theta_s{s}"], "buf": g[f"buf_s{s}"],
                "avg": g[f"avg_s{s}"]}
        ok &= all(got[k].tobytes() == want[k].tobytes() for k in want)
        torch.cuda.synchronize()
    assert emu.calls >= 2 * m.tree.n_buckets
    assert ok == (mode == "ordered"), (exchange, mode)
