"""Which GPU the outer step and the device p2p transport use when nobody set the current
device. The reference picks cuda:local_rank without calling
torch.cuda.set_device (src/utils.py:36-40, src/train.py:368) and builds the outer model while
the inner one is still on the CPU (src/train.py:382; the inner model moves at :163). So
get_outer_model(..., placement="device") on a CPU inner model must not place the outer model
on torch.cuda.current_device() -- cuda:0 on every rank of a node -- but wait for the inner
model's device, and TrainingComm(transport="device") defaults to cuda:local_rank. CPU-only:
the GPU steps are faked at the seams (the mirror class); the real path
runs in tests/test_dropin_gpu.py (_outer_steps, placement="device")."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist

from diloco_amd import utils
from diloco_amd.utils import compute_pseudo_gradient, get_optimizer, get_outer_model


class _Cfg:
    def __init__(self, **kw):
        self.__dict__.update(kw)


@pytest.fixture
def current_device_calls(monkeypatch):
    calls = []
    monkeypatch.setattr(torch.cuda, "current_device", lambda: calls.append(0) or 0)
    return calls


def test_device_outer_model_takes_the_inner_models_device(monkeypatch, current_device_calls):
    inner = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.Linear(3, 2))
    outer = get_outer_model(inner, "device")  # src/train.py:382: the inner model is on the CPU
    assert not utils.has_mirror(outer)
    assert all(p.device.type == "cpu" for p in outer.parameters())
    opt = get_optimizer(outer, _Cfg(type="SGD", lr=0.7, momentum=0.9, nesterov=True))
    made = {}

    class RecordingMirror:  # stands in for DeviceOuterMirror: records where it was built
        def __init__(self, model, device, kernels=None, bucket_cap_elems=0, fused=False,
                     wire="f32", exchange="sharded", keep_params=False):
            made.update(device=torch.device(device), keep=keep_params,
                        params=list(model.parameters()))

        def pseudo_gradient(self, inner_params):
            made["delta"] = len(list(inner_params))

    cuda3 = torch.device("cuda", 3)
    monkeypatch.setattr(utils, "DeviceOuterMirror", RecordingMirror)
    # the inner model has moved to cuda:3 (src/train.py:163 with local_rank 3)
    monkeypatch.setattr(utils, "_inner_device", lambda model: cuda3)
    monkeypatch.setattr(utils, "device_path", lambda t: True)
    compute_pseudo_gradient(inner, outer)
    assert made["device"] == cuda3
    # no whole-model device copy first: the mirror gets the CPU parameters
    assert all(p.device.type == "cpu" for p in made["params"])
    assert made["keep"]  # the optimizer's Parameter objects stay the outer model's
    assert all(a is b for a, b in zip(made["params"], opt.param_groups[0]["params"]))
    assert made["delta"] == 4
    assert not current_device_calls


def test_device_outer_model_on_a_cpu_inner_model_runs_the_reference_loops(
        current_device_calls):
    """Until the inner model reaches a GPU the four calls are the reference's host loops."""
    torch.manual_seed(0)
    inner = torch.nn.Linear(5, 4)
    outer = get_outer_model(inner, "device")
    opt = get_optimizer(outer, _Cfg(type="SGD", lr=0.7, momentum=0.9, nesterov=True))
    ref = torch.nn.Linear(5, 4)
    ref.load_state_dict(outer.state_dict())
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.7, momentum=0.9, nesterov=True)
    with torch.no_grad():
        for p in inner.parameters():
            p.add_(0.01)
    compute_pseudo_gradient(inner, outer)
    for po, pr, pi in zip(outer.parameters(), ref.parameters(), inner.parameters()):
        pr.grad = pr.data - pi.data
        assert torch.equal(po.grad, pr.grad)
    opt.step()
    ref_opt.step()
    utils.sync_inner_model(outer, inner)
    for po, pr, pi in zip(outer.parameters(), ref.parameters(), inner.parameters()):
        assert torch.equal(po, pr) and torch.equal(pi, pr)
    assert not utils.has_mirror(outer) and not current_device_calls


def test_device_p2p_transport_defaults_to_cuda_local_rank(monkeypatch, current_device_calls):
    from diloco_amd.comm import TrainingComm
    from diloco_amd.world import World

    monkeypatch.setenv("LOCAL_RANK", "3")
    dist.init_process_group("gloo", init_method="file://" + tempfile.mktemp(prefix="dl_pg_"),
                            rank=0, world_size=1)
    try:
        comm = TrainingComm(World.from_default_group(1), (2, 4, 8), None, transport="device")
        for t in (comm.forward_send_thread, comm.forward_recv_thread,
                  comm.backward_send_thread, comm.backward_recv_thread):
            assert t.device == torch.device("cuda", 3)
    finally:
        dist.destroy_process_group()
    assert not current_device_calls
    assert os.environ["LOCAL_RANK"] == "3"
