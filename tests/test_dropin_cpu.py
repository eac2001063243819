"""The drop-in surface on host tensors (the reference's --device cpu runs,
tests/test_memorize.py:35-39 of the reference): the Serializer frames CPU tensors like
src/serializer.py:11-15, and the pipeline threads surface their failures to the caller
instead of dying silently (src/comm.py:33-38,64-69 would leave the peer blocked)."""
import time

import pytest
import torch

from conftest import load_json
from diloco_amd.comm import RecvThread, SendThread, ThreadStopped
from diloco_amd.serializer import Serializer


def test_serializer_host_tensors_match_reference_fixture():
    for case in load_json("serializer.json"):
        dtype = getattr(torch, case["dtype"])
        x = torch.tensor(case["x"], dtype=torch.float32).to(dtype).view(case["shape"])
        s = Serializer(tuple(case["shape"]))
        assert list(s.shape) == case["serializer_shape"]
        y = s.serialize(x, tuple(case["meta"]))
        assert y.device.type == "cpu"
        assert list(y.shape) == case["out_shape"]
        assert str(y.dtype).split(".")[-1] == case["out_dtype"]
        assert y[0].flatten()[:2].tolist() == case["meta_plane"]
        assert y[1].flatten().tolist() == case["payload"]
        t, m = s.deserialize(y)
        assert list(t.shape) == case["deser_shape"] and list(m) == case["deser_meta"]
        assert torch.equal(t, y[1])


def test_serializer_host_promotion_autograd_and_errors():
    """torch.cat's promotion of the fp32 metadata plane (fp64 payload -> fp64 frame), the
    payload's autograd graph kept, and the reference's IndexError for < 2 elements."""
    x = torch.randn(3, 4, dtype=torch.float64, requires_grad=True)
    y = Serializer((3, 4)).serialize(x, (2, 9))
    assert y.dtype == torch.float64 and y.requires_grad
    assert y[0].flatten()[:2].tolist() == [2.0, 9.0] and torch.equal(y[1], x)
    y[1].sum().backward()
    assert torch.equal(x.grad, torch.ones_like(x))
    with pytest.raises(IndexError):
        Serializer((1,)).serialize(torch.ones(1), (0, 1))


# the dying thread re-raises (its traceback reaches threading.excepthook / stderr)
quiet_thread = pytest.mark.filterwarnings("ignore::pytest.PytestUnhandledThreadExceptionWarning")


@quiet_thread
def test_send_thread_failure_is_raised_to_the_caller():
    t = SendThread((1,), group=None)
    t.send(0, torch.ones(1), (0, 0))  # framing a 1-element tensor fails inside the thread
    deadline = time.time() + 10
    while t.error is None and time.time() < deadline:
        time.sleep(0.01)
    assert isinstance(t.error, IndexError)
    with pytest.raises(ThreadStopped) as e:
        t.send(0, torch.ones(4), (0, 0))
    assert isinstance(e.value.__cause__, IndexError)
    t.thread.join(10)  # its excepthook warning lands in this test, not a later one


@quiet_thread
def test_recv_thread_failure_wakes_a_blocked_receive():
    # no process group: dist.recv raises inside the thread
    t = RecvThread((2, 2), group=None)
    with pytest.raises(ThreadStopped):
        t.receive()
    t.thread.join(10)
    assert t.can_receive  # a training loop polling can_receive gets to the raise too
    with pytest.raises(ThreadStopped):
        t.receive()


@pytest.mark.parametrize("placement", ["host", "device"])
def test_parameterless_model_is_the_references_no_op(placement):
    """A model without parameters: compute_pseudo_gradient and sync_inner_model are the
    reference's loops over nothing (src/utils.py:218-226), and get_optimizer raises torch's own
    error for an empty parameter list, as torch.optim.SGD does there (src/utils.py:62-63)."""
    from types import SimpleNamespace

    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)

    inner = torch.nn.Sequential(torch.nn.ReLU())
    outer = get_outer_model(inner, placement)
    assert list(outer.parameters()) == []
    compute_pseudo_gradient(inner, outer)
    sync_inner_model(outer, inner)
    cfg = SimpleNamespace(type="SGD", lr=0.7, momentum=0.9, nesterov=True)
    with pytest.raises(ValueError) as ours:
        get_optimizer(outer, cfg)
    with pytest.raises(ValueError) as theirs:
        torch.optim.SGD(inner.parameters(), lr=0.7, momentum=0.9, nesterov=True)
    assert str(ours.value) == str(theirs.value)
