import sys, torch
sys.path[:0]=["diloco-swarm_amd","tests","."]
from diloco_amd.utils import get_outer_model, get_optimizer, outer_mirror, compute_pseudo_gradient
from diloco_amd.mirror import _DATA
class C:
    def __init__(s, **k): s.__dict__.update(k)
inner = torch.nn.Module()
inner.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(n)) for n in (37005, 5, 0, 4097)])
outer = get_outer_model(inner, "device", exchange="sharded")
inner = inner.to("cuda:0")
opt = get_optimizer(outer, C(type="SGD", lr=0.7, momentum=0.9, nesterov=True))
print("before", [p.device for p in outer.parameters()], flush=True)
m = outer_mirror(outer, torch.device("cuda:0"))
print("after mirror", [p.device for p in outer.parameters()], [type(p).__name__ for p in outer.parameters()], flush=True)
print("m.params", [p.device for p in m.params], [id(p) for p in m.params] == [id(p) for p in outer.parameters()], flush=True)
compute_pseudo_gradient(inner, outer)
print("ok", flush=True)
