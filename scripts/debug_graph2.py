"""Debug helper: which forward piece changes between HIP-graph replays."""
import sys
from argparse import Namespace

import torch

sys.path.insert(0, ".")
from raft_ros_amd.data.synthetic import synthetic_batch  # noqa: E402
from raft_ros_amd.models import RAFT  # noqa: E402
from raft_ros_amd.ops.norm import InstanceNorm2dNHWC  # noqa: E402

dev = torch.device("cuda", 0)
if "det" in sys.argv:
    torch.backends.cudnn.deterministic = True
torch.manual_seed(0)
m = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16")).to(dev).to(
    memory_format=torch.channels_last).train()
i1, i2, flow, valid = synthetic_batch(2, 128, 160, seed=0, device=dev)
x = (2 * (i1 / 255.0) - 1.0).contiguous(memory_format=torch.channels_last)
xb = torch.randn(4, 64, 64, 80, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
inorm = InstanceNorm2dNHWC(64)


def fnet():
    with torch.autocast("cuda", torch.bfloat16, cache_enabled=False):
        return m.fnet([x, x])[0]


def cnet():
    with torch.autocast("cuda", torch.bfloat16, cache_enabled=False):
        return m.cnet(x)


def inorm_only():
    return inorm(xb, relu=True)


def full():
    return m(i1, i2, iters=2)[-1]


def inorm_bwd():
    y = inorm(xb.detach().requires_grad_(True), relu=True)
    gx, = torch.autograd.grad(y, [y], torch.ones_like(y))
    return gx


def fnet_bwd():
    xr = x.detach().clone().requires_grad_(True)
    with torch.autocast("cuda", torch.bfloat16, cache_enabled=False):
        y = m.fnet([xr, xr])[0]
    g, = torch.autograd.grad(y.float().square().sum(), [xr])
    return g


from raft_ros_amd.ops import CorrPyramid  # noqa: E402
from raft_ros_amd.train.loss import sequence_loss  # noqa: E402

F1 = torch.randn(2, 256, 16, 20, device=dev)
F2 = torch.randn(2, 256, 16, 20, device=dev)
CO = torch.rand(2, 2, 16, 20, device=dev) * 16
WO = torch.randn(2, 16, 20, 328, device=dev)


def corr_bwd():
    f1 = F1.clone().requires_grad_(True)
    f2 = F2.clone().requires_grad_(True)
    c = CorrPyramid(f1, f2)
    loss = sum((c.lookup_padded(CO + k, 328).float() * WO).sum() for k in range(3))
    g1, g2 = torch.autograd.grad(loss, [f1, f2])
    return torch.cat([g1.flatten(), g2.flatten()])


PARAMS = [p for n, p in m.named_parameters()]


def full_bwd():
    loss, _ = sequence_loss(m(i1, i2, iters=2), flow, valid)
    gs = torch.autograd.grad(loss, PARAMS)
    return torch.cat([g.flatten() for g in gs])


def upd_bwd():
    gs = []
    for n, p in m.named_parameters():
        pass
    loss, _ = sequence_loss(m(i1, i2, iters=2), flow, valid)
    ps = [p for n, p in m.named_parameters() if n.startswith("update_block")]
    return torch.cat([g.flatten() for g in torch.autograd.grad(loss, ps)])


def cnet_bwd():
    xr = x.detach().clone().requires_grad_(True)
    with torch.autocast("cuda", torch.bfloat16, cache_enabled=False):
        y = m.cnet(xr)
    g, = torch.autograd.grad(y.float().square().sum(), [xr])
    return g


def sub_bwd(prefix):
    def fn():
        loss, _ = sequence_loss(m(i1, i2, iters=2), flow, valid)
        ps = [p for n, p in m.named_parameters() if n.startswith(prefix)]
        return torch.cat([g.flatten() for g in torch.autograd.grad(loss, ps)])
    return fn


def fnet_w_bwd():
    with torch.autocast("cuda", torch.bfloat16, cache_enabled=False):
        y = m.fnet([x, x])[0]
    ps = [p for n, p in m.fnet.named_parameters()]
    return torch.cat([g.flatten() for g in torch.autograd.grad(y.float().square().sum(), ps)])


PERSIST = {"i1": i1, "i2": i2, "flow": flow, "valid": valid, "x": x, "xb": xb,
           **{n: p for n, p in m.named_parameters()}, **{n: b for n, b in m.named_buffers()}}
snap = {k: v.detach().clone() for k, v in PERSIST.items()}


def changed():
    return [k for k, v in PERSIST.items() if not torch.equal(v, snap[k]) and "running" not in k and "num_batches" not in k]


for name, fn in [("cnet.conv2", sub_bwd("cnet.conv2")), ("cnet.layer3.1", sub_bwd("cnet.layer3.1")),
                 ("cnet.layer3.0", sub_bwd("cnet.layer3.0")), ("cnet.layer1", sub_bwd("cnet.layer1")),
                 ("fnet.conv2", sub_bwd("fnet.conv2")), ("fnet.layer3", sub_bwd("fnet.layer3")),
                 ("fnet.layer1", sub_bwd("fnet.layer1"))]:
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ref = fn().detach().clone()
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        out = fn()
    errs = []
    for i in range(3):
        g.replay()
        torch.cuda.synchronize()
        errs.append(float((out.float() - ref.float()).abs().max()))
    errs.append(bool(torch.isfinite(out).all()))
    print(f"{name:10s} ref max {float(ref.float().abs().max()):.3e} replay errs {errs}", flush=True)
    del g
print("done")
