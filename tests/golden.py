"""Shared helpers of the golden-fixture tests (fixture: scripts/make_golden.py)."""
import os
from argparse import Namespace

import numpy as np
import torch
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "golden_demo_frames.npz")
FRAMES = ["frame_0016.png", "frame_0017.png", "frame_0018.png"]


def fixture():
    return np.load(FIXTURE, allow_pickle=False)


def frames():
    """The reference's demo frames (436x1024), read with PIL as demo.py:20-23 does."""
    out = []
    for f in FRAMES:
        img = np.array(Image.open(os.path.join(ROOT, "demo-frames", f))).astype(np.uint8)
        out.append(torch.from_numpy(img).permute(2, 0, 1).float()[None])
    return out


def model(small: bool, fix, **kw):
    """Seed-0 random-init RAFT: the weights the fixture was computed with (checked by checksum)."""
    from raft_ros_amd.models import RAFT

    torch.manual_seed(0)
    m = RAFT(Namespace(small=small, **kw))
    name = "small" if small else "base"
    for k, v in m.state_dict().items():
        if v.dtype.is_floating_point:
            want = float(fix[f"{name}/ck/{k}"])
            got = float((v.double() ** 2).sum())
            assert abs(got - want) <= 1e-9 * max(abs(want), 1.0), (k, got, want)
    return m.eval()


def run(m, dev, fix, pair: int, **kw):
    """-> (flow_low, flow_up subsampled like the fixture) of one frame pair, demo.py-style."""
    from raft_ros_amd.utils.utils import InputPadder

    fr = frames()
    i1, i2 = fr[pair].to(dev), fr[pair + 1].to(dev)
    a, b = InputPadder(i1.shape).pad(i1, i2)
    with torch.no_grad():
        lo, up = m(a, b, iters=int(fix["iters"]), test_mode=True)
    s = int(fix["sub"])
    return lo.float().cpu(), up[:, :, ::s, ::s].float().cpu()


def epe(a, b) -> float:
    return float((torch.as_tensor(a) - torch.as_tensor(b)).norm(dim=1).mean())


# ------------------------------------------------------------------ training-gradient golden
GRAD_FIXTURE = os.path.join(ROOT, "tests", "fixtures", "golden_grads.npz")


def grad_fixture():
    return np.load(GRAD_FIXTURE, allow_pickle=False)


def grad_step(m, dev, **fwd):
    """One training step's loss + per-parameter fp32 gradients on the fixture batch
    (scripts/make_golden_grads.py: demo-frame crops, synthetic GT, reference sequence loss)."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from make_golden_grads import ITERS, batch

    from raft_ros_amd.train.loss import sequence_loss

    i1, i2, flow, valid = (t.to(dev) for t in batch())
    m.zero_grad(set_to_none=True)
    preds = m(i1, i2, iters=ITERS, **fwd)
    loss, _ = sequence_loss(preds, flow, valid, gamma=0.8)
    loss.backward()
    grads = {n: p.grad.detach().double().cpu().reshape(-1) for n, p in m.named_parameters() if p.grad is not None}
    return float(loss), preds[-1].detach().float().cpu(), grads


def grad_errors(grads, fix, name):
    """-> {param: relative error vs the reference gradient} (full tensor or its 16 fixed
    projections); parameters whose reference gradient is ~0 (conv biases in front of a norm)
    report their absolute norm relative to the whole gradient instead."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from make_golden_grads import projections

    total = float(np.sqrt(sum(float(fix[k]) ** 2 for k in fix.files if k.startswith(f"{name}/gnorm/"))))
    errs = {}
    for k in fix.files:
        if not k.startswith(f"{name}/gnorm/"):
            continue
        pn = k[len(f"{name}/gnorm/"):]
        g = grads.get(pn)
        assert g is not None, f"no gradient for {pn}"
        gn = float(fix[k])
        if gn < 1e-6 * total:
            errs[pn] = float(g.norm()) / total
            continue
        if f"{name}/gfull/{pn}" in fix.files:
            ref = torch.from_numpy(fix[f"{name}/gfull/{pn}"])
            errs[pn] = float((g - ref).norm() / ref.norm())
        else:
            ref = torch.from_numpy(fix[f"{name}/gproj/{pn}"])
            errs[pn] = float((projections(pn, g.numel()) @ g - ref).norm() / ref.norm())
    return errs
