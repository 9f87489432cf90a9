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
