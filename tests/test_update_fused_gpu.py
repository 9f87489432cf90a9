"""Fused HIP update block vs the PyTorch (MIOpen) update block: forward flows and all gradients."""
from argparse import Namespace

import pytest
import torch

from raft_ros_amd.models import RAFT

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("shape", [(2, 128, 192), (1, 136, 200)])
def test_fused_update_matches_torch_path(cuda, shape):
    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.train.loss import sequence_loss

    B, H, W = shape
    torch.manual_seed(0)
    ref = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16", fused_update=False)).to(cuda)
    fused = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16", fused_update=True)).to(cuda)
    fused.load_state_dict(ref.state_dict())
    ref.train(); fused.train()
    ref.freeze_bn(); fused.freeze_bn()  # identical BN statistics in both runs
    i1, i2, flow, valid = synthetic_batch(B, H, W, max_disp=6, seed=1, device=cuda)
    outs = {}
    for name, m in (("ref", ref), ("fused", fused)):
        m.zero_grad()
        preds = m(i1, i2, iters=3)
        loss, _ = sequence_loss(preds, flow, valid)
        loss.backward()
        outs[name] = (preds, {n: p.grad for n, p in m.named_parameters() if p.grad is not None})
    (pr, gr), (pf, gf) = outs["ref"], outs["fused"]
    for a, b in zip(pf, pr):
        assert _rel(a, b) < 3e-2, _rel(a, b)
    assert set(gf) == set(gr), set(gr) ^ set(gf)
    # parameters whose true gradient vanishes (biases feeding InstanceNorm) are pure noise:
    # compare every tensor against the norm of its module group's gradient instead
    groups = {}
    for n in gr:
        groups.setdefault(n.split(".")[0], []).append(n)
    bad = {}
    # conv biases directly followed by InstanceNorm have an identically-zero true gradient
    noise = {n for n in gr if n.startswith("fnet.") and n.endswith(".bias") and not n.startswith("fnet.conv2")}
    for grp, names in groups.items():
        names = [n for n in names if n not in noise]
        if not names:
            continue
        scale = max(torch.stack([gr[n].float().norm() for n in names]).max().item(), 1e-12)
        for n in names:
            err = (gf[n].float() - gr[n].float()).norm().item()
            # encoder grads pass through the bf16 corr GEMM backward and 10+ bf16 layers in both
            # paths; the update block itself is held to 10 %
            tol = 0.1 if grp == "update_block" else 0.25
            if err > tol * max(gr[n].float().norm().item(), 1e-2 * scale):
                bad[n] = (err, gr[n].float().norm().item())
    assert not bad, bad
