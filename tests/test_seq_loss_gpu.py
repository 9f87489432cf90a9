"""Fused HIP sequence loss (raft_ros_amd/csrc/seq_loss.hip) vs the plain PyTorch
fp32 formulation of reference train.py:47-72."""
import pytest
import torch

from raft_ros_amd.train import loss as L


def _torch_loss(preds, gt, valid, gamma=0.8, max_flow=400.0):
    n = len(preds)
    mag = torch.sum(gt ** 2, dim=1).sqrt()
    v = (valid >= 0.5) & (mag < max_flow)
    loss = 0.0
    for i, p in enumerate(preds):
        loss = loss + gamma ** (n - i - 1) * (v[:, None] * (p - gt).abs()).mean()
    epe = torch.sum((preds[-1] - gt) ** 2, dim=1).sqrt()[v]
    return loss, {"epe": epe.mean(), "1px": (epe < 1).float().mean(), "3px": (epe < 3).float().mean(),
                  "5px": (epe < 5).float().mean()}


@pytest.mark.gpu
@pytest.mark.parametrize("n,B,H,W", [(12, 2, 64, 96), (3, 1, 40, 56)])
def test_fused_sequence_loss_matches_torch(n, B, H, W):
    from raft_ros_amd.ops import _ext

    assert _ext.is_loaded(), _ext.load_error()
    torch.manual_seed(0)
    dev = torch.device("cuda")
    gt = torch.randn(B, 2, H, W, device=dev) * 5
    gt[0, :, :4] = 500.0  # some |gt| >= max_flow pixels
    valid = (torch.rand(B, H, W, device=dev) > 0.2).float()
    base = [gt + torch.randn_like(gt) * (3.0 / (i + 1)) for i in range(n)]
    preds = [b.clone().requires_grad_(True) for b in base]
    preds_ref = [b.clone().requires_grad_(True) for b in base]

    assert L._fused_ok(preds, gt)
    loss, m = L.sequence_loss(preds, gt, valid)
    loss.backward()
    loss_r, m_r = _torch_loss(preds_ref, gt, valid)
    loss_r.backward()

    torch.testing.assert_close(loss, loss_r, rtol=1e-5, atol=1e-5)
    for k in m_r:
        torch.testing.assert_close(m[k], m_r[k], rtol=1e-5, atol=1e-5)
    for p, r in zip(preds, preds_ref):
        torch.testing.assert_close(p.grad, r.grad, rtol=1e-6, atol=1e-9)
