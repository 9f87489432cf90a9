"""The native clip + AdamW step (ops/optim.py ClipAdamW, csrc/optim.hip) against torch's
clip_grad_norm_ + AdamW in fp32 (reference train.py:75-86, 154-157)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _params(cuda, n=150):
    g = torch.Generator(device="cpu").manual_seed(0)
    shapes = [(64, 3, 7, 7), (257,), (16385,), (40000,), (3, 5)] + [(17 + i % 9, 13) for i in range(n - 5)]
    ps = []
    for i, s in enumerate(shapes):
        t = torch.randn(s, generator=g)
        if len(s) == 4:
            t = t.contiguous(memory_format=torch.channels_last)
        ps.append(torch.nn.Parameter(t.to(cuda)))
    return ps


def _grads(ps, step, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(100 + step)
    return [(scale * torch.randn(p.shape, generator=g)).to(p.device).contiguous(
        memory_format=torch.channels_last if p.dim() == 4 else torch.contiguous_format) for p in ps]


@pytest.mark.parametrize("max_norm", [1.0, 0.0])
def test_clip_adamw_matches_torch(cuda, max_norm):
    from raft_ros_amd.ops.optim import ClipAdamW

    a = _params(cuda)
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    opt = ClipAdamW(a, lr=4e-4, eps=1e-8, weight_decay=1e-4, max_norm=max_norm)
    ref = torch.optim.AdamW(b, lr=4e-4, eps=1e-8, weight_decay=1e-4)
    skipped = torch.zeros((), device=cuda)
    for step in range(4):
        lr = 4e-4 * (1 + step)  # a schedule writes param_groups[0]["lr"] between steps
        opt.param_groups[0]["lr"] = lr
        ref.param_groups[0]["lr"] = lr
        gs = _grads(a, step, scale=0.05 if step % 2 else 3.0)  # clipped and unclipped steps
        for p, q, g in zip(a, b, gs):
            p.grad = g.clone()
            q.grad = g.clone()
        norm = opt.step(skipped=skipped)
        if max_norm > 0:
            rn = torch.nn.utils.clip_grad_norm_(b, max_norm)
            torch.testing.assert_close(norm, rn, rtol=1e-5, atol=0)
        ref.step()
        for p, q in zip(a, b):
            assert p.stride() == q.stride()
            torch.testing.assert_close(p, q, rtol=2e-5, atol=2e-7)
    assert skipped.item() == 0
    # the state dict is torch AdamW's: load it into a fresh torch AdamW and both continue alike
    sd = opt.state_dict()
    st0 = sd["state"][0]
    assert set(st0) == {"step", "exp_avg", "exp_avg_sq"} and float(st0["step"]) == 4.0
    torch.testing.assert_close(st0["exp_avg"], ref.state_dict()["state"][0]["exp_avg"], rtol=2e-5, atol=1e-6)


def test_clip_adamw_skips_non_finite_and_resumes(cuda):
    from raft_ros_amd.ops.optim import ClipAdamW

    a = _params(cuda, n=8)
    opt = ClipAdamW(a, lr=1e-3, weight_decay=1e-4, max_norm=1.0)
    skipped = torch.zeros((), device=cuda)
    for p, g in zip(a, _grads(a, 0)):
        p.grad = g
    opt.step(skipped=skipped)
    before = [p.detach().clone() for p in a]
    gs = _grads(a, 1)
    gs[3][0] = float("inf")
    for p, g in zip(a, gs):
        p.grad = g
    norm = opt.step(skipped=skipped)
    assert not torch.isfinite(norm) and skipped.item() == 1
    for p, q in zip(a, before):
        assert torch.equal(p, q)  # no update on a non-finite step
    assert float(opt.state_dict()["state"][0]["step"]) == 1.0  # and the step count is kept
    # resume: a fresh optimizer loaded from the state dict continues from step 1
    opt2 = ClipAdamW(a, lr=1e-3, weight_decay=1e-4, max_norm=1.0)
    opt2.load_state_dict(opt.state_dict())
    for p, g in zip(a, _grads(a, 2)):
        p.grad = g
    opt2.step()
    assert float(opt2.state_dict()["state"][0]["step"]) == 2.0
