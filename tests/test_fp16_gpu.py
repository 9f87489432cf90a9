"""Native fp16 AMP (the reference's --mixed_precision dtype: fp16 autocast + GradScaler,
core/raft.py:11-21, train.py:24-38,154) on the hand-written kernels (v_mfma_f32_32x32x16_f16).

Oracle: the fp32 module path.  Tolerance: the error of PyTorch's own fp16 autocast of the module
path (MIOpen) against that oracle -- the native fp16 kernels must be about as close to fp32."""
from argparse import Namespace

import pytest
import torch

from raft_ros_amd.models import RAFT

pytestmark = pytest.mark.gpu
SCALE = 1024.0  # static loss scale (GradScaler's role): keeps small gradients out of fp16 underflow


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _run(m, batch, iters):
    from raft_ros_amd.train.loss import sequence_loss

    i1, i2, flow, valid = batch
    m.zero_grad()
    preds = m(i1, i2, iters=iters)
    loss, _ = sequence_loss(preds, flow, valid)
    (loss * SCALE).backward()
    torch.cuda.synchronize()
    return preds, {n: p.grad.float() / SCALE for n, p in m.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("small", [False, True])
def test_native_fp16_amp_matches_fp32_module(cuda, small):
    from raft_ros_amd.data.synthetic import synthetic_batch

    torch.manual_seed(0)
    mk = lambda **kw: RAFT(Namespace(small=small, **kw)).to(cuda)  # noqa: E731
    f32 = mk(mixed_precision=False, fused_update=False, native_encoder=False)
    amp = mk(mixed_precision=True, amp_dtype="fp16", fused_update=False, native_encoder=False)
    nat = mk(mixed_precision=True, amp_dtype="fp16")
    for m in (amp, nat):
        m.load_state_dict(f32.state_dict())
    for m in (f32, amp, nat):
        m.train()
        m.freeze_bn()
    i1 = torch.zeros(1, 3, 128, 192, device=cuda)
    assert nat._use_fused(i1, True) and nat._use_native_encoders(i1, True)
    batch = synthetic_batch(2, 128, 192, max_disp=6, seed=1, device=cuda)
    pr, gr = _run(f32, batch, 3)
    pa, ga = _run(amp, batch, 3)
    pn, gn = _run(nat, batch, 3)
    for a, m, r in zip(pn, pa, pr):
        assert _rel(a, r) <= 1.5 * _rel(m, r) + 1e-3, (_rel(a, r), _rel(m, r))
    bad, rows = {}, []
    for n in gr:
        ref_norm = gr[n].norm().item()
        if ref_norm < 1e-6:
            continue
        floor = (ga[n] - gr[n]).norm().item()
        err = (gn[n] - gr[n]).norm().item()
        rows.append((err / ref_norm, floor / ref_norm))
        if not torch.isfinite(gn[n]).all() or err > 2.0 * floor + 0.01 * ref_norm:
            bad[n] = (err / ref_norm, floor / ref_norm)
    print(f"\nfp16 native vs fp32: median grad rel err {sorted(r[0] for r in rows)[len(rows) // 2]:.2e} "
          f"(torch fp16 autocast {sorted(r[1] for r in rows)[len(rows) // 2]:.2e})")
    assert not bad, bad


def test_native_fp16_training_step_runs_no_torch_conv(cuda):
    """bench.py --amp_dtype fp16 path: every conv of the training step on the HIP kernels."""
    from raft_ros_amd.data.synthetic import synthetic_batch

    m = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="fp16")).to(cuda).train()
    calls = []
    orig = torch.nn.functional.conv2d

    def spy(*a, **k):
        calls.append(a[1].shape)
        return orig(*a, **k)

    torch.nn.functional.conv2d = spy
    try:
        i1, i2, flow, valid = synthetic_batch(1, 128, 160, seed=0, device=cuda)
        preds = m(i1, i2, iters=2)
        sum(p.sum() for p in preds).backward()
    finally:
        torch.nn.functional.conv2d = orig
    assert not calls, calls
