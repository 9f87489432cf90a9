"""Fused HIP path (native encoders + fused update steps) vs the fp32 module path.

Oracle: the same RAFT in fp32 on the module path (``mixed_precision=False, fused_update=False,
native_encoder=False``: PyTorch/MIOpen convs, fp32-faithful correlation).  Tolerance: the error of the module path's own bf16 autocast
(MIOpen, ``fused_update=False, native_encoder=False``) against that oracle -- the fused
bf16 kernels must be at least about as close to fp32 as PyTorch's bf16 AMP is.
"""
from argparse import Namespace

import pytest
import torch

from raft_ros_amd.models import RAFT

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _run(m, batch, iters):
    from raft_ros_amd.train.loss import sequence_loss

    i1, i2, flow, valid = batch
    m.zero_grad()
    preds = m(i1, i2, iters=iters)
    loss, _ = sequence_loss(preds, flow, valid)
    loss.backward()
    return preds, {n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("small,shape", [(False, (2, 128, 192)), (False, (1, 136, 200)), (True, (2, 128, 192))])
def test_fused_path_matches_fp32_module(cuda, small, shape):
    from raft_ros_amd.data.synthetic import synthetic_batch

    B, H, W = shape
    torch.manual_seed(0)
    mk = lambda **kw: RAFT(Namespace(small=small, **kw)).to(cuda)  # noqa: E731
    f32 = mk(mixed_precision=False, fused_update=False, native_encoder=False)
    amp = mk(mixed_precision=True, amp_dtype="bf16", fused_update=False, native_encoder=False)
    fused = mk(mixed_precision=True, amp_dtype="bf16")
    for m in (amp, fused):
        m.load_state_dict(f32.state_dict())
    for m in (f32, amp, fused):
        m.train()
        m.freeze_bn()  # identical BN statistics in every run
    batch = synthetic_batch(B, H, W, max_disp=6, seed=1, device=cuda)
    pr, gr = _run(f32, batch, 3)
    pa, ga = _run(amp, batch, 3)
    pf, gf = _run(fused, batch, 3)
    for a, m, r in zip(pf, pa, pr):
        assert _rel(a, r) <= 1.5 * _rel(m, r) + 1e-2, (_rel(a, r), _rel(m, r))
    assert set(gf) == set(gr), set(gr) ^ set(gf)
    bad = {}
    for n in gr:
        ref_norm = gr[n].norm().item()
        floor = (ga[n] - gr[n]).norm().item()
        err = (gf[n] - gr[n]).norm().item()
        # conv biases in front of InstanceNorm: the true gradient is 0 (fused writes exactly 0)
        if ref_norm < 1e-6:
            if gf[n].abs().max().item() > 1e-3:
                bad[n] = ("nonzero", gf[n].abs().max().item())
            continue
        if err > 1.5 * floor + 0.02 * ref_norm:
            bad[n] = (err / ref_norm, floor / ref_norm)
    assert not bad, bad


@pytest.mark.parametrize("alt", [False, True], ids=["dense", "alternate_corr"])
def test_native_step_executor_matches_python_body(cuda, monkeypatch, alt):
    """fused_step_fwd (the step's launches issued from C++) vs the Python body of
    _Step.forward: the same kernels on the same operands, so the predictions are bitwise equal
    (training, with the tail stream) and so are the inference outputs (test_mode: the steps
    without upsampling); the gradients agree up to the backward's atomics."""
    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.ops import update_fused as uf

    torch.manual_seed(0)
    m = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16", alternate_corr=alt)).to(cuda).train()
    m.freeze_bn()
    batch = synthetic_batch(2, 128, 192, max_disp=6, seed=3, device=cuda)
    outs = {}
    for native in (False, True):
        monkeypatch.setattr(uf, "NATIVE_STEP", native)
        preds, grads = _run(m, batch, 4)
        m.eval()
        with torch.no_grad():
            lo, up = m(batch[0], batch[1], iters=5, test_mode=True)
        m.train()
        m.freeze_bn()
        outs[native] = (preds, grads, lo, up)
    (p0, g0, lo0, up0), (p1, g1, lo1, up1) = outs[False], outs[True]
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)
    assert torch.equal(lo0, lo1) and torch.equal(up0, up1)
    assert set(g0) == set(g1)
    tol = 1e-2 if alt else 1e-3  # the local-correlation backward accumulates with atomics
    for n in g0:
        assert _rel(g1[n], g0[n]) < tol, n


@pytest.mark.parametrize("alt", [False, True], ids=["dense", "alternate_corr"])
def test_native_backward_executor_matches_python_body(cuda, monkeypatch, alt):
    """fused_step_bwd (the step's backward launches issued from C++) vs the Python body of
    _Step.backward: the same kernels on the same operands in the same stream order, so with the
    deterministic dense backward every gradient is bitwise equal."""
    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.ops import update_fused as uf

    torch.manual_seed(0)
    m = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16", alternate_corr=alt)).to(cuda).train()
    m.freeze_bn()
    batch = synthetic_batch(2, 128, 192, max_disp=6, seed=3, device=cuda)
    outs = {}
    for native in (False, True):
        monkeypatch.setattr(uf, "NATIVE_BWD", native)
        outs[native] = _run(m, batch, 4)
    (p0, g0), (p1, g1) = outs[False], outs[True]
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)
    assert set(g0) == set(g1)
    for n in g0:
        if alt:  # the local-correlation backward accumulates with atomics
            assert _rel(g1[n], g0[n]) < 1e-2, n
        else:
            assert torch.equal(g1[n], g0[n]), n
