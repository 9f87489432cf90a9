"""End-to-end RAFT on the GPU: native HIP path vs the PyTorch reference op path."""
from argparse import Namespace

import pytest
import torch

from raft_ros_amd.models import RAFT
from raft_ros_amd.ops import _ext

pytestmark = pytest.mark.gpu


def _pair(dev, B=1, H=128, W=160, seed=0):
    from raft_ros_amd.data.synthetic import synthetic_batch

    return synthetic_batch(B, H, W, max_disp=8, seed=seed, device=dev)


@pytest.mark.parametrize("small", [False, True])
def test_native_matches_reference_path_fp32(cuda, small):
    torch.manual_seed(0)
    model = RAFT(Namespace(small=small, mixed_precision=False)).to(cuda).eval()
    i1, i2, _, _ = _pair(cuda)
    with torch.no_grad():
        _ext.set_backend("reference")
        try:
            lo_r, up_r = model(i1, i2, iters=4, test_mode=True)
        finally:
            _ext.set_backend("native")
        lo, up = model(i1, i2, iters=4, test_mode=True)
    # without AMP the native correlation is the split-bf16 (hi/lo, 3-MFMA) fp32-faithful
    # GEMM and the lookup / upsampling kernels are fp32: compare as flow error in pixels
    epe = (up - up_r).norm(dim=1).mean().item()
    print(f"\nsmall={small} EPE native fp32 vs reference op path: {epe:.2e} px")
    assert epe <= 1e-2, epe


def test_fp32_native_inference_tracks_trained_weights_and_bn_stats(cuda):
    """fp32 inference on the native split-bf16 encoders / update block after the weights move
    under a fused AdamW step (which does not bump parameter versions) and with non-trivial
    BatchNorm running statistics == the module path (regression: a version-keyed split-weight
    cache served the pre-step weights, val EPE 88 px in an fp32 convergence run)."""
    torch.manual_seed(0)
    args = Namespace(small=False, mixed_precision=False, channels_last=True)
    model = RAFT(args).to(cuda).to(memory_format=torch.channels_last).eval()
    i1, i2, _, _ = _pair(cuda)
    with torch.no_grad():
        model(i1, i2, iters=2, test_mode=True)  # warm every cache of the native path
    opt = torch.optim.AdamW(model.parameters(), lr=5e-2, fused=True)
    for p in model.parameters():
        p.grad = torch.randn_like(p)
    opt.step()
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-2, 2)
            m.running_var.uniform_(0.05, 8)
    with torch.no_grad():
        lo, up = model(i1, i2, iters=4, test_mode=True)
        args.native_encoder = args.fused_update = False
        lo_m, up_m = model(i1, i2, iters=4, test_mode=True)
    epe = (up - up_m).norm(dim=1).mean().item()
    print(f"\nEPE native split vs module path after an optimizer step: {epe:.2e} px")
    assert epe <= 1e-2 * max(1.0, up_m.norm(dim=1).mean().item()), epe


def test_training_step_runs_and_decreases_loss(cuda):
    from raft_ros_amd.train.loss import sequence_loss

    torch.manual_seed(0)
    model = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16")).to(cuda)
    model = model.to(memory_format=torch.channels_last).train()
    opt = torch.optim.AdamW(model.parameters(), lr=2e-4)
    i1, i2, flow, valid = _pair(cuda, B=2, H=128, W=192)
    losses = []
    for _ in range(8):
        opt.zero_grad()
        preds = model(i1, i2, iters=4)
        loss, _ = sequence_loss(preds, flow, valid)
        loss.backward()
        for p in model.parameters():
            assert p.grad is None or torch.isfinite(p.grad).all()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("small,amp", [(False, True), (False, False), (True, True)])
def test_test_mode_skips_intermediate_upsampling_bitwise(cuda, small, amp):
    """test_mode without autograd skips the mask head / upsampling of all but the last step:
    the returned flows equal the last of the full per-step predictions (bit for bit on the
    bf16 fused path; the fp32 path's library convs may pick other algorithms per call)."""
    torch.manual_seed(0)
    model = RAFT(Namespace(small=small, mixed_precision=amp, amp_dtype="bf16")).to(cuda).eval()
    i1, i2, _, _ = _pair(cuda, B=2)
    with torch.no_grad():
        lo, up = model(i1, i2, iters=5, test_mode=True)
        preds = model(i1, i2, iters=5, test_mode=False)
    if amp:
        assert torch.equal(up, preds[-1])
    else:
        torch.testing.assert_close(up, preds[-1], rtol=1e-5, atol=1e-5)
    assert lo.shape[-2:] == (up.shape[-2] // 8, up.shape[-1] // 8) and torch.isfinite(lo).all()


def test_alternate_corr_inference(cuda):
    torch.manual_seed(0)
    model = RAFT(Namespace(small=False, mixed_precision=False)).to(cuda).eval()
    alt = RAFT(Namespace(small=False, mixed_precision=False, alternate_corr=True)).to(cuda).eval()
    alt.load_state_dict(model.state_dict())
    i1, i2, _, _ = _pair(cuda)
    with torch.no_grad():
        _, up = model(i1, i2, iters=3, test_mode=True)
        _, up_alt = alt(i1, i2, iters=3, test_mode=True)
    # both fp32-faithful (local correlation in fp32 vs the split-bf16 dense volume)
    epe = (up - up_alt).norm(dim=1).mean().item()
    print(f"\nEPE alternate_corr vs dense (fp32): {epe:.2e} px")
    assert epe <= 1e-2, epe


def test_fp16_amp_dense_correlation_is_fp32_faithful(cuda, monkeypatch):
    """Under fp16 autocast the reference still builds the volume in fp32 (core/raft.py:102-103):
    the dense pyramid must be the split (fp32-faithful) one, and its lookups must match the
    fp32 reference volume built from the same feature maps."""
    import raft_ros_amd.models.raft as R
    from raft_ros_amd.ops import reference as ref

    seen = {}
    orig = R.CorrPyramid

    class Recorded(orig):  # a subclass: the model dispatches on isinstance(corr_fn, CorrPyramid)
        def __init__(self, fmap1, fmap2, **kw):
            seen.update(split=kw.get("split"), f=(fmap1.detach().clone(), fmap2.detach().clone()))
            super().__init__(fmap1, fmap2, **kw)
            seen["pyr"] = self

    monkeypatch.setattr(R, "CorrPyramid", Recorded)
    torch.manual_seed(0)
    model = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="fp16")).to(cuda).eval()
    i1, i2, _, _ = _pair(cuda, B=1, H=128, W=192)
    with torch.no_grad():
        model(i1, i2, iters=2, test_mode=True)
    assert seen["split"] is True
    f1, f2 = seen["f"]
    B, _, H, W = f1.shape
    g = torch.Generator(device=cuda).manual_seed(3)
    coords = ref.coords_grid(B, H, W, device=cuda) + 4 * torch.randn(B, 2, H, W, device=cuda, generator=g)
    with torch.no_grad():
        got = seen["pyr"](coords)
        want = ref.pyramid_lookup(ref.build_pyramid(ref.corr_volume(f1.float(), f2.float()), 4), coords, 4)
    err = ((got - want).abs().max() / want.abs().max()).item()
    assert err < 1e-4, err


@pytest.mark.parametrize("small,amp", [(True, False), (False, True)])
def test_graphed_inference_matches_eager(cuda, small, amp):
    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.runtime import GraphedRAFT

    torch.manual_seed(0)
    model = RAFT(Namespace(small=small, mixed_precision=amp, alternate_corr=False)).to(cuda).eval()
    runner = GraphedRAFT(model, iters=4)
    for seed in (1, 2):  # second pair replays the captured graph on new inputs
        i1, i2, _, _ = synthetic_batch(2, 128, 192, seed=seed, device=cuda)
        with torch.no_grad():
            ref_low, ref_up = model(i1, i2, iters=4, test_mode=True)
        low, up = runner(i1, i2)
        if amp:  # bf16: MIOpen may pick other solvers under capture -> rounding-level differences
            for a, b in ((up, ref_up), (low, ref_low)):
                rel = ((a - b).abs().mean() / b.abs().mean()).item()
                assert rel < 2e-2, (rel, b.abs().mean().item())
        else:
            torch.testing.assert_close(up, ref_up, rtol=1e-3, atol=1e-3)
            torch.testing.assert_close(low, ref_low, rtol=1e-3, atol=1e-3)
    assert runner.num_graphs == 1


def _epe(a, b):
    return (a.float() - b.float()).norm(dim=1).mean().item()


@pytest.mark.parametrize("iters", [12, 32])
def test_bench_resolution_epe_vs_fp32_reference(cuda, iters):
    """368x496 (BASELINE config #2 resolution), test_mode flows after 12 / 32 iterations.

    * native fp32 path (mixed_precision=False: fp32-faithful split-bf16 correlation, native
      lookup / upsampling) vs the reference op sequence in fp32: EPE delta <= 0.01 px;
    * native bf16 path (native encoders + fused update kernels) vs the same fp32 oracle:
      bounded by 3x the delta of PyTorch's own bf16 autocast (module path, MIOpen) and by
      5 % of the mean flow magnitude.  The measured deltas are printed (pytest -s).
    """
    torch.manual_seed(0)
    f32 = RAFT(Namespace(small=False, mixed_precision=False)).to(cuda).eval()
    bf = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16")).to(cuda).eval()
    amp = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16", fused_update=False,
                         native_encoder=False)).to(cuda).eval()
    for m in (bf, amp):
        m.load_state_dict(f32.state_dict())
    i1, i2, _, _ = _pair(cuda, B=1, H=368, W=496, seed=5)
    with torch.no_grad():
        _ext.set_backend("reference")
        try:
            _, up_ref = f32(i1, i2, iters=iters, test_mode=True)
        finally:
            _ext.set_backend("native")
        _, up_f32 = f32(i1, i2, iters=iters, test_mode=True)
        _, up_bf = bf(i1, i2, iters=iters, test_mode=True)
        _, up_amp = amp(i1, i2, iters=iters, test_mode=True)
    mag = up_ref.norm(dim=1).mean().item()
    d32, dbf, damp = _epe(up_f32, up_ref), _epe(up_bf, up_ref), _epe(up_amp, up_ref)
    print(f"\niters={iters} mean|flow|={mag:.3f}  EPE delta: native fp32 {d32:.5f}  native bf16 {dbf:.4f}  "
          f"torch bf16 autocast {damp:.4f}")
    assert d32 <= 0.01, d32
    assert dbf <= max(3 * damp, 1e-3) and dbf <= 0.05 * max(mag, 1.0), (dbf, damp, mag)
