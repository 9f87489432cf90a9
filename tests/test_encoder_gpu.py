"""Native encoder kernels (csrc/encoder.hip, ops/encoder.py) against fp32 PyTorch.

Each HIP op is compared with the plain fp32 PyTorch op on the same bf16-rounded
inputs; the whole-encoder tests compare the native autograd node (bf16 operands,
fp32 accumulation) with the module path in fp32 (reference core/extractor.py).
"""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

cuda = torch.device("cuda", 0)


def _ops():
    from raft_ros_amd.ops._ext import ops
    return ops()


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _nchw(t):
    return t.permute(0, 3, 1, 2).float()


CONVS = [  # (B, Cin, Cx, H, W, Cout, k, stride, pad)
    (2, 3, 8, 64, 80, 64, 7, 2, 3),
    (2, 64, 64, 48, 40, 64, 3, 1, 1),   # resident-weight 3x3 kernel (16x16 tiles, partial last column)
    (3, 64, 64, 37, 45, 64, 3, 1, 1),   # partial tiles on both edges
    (1, 64, 64, 9, 200, 64, 3, 1, 1),   # image shorter than a tile
    (2, 128, 128, 20, 18, 128, 3, 1, 1),  # tap-batched halo-block weight gradient, 2 chunks
    (2, 64, 64, 48, 40, 96, 3, 2, 1),
    (2, 96, 96, 24, 20, 128, 3, 2, 1),
    (2, 64, 64, 48, 40, 96, 1, 2, 0),
    (2, 128, 128, 12, 10, 256, 1, 1, 0),
    (2, 96, 96, 13, 11, 160, 1, 1, 0),
    (2, 24, 24, 17, 15, 24, 3, 2, 1),
    (3, 8, 8, 33, 31, 32, 3, 1, 1),
]


@pytest.mark.parametrize("cfg", CONVS, ids=lambda c: f"k{c[6]}s{c[7]}c{c[1]}n{c[5]}")
def test_conv_fwd_stats_dgrad_wgrad(cfg):
    B, Cin, Cx, H, W, Cout, k, s, p = cfg
    g = torch.Generator(device=cuda).manual_seed(0)
    x = torch.randn(B, Cx, H, W, device=cuda, generator=g).bfloat16()
    if Cx > Cin:
        x[:, Cin:] = 0
    w = (torch.randn(Cout, Cin, k, k, device=cuda, generator=g) / (Cin * k * k) ** 0.5).contiguous(
        memory_format=torch.channels_last)
    bias = torch.randn(Cout, device=cuda, generator=g)
    xf = x[:, :Cin].float().requires_grad_(True)
    wf = w.bfloat16().float().requires_grad_(True)
    bf = bias.clone().requires_grad_(True)
    ref = F.conv2d(xf, wf, bf, stride=s, padding=p)

    y, st = _ops().enc_conv_fwd(_nhwc(x), w, bias, s, p, True)
    assert y.shape == (B, ref.shape[2], ref.shape[3], Cout)
    assert _rel(_nchw(y), ref) < 1e-2
    # tile statistics -> per-image mean / variance
    Ho, Wo = ref.shape[2], ref.shape[3]
    HW = Ho * Wo
    if st.dim() == 5:  # square 16x16 tiles of the resident-weight 3x3 kernel, row-major
        assert st.shape[1:3] == (-(-Ho // 16), -(-Wo // 16))
        tile_n = torch.tensor([min(16, Ho - ty * 16) * min(16, Wo - tx * 16) for ty in range(st.shape[1])
                               for tx in range(st.shape[2])], device=cuda, dtype=torch.float32)
        st = st.reshape(B, -1, 2, Cout)
    else:
        tile_n = torch.tensor([min(128, HW - t * 128) for t in range(st.shape[1])], device=cuda, dtype=torch.float32)
    sums, m2 = st[:, :, 0], st[:, :, 1]
    mean = sums.sum(1) / HW
    tmean = sums / tile_n[None, :, None]
    var = (m2 + tile_n[None, :, None] * (tmean - mean[:, None]) ** 2).sum(1) / HW
    rmean = ref.mean((2, 3))
    rvar = ref.var((2, 3), unbiased=False)
    assert torch.allclose(mean, rmean, atol=2e-2, rtol=1e-2)
    assert torch.allclose(var, rvar, atol=2e-2, rtol=2e-2)

    gy = torch.randn(ref.shape, device=cuda, generator=g).bfloat16()
    ref.backward(gy.float())
    if Cin % 8 == 0:  # (the stem's data gradient is never needed)
        dx = _ops().enc_conv_dgrad([_nhwc(gy)], [w], [s], [p], H, W, None, None)
        assert _rel(_nchw(dx), xf.grad) < 1e-2
    dw = torch.zeros_like(w)
    db = torch.zeros(Cout, device=cuda)
    _ops().enc_conv_wgrad(_nhwc(x), _nhwc(gy), dw, db, s, p, False)
    assert _rel(dw, wf.grad) < 1e-2
    assert _rel(db, bf.grad) < 1e-3
    # accumulate mode adds
    _ops().enc_conv_wgrad(_nhwc(x), _nhwc(gy), dw, db, s, p, True)
    assert _rel(dw, 2 * wf.grad) < 1e-2


@pytest.mark.parametrize("case", ["resblock_s2", "bottleneck_s2", "s1_res_mask"])
def test_merged_dgrad_residual_mask(case):
    g = torch.Generator(device=cuda).manual_seed(1)
    B, C, H, W = 2, 64, 30, 26
    x = torch.randn(B, C, H, W, device=cuda, generator=g).bfloat16()
    if case == "resblock_s2":
        convs = [(96, 3, 2, 1), (96, 1, 2, 0)]
    elif case == "bottleneck_s2":
        convs = [(16, 1, 1, 0), (64, 1, 2, 0)]
    else:
        convs = [(64, 3, 1, 1)]
    ws, gys, outs = [], [], []
    xf = x.float().requires_grad_(True)
    for (co, k, s, p) in convs:
        w = (torch.randn(co, C, k, k, device=cuda, generator=g) / (C * k * k) ** 0.5).bfloat16().float()
        ws.append(w)
        o = F.conv2d(xf, w, None, stride=s, padding=p)
        gy = torch.randn(o.shape, device=cuda, generator=g).bfloat16()
        gys.append(gy)
        outs.append((o * gy.float()).sum())
    sum(outs).backward()
    ref = xf.grad
    res = mask = None
    if case == "s1_res_mask":
        res = torch.randn(B, C, H, W, device=cuda, generator=g).bfloat16()
        mask = torch.relu(torch.randn(B, C, H, W, device=cuda, generator=g)).bfloat16()
        ref = (ref + res.float()) * (mask.float() > 0)
    dx = _ops().enc_conv_dgrad([_nhwc(t) for t in gys], ws, [c[2] for c in convs], [c[3] for c in convs], H, W,
                               _nhwc(res) if res is not None else None, _nhwc(mask) if mask is not None else None)
    assert _rel(_nchw(dx), ref) < 1e-2


def _encoders():
    from raft_ros_amd.models.extractor import BasicEncoder, SmallEncoder
    return {
        "basic_instance": lambda: BasicEncoder(256, "instance"),
        "basic_batch": lambda: BasicEncoder(256, "batch"),
        "basic_batch_eval": lambda: BasicEncoder(256, "batch"),
        "small_instance": lambda: SmallEncoder(128, "instance"),
        "small_none": lambda: SmallEncoder(160, "none"),
    }


@pytest.mark.parametrize("name", list(_encoders()))
def test_encoder_matches_fp32_module(name):
    """Native node vs the fp32 module.  Backward through a random-init ReLU network with
    bf16 activations is not a few-ulp computation (masks flip, errors compound over 8
    layers), so the tolerance is the error of the module's own bf16-autocast path
    (MIOpen) against the same fp32 module: native must be at least as close."""
    from raft_ros_amd.ops import encoder as enc_native
    torch.manual_seed(0)
    enc = _encoders()[name]().to(cuda).to(memory_format=torch.channels_last)
    enc.train()
    if name.endswith("eval"):
        for m in enc.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.normal_(0, 0.2)
                m.running_var.uniform_(0.5, 2.0)
                m.eval()
    ref = copy.deepcopy(enc)
    amp = copy.deepcopy(enc)
    g = torch.Generator(device=cuda).manual_seed(2)
    B, H, W = 2, 128, 160
    im1 = torch.rand(B, 3, H, W, device=cuda, generator=g) * 255
    im2 = torch.rand(B, 3, H, W, device=cuda, generator=g) * 255
    assert enc_native.supported(enc, im1)

    out = enc_native.encode(enc, im1, im2)
    n1 = 2 * (im1 / 255) - 1
    n2 = 2 * (im2 / 255) - 1
    rout = torch.cat(ref([n1, n2]), 0)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        aout = torch.cat(amp([n1, n2]), 0)
    assert out.shape == rout.shape and out.dtype == torch.bfloat16
    assert _rel(out, rout) <= 1.25 * _rel(aout, rout) + 2e-3, name
    gy = torch.randn(rout.shape, device=cuda, generator=g)
    (out.float() * gy).sum().backward()
    (rout * gy).sum().backward()
    (aout.float() * gy).sum().backward()
    refp = dict(ref.named_parameters())
    ampp = dict(amp.named_parameters())
    for n, p in enc.named_parameters():
        assert p.grad is not None, n
        q, a = refp[n], ampp[n]
        scale = refp[n.replace("bias", "weight")].grad.norm()
        if q.grad.norm() < 1e-4 * scale:
            # conv bias in front of a re-centring norm: the true gradient is 0
            assert p.grad.abs().max() < 1e-3 * scale, n
            continue
        floor = _rel(a.grad, q.grad)
        # BatchNorm affine and conv bias gradients are sums of dy (* xhat) over whole batches:
        # more cancellation, so bf16 noise is a larger fraction of them (a norm-free encoder's
        # bias gradients measured 0.12-0.16 relative for both MIOpen autocast and native)
        factor = 1.5 if (".norm" in n or n.endswith(".bias")) else 1.25
        assert _rel(p.grad, q.grad) <= factor * floor + 5e-3, (n, _rel(p.grad, q.grad), floor)
    for (n, b), (_, rb) in zip(enc.named_buffers(), ref.named_buffers()):
        if b.dtype.is_floating_point:
            assert torch.allclose(b, rb, atol=2e-3, rtol=2e-2), n
        else:
            assert torch.equal(b, rb), n


@pytest.mark.parametrize("name", list(_encoders()))
def test_split_encoder_inference_is_fp32_faithful(name):
    """fp32 inference (split-bf16 planes, [W_hi | W_hi | W_lo] packing, fp32 statistics and
    apply): the native encoder equals the fp32 module to ~1e-5 relative -- where the plain
    bf16 kernels are ~1e-2 off.  Eval mode: running BatchNorm statistics, InstanceNorm
    statistics per image."""
    from raft_ros_amd.ops import encoder as enc_native
    torch.manual_seed(0)
    enc = _encoders()[name]().to(cuda).to(memory_format=torch.channels_last).eval()
    for m in enc.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.normal_(0, 0.2)
            m.running_var.uniform_(0.5, 2.0)
    g = torch.Generator(device=cuda).manual_seed(2)
    B, H, W = 2, 128, 160
    im1 = torch.rand(B, 3, H, W, device=cuda, generator=g) * 255
    im2 = torch.rand(B, 3, H, W, device=cuda, generator=g) * 255
    with torch.no_grad():
        out = enc_native.encode(enc, im1, im2, split=True)
        ref = torch.cat(enc([2 * (im1 / 255) - 1, 2 * (im2 / 255) - 1]), 0)
    assert out.dtype == torch.float32 and out.shape == ref.shape
    err = _rel(out, ref)
    assert err < 2e-4, (name, err)  # measured 1e-5 (basic) .. 5.5e-5 (small)


@pytest.mark.parametrize("mode", ["bf16", "f16", "split", "split_infer"])
@pytest.mark.parametrize("name", ["basic_batch", "small_instance"])
def test_prepacked_weights_match_per_conv_packing(name, mode, monkeypatch):
    """Weights packed ahead by the one-launch multi-conv packing (ops/encoder.py _Prepack) give
    bit-identical outputs and gradients to the per-conv packing, also after an in-place weight
    update (the optimizer step the next forward's packing must see)."""
    from raft_ros_amd.ops import encoder as enc_native
    torch.manual_seed(0)
    base = _encoders()[name]().to(cuda).to(memory_format=torch.channels_last).train()
    nets = {flag: copy.deepcopy(base) for flag in (True, False)}
    g = torch.Generator(device=cuda).manual_seed(3)
    B, H, W = 2, 96, 128
    ims = [torch.rand(B, 3, H, W, device=cuda, generator=g) * 255 for _ in range(2)]
    gy = None
    res = {}
    for flag, enc in nets.items():
        monkeypatch.setattr(enc_native, "PREPACK", flag)
        outs, grads = [], []
        for step in range(2):
            if step == 1:
                with torch.no_grad():
                    for p in enc.parameters():
                        p.mul_(1.01).add_(1e-3)
            enc.zero_grad(set_to_none=True)
            with torch.set_grad_enabled(mode != "split_infer"):
                out = enc_native.encode(enc, ims[0], ims[1], split=mode.startswith("split"), f16=mode == "f16")
            outs.append(out.float().clone())
            if mode != "split_infer":
                if gy is None:
                    gy = torch.randn(out.shape, device=cuda, generator=g)
                (out.float() * gy).sum().backward()
                grads.append([p.grad.clone() for p in enc.parameters()])
        torch.cuda.synchronize()
        res[flag] = (outs, grads)
    assert bool(enc_native._layout(nets[True]).__dict__.get("prepacks")), "prepacking did not run"
    for a, b in zip(res[True][0], res[False][0]):
        assert torch.equal(a, b)
    for ga, gb in zip(res[True][1], res[False][1]):
        for x, y in zip(ga, gb):
            assert torch.equal(x, y)
