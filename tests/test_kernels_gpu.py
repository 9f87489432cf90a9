"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op."""
import math

import pytest
import torch
import torch.nn.functional as F

from raft_ros_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _ops():
    from raft_ros_amd.ops._ext import ops

    return ops()


@pytest.mark.parametrize("M,N,K,batch", [(2852, 2852, 256, 2), (100, 70, 128, 1), (257, 129, 64, 3)])
def test_gemm_nt_bf16(cuda, M, N, K, batch):
    torch.manual_seed(0)
    A = torch.randn(batch, M, K, device=cuda).bfloat16()
    B = torch.randn(batch, N, K, device=cuda).bfloat16()
    C = _ops().gemm_nt(A, B, 0.5, torch.float32)
    R = 0.5 * torch.matmul(A.float(), B.float().transpose(1, 2))
    torch.testing.assert_close(C, R, rtol=1e-3, atol=1e-3)
    # asymmetric operands catch a transposed C/D write
    Cb = _ops().gemm_nt(A, B, 1.0, torch.bfloat16)
    torch.testing.assert_close(Cb.float(), 2 * R, rtol=2e-2, atol=5e-2)


@pytest.mark.parametrize("M,N,K,batch", [(2852, 3808, 256, 2), (300, 1000, 128, 3), (64, 8, 64, 1)])
def test_corr_volume_v2_matches_generic(cuda, M, N, K, batch):
    """The store-oriented bf16 volume kernel (corr_volume_bf16_kernel: DMA ring, swizzled
    LDS, LDS-staged 16-byte stores) vs the generic kernel (cfg=1) and an fp32 matmul: partial
    tiles in M and N, odd N (partial 16-byte chunks at the row end)."""
    torch.manual_seed(3)
    ops = _ops()
    A = torch.randn(batch, M, K, device=cuda).bfloat16()
    B = torch.randn(batch, N, K, device=cuda).bfloat16()
    outs = []
    cfgs = (0, 1, 7, 8, 9, 11)  # 0 / 7 / 8: the v3 kernel (BK 32 at four per CU, GM 8, BK 64); 9: v2; 11: v3 + NT stores
    for cfg in cfgs:
        C = torch.full((batch, M, N), float("nan"), device=cuda, dtype=torch.bfloat16)
        ops.corr_gemm(A, B, C, M, N, K, batch, K, M * K, K, N * K, N, M * N, 0.0625, False, False, 0, cfg)
        outs.append(C.float())
    want = 0.0625 * torch.matmul(A.float(), B.float().transpose(1, 2))
    for cfg, out in zip(cfgs, outs):
        assert torch.isfinite(out).all(), cfg
        torch.testing.assert_close(out, want, rtol=1e-2, atol=1e-2)
        assert (out - outs[1]).abs().max().item() <= 2 * want.abs().max().item() * 2 ** -8, cfg


@pytest.mark.parametrize("HW,ld,C,batch", [(2852, 3936, 256, 2), (130, 200, 72, 3), (21, 48, 136, 1)])
def test_corr_bwd_kernel_matches_fp32(cuda, HW, ld, C, batch):
    """The pyramid-backward GEMMs on corr_bwd_kernel (cfg 10) vs fp32 matmuls of the same bf16
    operands: dF1 = a dL . f2t^T (bf16 out) and G = a dL^T . f1t^T (A read transposed, fp32 out),
    with K tails (HW % 32, ld % 32), partial M / N tiles and a padded f1t pitch; the outputs start
    as NaN so an unwritten element fails."""
    torch.manual_seed(9)
    ops = _ops()
    a = 0.0625
    dL = torch.randn(batch, HW, ld, device=cuda).bfloat16()
    f2t = torch.randn(batch, C, ld, device=cuda).bfloat16()
    hp = (HW + 7) // 8 * 8
    f1t = torch.zeros(batch, C, hp, device=cuda).bfloat16()
    f1t[:, :, :HW] = torch.randn(batch, C, HW, device=cuda).bfloat16()
    d1 = torch.full((batch, HW, C), float("nan"), device=cuda, dtype=torch.bfloat16)
    ops.corr_gemm(dL, f2t, d1, HW, C, ld, batch, ld, HW * ld, ld, C * ld, C, HW * C, a, False, False, 0, 10)
    want1 = a * torch.matmul(dL.float(), f2t.float().transpose(1, 2))
    assert torch.isfinite(d1.float()).all()
    torch.testing.assert_close(d1.float(), want1, rtol=1e-2, atol=1e-2 * want1.abs().max().item())
    G = torch.full((batch, ld, C), float("nan"), device=cuda)
    ops.corr_gemm(dL, f1t, G, ld, C, HW, batch, ld, HW * ld, hp, C * hp, C, ld * C, a, True, False, 0, 10)
    want2 = a * torch.matmul(dL.float().transpose(1, 2), f1t[:, :, :HW].float().transpose(1, 2))
    assert torch.isfinite(G).all()
    torch.testing.assert_close(G, want2, rtol=1e-3, atol=1e-3 * want2.abs().max().item())
    # both GEMMs in one launch (the training path): the same tiles, bitwise
    d1p = torch.full_like(d1, float("nan"))
    Gp = torch.full_like(G, float("nan"))
    ops.corr_pyramid_bwd(dL, f2t, f1t, d1p, Gp, a)
    assert torch.equal(d1p, d1) and torch.equal(Gp, G)


def test_gemm_nt_identity_asymmetric(cuda):
    M, K = 128, 128
    A = torch.eye(M, K, device=cuda).bfloat16()[None]
    B = (torch.arange(M * K, device=cuda).reshape(M, K) % 7 - 3).float().bfloat16()[None]
    C = _ops().gemm_nt(A, B, 1.0, torch.float32)
    torch.testing.assert_close(C[0], B[0].float().t())


@pytest.mark.parametrize("split", [False, True])
def test_corr_gemm_modes(cuda, split):
    """Transposed A operand, fp32 inputs (split: 3-pass bf16), accumulate and unpool epilogues."""
    torch.manual_seed(5)
    ops = _ops()
    B, M, N, K = 2, 90, 40, 200  # odd sizes: partial tiles, K % 8 == 0
    A = torch.randn(B, K, M + 6, device=cuda)  # stored transposed, padded pitch
    Bm = torch.randn(B, N, K, device=cuda)
    C = torch.randn(B, M, N, device=cuda)
    C0 = C.clone()
    ops.corr_gemm(A, Bm, C, M, N, K, B, M + 6, K * (M + 6), K, N * K, N, M * N, 0.5, True, split, 1)
    want = C0 + 0.5 * torch.matmul(A[:, :, :M].transpose(1, 2), Bm.transpose(1, 2))
    tol = 1e-4 if split else 2e-2
    assert ((C - want).norm() / want.norm()).item() < tol


def test_pyramid_unpool_is_the_pool_adjoint(cuda):
    torch.manual_seed(7)
    B, C, H, W = 2, 16, 13, 22
    sizes, off = [], 0
    for l in range(4):
        Hl, Wl = H >> l, W >> l
        sizes.append((off, Hl, Wl))
        off += (Hl * Wl + 7) // 8 * 8
    G = torch.randn(B, off, C, device=cuda)
    out = _ops().pyramid_unpool(G, H, W, [v for s_ in sizes for v in s_])
    # adjoint check: <unpool(G), x> == sum_l <G_l, pool_l(x)>
    x = torch.randn(B, C, H, W, device=cuda, dtype=torch.float64)
    lhs = (out.double() * x.permute(0, 2, 3, 1).reshape(B, H * W, C)).sum()
    rhs, p = 0.0, x
    for l, (o, Hl, Wl) in enumerate(sizes):
        if l:
            p = F.avg_pool2d(p, 2, 2)
        rhs = rhs + (G[:, o:o + Hl * Wl].double() * p.permute(0, 2, 3, 1).reshape(B, Hl * Wl, C)).sum()
    assert abs((lhs - rhs) / rhs).item() < 1e-6


def test_corr_pyramid_split_is_fp32_faithful(cuda):
    """Without AMP the native pyramid (split bf16 MFMA) matches the fp32 reference volume and
    its gradients closely (reference core/raft.py:102-103 keeps the volume fp32)."""
    torch.manual_seed(6)
    from raft_ros_amd.ops.corr import CorrPyramid

    B, C, H, W, r = 2, 256, 46, 62, 4
    f1 = torch.randn(B, C, H, W, device=cuda, requires_grad=True)
    f2 = torch.randn(B, C, H, W, device=cuda, requires_grad=True)
    coords = ref.coords_grid(B, H, W, cuda) + 4 * torch.randn(B, 2, H, W, device=cuda)
    g = torch.randn(B, 4 * (2 * r + 1) ** 2, H, W, device=cuda)
    out = CorrPyramid(f1, f2, 4, r, split=True)(coords)
    f1r = f1.detach().clone().requires_grad_(True)
    f2r = f2.detach().clone().requires_grad_(True)
    want = ref.pyramid_lookup(ref.build_pyramid(ref.corr_volume(f1r, f2r), 4), coords, r)
    assert ((out - want).norm() / want.norm()).item() < 3e-5
    (out * g).sum().backward()
    (want * g).sum().backward()
    for got, exp in ((f1.grad, f1r.grad), (f2.grad, f2r.grad)):
        assert ((got - exp).norm() / exp.norm()).item() < 3e-5


def test_avgpool(cuda):
    x = torch.randn(37, 23, 31, device=cuda)
    torch.testing.assert_close(_ops().avgpool2x2(x), F.avg_pool2d(x[:, None], 2, 2)[:, 0])


def _pyramid(B, C, H, W, dev, levels=4):
    f1 = torch.randn(B, C, H, W, device=dev)
    f2 = torch.randn(B, C, H, W, device=dev)
    corr = ref.corr_volume(f1, f2)
    return f1, f2, ref.build_pyramid(corr, levels)


@pytest.mark.parametrize("radius,shape", [(4, (2, 46, 62)), (3, (1, 17, 23))])
def test_corr_lookup_fwd(cuda, radius, shape):
    torch.manual_seed(1)
    B, H, W = shape
    _, _, pyr = _pyramid(B, 64, H, W, cuda)
    coords = ref.coords_grid(B, H, W, cuda) + 6 * torch.randn(B, 2, H, W, device=cuda)
    coords[0, :, 0, 0] = torch.tensor([-30.0, 500.0])  # fully out of range
    want = ref.pyramid_lookup(pyr, coords, radius)
    got = _ops().corr_lookup([p[:, 0].contiguous() for p in pyr], coords.contiguous(), radius, torch.float32)
    torch.testing.assert_close(got.permute(0, 3, 1, 2), want, rtol=1e-4, atol=1e-4)
    got16 = _ops().corr_lookup([p[:, 0].contiguous() for p in pyr], coords.contiguous(), radius, torch.bfloat16)
    torch.testing.assert_close(got16.permute(0, 3, 1, 2).float(), want, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("radius,T", [(4, 12), (3, 35)])
def test_lookup_grad_rows_match_per_lookup_backward(cuda, radius, T):
    """Deferred lookup backward (one LDS-accumulated row pass over all T lookups, T > 32 in
    two launches) == T per-lookup read-modify-write passes into a zeroed fp32 buffer; the
    bf16 rows are those fp32 rows rounded once."""
    from raft_ros_amd.ops.corr import _PyramidState

    torch.manual_seed(12)
    B, H, W, L = 2, 19, 45, 4
    st = _PyramidState(L, radius)
    sizes, off = [], 0
    for l in range(L):
        Hl, Wl = H >> l, W >> l
        sizes.append((Hl, Wl, off))
        off += -(-Wl // 16) * 16 * Hl
    st.sizes, st.ld = sizes, off
    win = (2 * radius + 1) ** 2
    coords = [(ref.coords_grid(B, H, W, cuda) + 6 * torch.randn(B, 2, H, W, device=cuda)).contiguous()
              for _ in range(T)]
    coords[1][0, :, 2, 2] = float("nan")
    grads = [torch.randn(B, H, W, L * win + 4, device=cuda).bfloat16() for _ in range(T)]
    want = torch.zeros(B * H * W, off, device=cuda)
    lv = st.views(want)
    for c, g in zip(coords, grads):
        _ops().corr_lookup_backward_(lv, c, g, radius)
    segs = st.segments()
    for dt in (torch.float32, torch.bfloat16):
        got = torch.full((B * H * W, off), float("nan"), device=cuda, dtype=dt)
        for i in range(0, T, 32):
            _ops().corr_lookup_grad_rows(got, coords[i:i + 32], grads[i:i + 32], segs, radius, i > 0)
        if dt == torch.float32:
            torch.testing.assert_close(got, want, rtol=1e-6, atol=1e-6)
        elif T <= 32:
            assert torch.equal(got, want.bfloat16())
        else:  # the second launch re-reads the bf16 partial rows: rounded twice
            assert ((got.float() - want).norm() / want.norm()).item() < 4e-3


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("blocked", [True, False])
@pytest.mark.parametrize("fmt", ["cl", "nchw"])
def test_pyramid_operand_matches_torch_ops(cuda, dtype, blocked, fmt):
    """The one-launch pyramid GEMM operand == F.avg_pool2d levels + pad/permute copies, bit for bit
    (channels-last sources take the 4-channel vector loads, NCHW ones the per-channel path)."""
    from raft_ros_amd.ops.corr import _concat_levels, _pad_to, _pooled

    torch.manual_seed(8)
    B, C, H, W = 2, 64, 27, 45  # odd sizes: floor pooling, partial 16-column blocks
    fmap = torch.randn(B, C, H, W, device=cuda).to(dtype)
    if fmt == "cl":
        fmap = fmap.contiguous(memory_format=torch.channels_last)
    fs = _pooled(fmap.float(), 4)
    segs, off = [], 0
    for f in fs:
        Hl, Wl = f.shape[-2:]
        segs += [off, Hl, Wl]
        off += -(-Wl // 16) * 16 * Hl if blocked else _pad_to(Hl * Wl, 8)
    for nchw in (False, True):
        want = _concat_levels(fs, off, segs[0::3], nchw=nchw, blocked=blocked)
        got = _ops().pyramid_operand(fmap, segs, off, blocked, nchw)
        assert torch.equal(got, want), (nchw, (got - want).abs().max().item())
    # level 0 only, transposed and zero-padded: the dF2 GEMM's f1 operand
    f1t = _ops().pyramid_operand(fmap, [0, H, W], _pad_to(H * W, 8), False, True)
    assert torch.equal(f1t[:, :, :H * W], fmap.float().reshape(B, C, H * W)) and not f1t[:, :, H * W:].any()


def test_corr_lookup_into_packs_flow_like_pack_flow(cuda):
    """The lookup launch's folded flow packing == the standalone pack_flow op, bit for bit."""
    torch.manual_seed(7)
    B, H, W, r = 2, 13, 17, 4
    _, _, pyr = _pyramid(B, 64, H, W, cuda)
    levels = [p[:, 0].contiguous() for p in pyr]
    coords = (ref.coords_grid(B, H, W, cuda) + 5 * torch.randn(B, 2, H, W, device=cuda)).contiguous()
    P = B * H * W
    out = torch.empty(B, H, W, 328, device=cuda, dtype=torch.bfloat16)
    flow8, motion = torch.full((P, 8), 7.0, device=cuda).bfloat16(), torch.zeros(P, 128, device=cuda).bfloat16()
    _ops().corr_lookup_into(levels, coords, r, out, flow8, motion[:, 126:])
    f8_ref, mo_ref = torch.empty_like(flow8), torch.zeros_like(motion)
    _ops().pack_flow(coords, f8_ref, mo_ref[:, 126:], True)
    assert torch.equal(flow8, f8_ref) and torch.equal(motion, mo_ref)
    # the correlation features are unchanged by the extra outputs
    want = _ops().corr_lookup(levels, coords, r, torch.bfloat16)
    torch.testing.assert_close(out[..., :324], want, rtol=0, atol=0)


def test_corr_lookup_window_order_is_x_major(cuda):
    # a volume that is a pure ramp in x: tap channel ix*(2r+1)+iy must move x with ix
    B, H, W, r = 1, 16, 16, 2
    xs = torch.arange(W, device=cuda, dtype=torch.float32).view(1, 1, W).expand(B * H * W, H, W).contiguous()
    coords = ref.coords_grid(B, H, W, cuda)
    out = _ops().corr_lookup([xs], coords, r, torch.float32)  # (B, H, W, 25)
    rd = 2 * r + 1
    px = out[0, 8, 8].view(rd, rd)  # [ix, iy]
    assert torch.allclose(px[:, 0], torch.arange(8 - r, 8 + r + 1, device=cuda, dtype=torch.float32))
    assert torch.allclose(px[2], torch.full((rd,), 8.0, device=cuda))


def test_corr_pyramid_autograd_matches_reference(cuda):
    torch.manual_seed(2)
    from raft_ros_amd.ops.corr import CorrPyramid

    B, C, H, W, r = 2, 256, 20, 28, 4
    f1 = torch.randn(B, C, H, W, device=cuda, requires_grad=True)
    f2 = torch.randn(B, C, H, W, device=cuda, requires_grad=True)
    coords_list = [ref.coords_grid(B, H, W, cuda) + 3 * torch.randn(B, 2, H, W, device=cuda) for _ in range(3)]
    gouts = [torch.randn(B, 4 * (2 * r + 1) ** 2, H, W, device=cuda) for _ in range(3)]

    cp = CorrPyramid(f1, f2, 4, r)
    outs_native = [cp(c) for c in coords_list]
    f1r = f1.detach().clone().requires_grad_(True)
    f2r = f2.detach().clone().requires_grad_(True)
    pyr = ref.build_pyramid(ref.corr_volume(f1r, f2r), 4)
    outs = [ref.pyramid_lookup(pyr, c, r) for c in coords_list]
    for o, c in zip(outs, outs_native):
        # bf16 MFMA volume vs fp32 reference
        assert (o.detach() - c.detach().float()).abs().max() < 0.05 * o.detach().abs().max()
    loss = sum((o * g).sum() for o, g in zip(outs_native, gouts))
    loss.backward()
    g1, g2 = f1.grad.clone(), f2.grad.clone()
    lr = sum((o * g).sum() for o, g in zip(outs, gouts))
    lr.backward()
    for got, want in ((g1, f1r.grad), (g2, f2r.grad)):
        err = (got - want).norm() / want.norm()
        assert err < 1e-2, err


@pytest.mark.parametrize("shape,layout", [((2, 13, 17), "cl"), ((1, 9, 40), "cl"), ((2, 13, 17), "nchw")])
def test_convex_upsample_fwd_bwd(cuda, shape, layout):
    """channels-last masks take the row-segment kernels (16 pixels per workgroup, partial last
    segment at W = 17 / 40), NCHW masks the per-pixel ones."""
    torch.manual_seed(3)
    from raft_ros_amd.ops.upsample import convex_upsample

    B, H, W = shape
    fmt = torch.channels_last if layout == "cl" else torch.contiguous_format
    flow = torch.randn(B, 2, H, W, device=cuda, requires_grad=True)
    mask = torch.randn(B, 576, H, W, device=cuda).contiguous(memory_format=fmt).requires_grad_(True)
    out = convex_upsample(flow, mask)
    want = ref.convex_upsample(flow, mask)
    torch.testing.assert_close(out, want, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(out)
    df, dm = torch.autograd.grad(out, (flow, mask), g)
    rf, rm = torch.autograd.grad(want, (flow, mask), g)
    torch.testing.assert_close(df, rf, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dm, rm, rtol=1e-4, atol=1e-4)
    # bf16 mask (autocast output of the mask head)
    mb = mask.detach().bfloat16()
    torch.testing.assert_close(convex_upsample(flow.detach(), mb), ref.convex_upsample(flow.detach(), mb.float()),
                               rtol=1e-4, atol=1e-4)
    # bf16 backward: dmask in the mask's dtype and layout, the flow gradient in fp32
    dfb, dmb = _ops().convex_upsample_backward(flow.detach(), mb, g)
    assert dmb.dtype == torch.bfloat16 and dmb.stride() == mb.stride()
    mf = mb.float().requires_grad_(True)
    rfb, rmb = torch.autograd.grad(ref.convex_upsample(flow, mf), (flow, mf), g)
    torch.testing.assert_close(dfb, rfb, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(dmb.float(), rmb, rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gru_gates_and_blend(cuda, dtype):
    torch.manual_seed(4)
    from raft_ros_amd.ops import gru

    B, C, H, W = 2, 128, 9, 11
    cl = torch.channels_last
    zr = torch.randn(B, 2 * C, H, W, device=cuda).to(dtype).contiguous(memory_format=cl).requires_grad_(True)
    h = torch.randn(B, C, H, W, device=cuda).to(dtype).contiguous(memory_format=cl).requires_grad_(True)
    q = torch.randn(B, C, H, W, device=cuda).to(dtype).contiguous(memory_format=cl).requires_grad_(True)
    z, rh = gru.gates_zr(zr, h)
    out = gru.blend(z, q, h)
    zr32, h32, q32 = (t.detach().float().requires_grad_(True) for t in (zr, h, q))
    zz = torch.sigmoid(zr32[:, :C])
    rr = torch.sigmoid(zr32[:, C:]) * h32
    want = (1 - zz) * h32 + zz * torch.tanh(q32)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(rh.float(), rr, **tol)
    torch.testing.assert_close(out.float(), want, **tol)
    g = torch.randn_like(want)
    got = torch.autograd.grad(out, (zr, h, q), g.to(dtype))
    exp = torch.autograd.grad(want, (zr32, h32, q32), g)
    for a, b in zip(got, exp):
        torch.testing.assert_close(a.float(), b, **tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_local_corr_fwd_bwd(cuda, dtype):
    torch.manual_seed(5)
    from raft_ros_amd.ops.corr import _LocalCorr

    B, C, H1, W1, H2, W2, r = 2, 64, 11, 13, 6, 7, 4
    f1 = torch.randn(B, H1, W1, C, device=cuda).to(dtype).requires_grad_(True)
    f2 = torch.randn(B, H2, W2, C, device=cuda).to(dtype).requires_grad_(True)
    coords = (ref.coords_grid(B, H1, W1, cuda) / 2 + 2 * torch.randn(B, 2, H1, W1, device=cuda)).contiguous()
    scale = 1 / math.sqrt(C)
    out = _LocalCorr.apply(f1, f2, coords, r, scale)
    f1r = f1.detach().float().permute(0, 3, 1, 2).requires_grad_(True)
    f2r = f2.detach().float().permute(0, 3, 1, 2).requires_grad_(True)
    want = ref.local_corr(f1r, f2r, coords, r).permute(0, 2, 3, 1) * scale
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(out, want, **tol)
    g = torch.randn_like(want)
    d1, d2 = torch.autograd.grad(out, (f1, f2), g)
    r1, r2 = torch.autograd.grad(want, (f1r, f2r), g)
    torch.testing.assert_close(d1.float(), r1.permute(0, 2, 3, 1), **tol)
    torch.testing.assert_close(d2.float(), r2.permute(0, 2, 3, 1), **tol)


@pytest.mark.parametrize("C,relu,dtype", [(64, True, torch.bfloat16), (96, False, torch.float32), (128, True, torch.float32)])
def test_instance_norm_nhwc(cuda, C, relu, dtype):
    torch.manual_seed(6)
    from raft_ros_amd.ops.norm import InstanceNorm2dNHWC

    x = (torch.randn(3, C, 37, 29, device=cuda) * 2 + 0.5).to(dtype).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = InstanceNorm2dNHWC(C)(x, relu=relu)
    xr = x.detach().float().requires_grad_(True)
    yr = torch.nn.functional.instance_norm(xr)
    if relu:
        yr = torch.relu(yr)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(y.float(), yr, **tol)
    g = torch.randn_like(yr)
    (dx,) = torch.autograd.grad(y, x, g.to(dtype))
    (dxr,) = torch.autograd.grad(yr, xr, g)
    torch.testing.assert_close(dx.float(), dxr, **tol)


@pytest.mark.parametrize("C,r", [(256, 4), (128, 3)], ids=["base", "small"])
@pytest.mark.parametrize("jitter", [3.0, 40.0])  # smooth flow (one window chunk) / wild flow (many chunks)
def test_local_corr_mfma_matches_dense_reference(cuda, jitter, C, r):
    """MFMA local correlation (all levels, one launch) vs the dense reference pyramid lookup,
    forward and both feature gradients (bf16 operands -> bf16-level tolerance).  The fmap2
    gradient comes from the gather backward (per-block query lists; the coarse levels' lists
    exceed one 512-query segment, so its atomic path runs too)."""
    torch.manual_seed(8)
    from raft_ros_amd.ops.corr import LocalCorrPyramid

    B, H, W = 2, 23, 37
    f1 = torch.randn(B, C, H, W, device=cuda).bfloat16().float().requires_grad_(True)
    f2 = torch.randn(B, C, H, W, device=cuda).bfloat16().float().requires_grad_(True)
    coords = ref.coords_grid(B, H, W, cuda) + jitter * torch.randn(B, 2, H, W, device=cuda)
    lc = LocalCorrPyramid(f1, f2, 4, r, split=False)
    assert lc.mfma
    out = lc(coords)
    f1r = f1.detach().clone().requires_grad_(True)
    f2r = f2.detach().clone().requires_grad_(True)
    want = ref.pyramid_lookup(ref.build_pyramid(ref.corr_volume(f1r, f2r), 4), coords, r)
    assert ((out - want).norm() / want.norm()).item() < 1e-2
    g = torch.randn_like(want)
    (out * g).sum().backward()
    (want * g).sum().backward()
    for got, exp in ((f1.grad, f1r.grad), (f2.grad, f2r.grad)):
        assert ((got - exp).norm() / exp.norm()).item() < 2e-2
    # padded fused layout: zeros beyond the 324 taps
    padded = lc.lookup_padded(coords, 328)
    assert padded.shape == (B, H, W, 328) and (padded[..., 324:] == 0).all()


@pytest.mark.parametrize("jitter", [3.0, 40.0])
def test_local_corr_split_mfma_inference_is_fp32_faithful(cuda, jitter):
    """fp32 inference of the alternate correlation on the MFMA kernel with split-bf16 operands
    ([hi | lo | hi] . [hi | hi | lo] along K) == the fp32 dense reference lookup to ~1e-5."""
    torch.manual_seed(9)
    from raft_ros_amd.ops.corr import LocalCorrPyramid

    B, C, H, W, r = 2, 256, 23, 37, 4
    f1 = torch.randn(B, C, H, W, device=cuda)
    f2 = torch.randn(B, C, H, W, device=cuda)
    coords = ref.coords_grid(B, H, W, cuda) + jitter * torch.randn(B, 2, H, W, device=cuda)
    with torch.no_grad():
        lc = LocalCorrPyramid(f1, f2, 4, r, split=True)
        assert lc.mfma and lc.split_mfma
        out = lc(coords)
        want = ref.pyramid_lookup(ref.build_pyramid(ref.corr_volume(f1, f2), 4), coords, r)
    err = ((out - want).norm() / want.norm()).item()
    print(f"\nsplit-MFMA local corr rel err {err:.2e}")
    assert err < 3e-5
    # with autograd the exact scalar kernel keeps training fp32
    assert not LocalCorrPyramid(f1.requires_grad_(True), f2, 4, r, split=True).mfma


@pytest.mark.parametrize("hw", [(1, 1), (5, 7), (46, 62)])
def test_upflow8_matches_reference_fwd_bwd(hw):
    from raft_ros_amd.ops import reference as ref
    from raft_ros_amd.ops._ext import ops

    cuda = torch.device("cuda", 0)
    H, W = hw
    g = torch.Generator(device=cuda).manual_seed(3)
    flow = torch.randn(2, 2, H, W, device=cuda, generator=g)
    out = ops().upflow8(flow)
    fr = flow.clone().requires_grad_(True)
    r = ref.upflow8(fr)
    torch.testing.assert_close(out, r, rtol=1e-5, atol=2e-4)  # fma contraction vs ATen's order
    go = torch.randn(r.shape, device=cuda, generator=g)
    r.backward(go)
    rows = torch.empty(2 * H * W, 8, device=cuda, dtype=torch.bfloat16)
    d = ops().upflow8_backward(go, H, W, rows)
    torch.testing.assert_close(d, fr.grad, rtol=1e-4, atol=1e-3)
    got = rows.float().reshape(2, H, W, 8)
    torch.testing.assert_close(got[..., :2], fr.grad.permute(0, 2, 3, 1), rtol=1e-2, atol=1e-2)
    assert (got[..., 2:] == 0).all()


@pytest.mark.parametrize("alt", [False, True])
def test_training_step_bitwise_deterministic(alt):
    """torch.use_deterministic_algorithms(True): two identical training steps give bitwise
    identical gradients (every native backward is atomic-free or uses order-independent
    fixed-point integer atomics)."""
    from argparse import Namespace
    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.train.loss import sequence_loss

    cuda = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16", alternate_corr=alt)).to(cuda)
    model = model.to(memory_format=torch.channels_last).train()
    model.freeze_bn()
    batch = synthetic_batch(2, 128, 192, seed=4, device=cuda)
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        grads = []
        for _ in range(2):
            model.zero_grad(set_to_none=True)
            loss, _ = sequence_loss(model(batch[0], batch[1], iters=3), batch[2], batch[3])
            loss.backward()
            grads.append([p.grad.clone() for p in model.parameters()])
    finally:
        torch.use_deterministic_algorithms(prev)
    for (n, _), a, b in zip(model.named_parameters(), grads[0], grads[1]):
        assert torch.equal(a, b), n


@pytest.mark.parametrize("split", [True, False])  # scalar fp32 kernel / MFMA kernel
@pytest.mark.parametrize("gscale", [1.0, 1e-7])
def test_deterministic_local_corr_grads_match_float_atomics(split, gscale):
    """The deterministic (fixed-point integer atomic) dF2 accumulation vs the float-atomic one,
    at unit-scale and at realistic loss-gradient magnitudes (a sequence loss over 8x368x496
    puts ~1e-7 on each correlation tap): the fixed-point scale is chosen per tensor, so the
    deterministic gradient keeps fp32-level accuracy at both."""
    from raft_ros_amd.ops import LocalCorrPyramid
    from raft_ros_amd.ops.reference import coords_grid

    cuda = torch.device("cuda", 0)
    g = torch.Generator(device=cuda).manual_seed(5)
    B, C, H, W = 2, 256, 24, 32
    f1 = torch.randn(B, C, H, W, device=cuda, generator=g)
    f2 = torch.randn(B, C, H, W, device=cuda, generator=g)
    coords = coords_grid(B, H, W, device=cuda) + 3 * torch.randn(B, 2, H, W, device=cuda, generator=g)
    gout = None
    grads = {}
    prev = torch.are_deterministic_algorithms_enabled()
    try:
        for det in (False, True):
            torch.use_deterministic_algorithms(det, warn_only=True)
            a, b = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
            out = LocalCorrPyramid(a, b, radius=4, split=split)(coords, out_dtype=torch.float32)
            if gout is None:
                gout = torch.randn(out.shape, device=cuda, generator=g) * gscale
            out.backward(gout)
            grads[det] = b.grad.detach().clone()
    finally:
        torch.use_deterministic_algorithms(prev)
    ref, det = grads[False], grads[True]
    rel = ((det - ref).norm() / ref.norm()).item()
    assert ref.norm() > 0 and rel < 1e-5, rel
