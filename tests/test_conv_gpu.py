"""Implicit-GEMM NHWC conv kernels vs torch.nn.functional.conv2d in fp32."""
import pytest
import torch
import torch.nn.functional as F

from raft_ros_amd.ops import conv as C

pytestmark = pytest.mark.gpu


def _pm(t):
    """(B, C, H, W) -> bf16 pixel-major (P, C) contiguous."""
    B, Ch, H, W = t.shape
    return t.permute(0, 2, 3, 1).reshape(B * H * W, Ch).to(torch.bfloat16).contiguous()


def _from_pm(t, B, H, W):
    return t.reshape(B, H, W, -1).permute(0, 3, 1, 2).float()


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-6)).item()


CASES = [
    # (Cin segments (real, padded), Cout, kh, kw, act)
    ([(256, 256)], 192, 3, 3, 1),
    ([(128, 128), (128, 128), (128, 128)], 256, 1, 5, 0),
    ([(128, 128), (256, 256)], 128, 5, 1, 0),
    ([(2, 8)], 128, 7, 7, 1),
    ([(324, 328)], 256, 1, 1, 1),
    ([(256, 256)], 2, 3, 3, 0),
    ([(128, 128)], 2, 3, 3, 0),
    ([(256, 256)], 576, 1, 1, 0),
]


@pytest.mark.parametrize("segs,cout,kh,kw,act", CASES)
def test_conv_fwd_dgrad_wgrad(cuda, segs, cout, kh, kw, act):
    torch.manual_seed(0)
    B, H, W = 2, 13, 19
    ph, pw = kh // 2, kw // 2
    cin = sum(r for r, _ in segs)
    x_parts = [torch.randn(B, r, H, W, device=cuda) for r, _ in segs]
    w = torch.randn(cout, cin, kh, kw, device=cuda) / (cin * kh * kw) ** 0.5
    bias = torch.randn(cout, device=cuda)
    # bf16-rounded operands for the fp32 reference
    xr = torch.cat([p.bfloat16().float() for p in x_parts], dim=1).requires_grad_(True)
    wr = w.bfloat16().float().requires_grad_(True)
    br = bias.clone().requires_grad_(True)
    y = F.conv2d(xr, wr, br, padding=(ph, pw))
    if act:
        y = F.relu(y)

    P = B * H * W
    srcs = []
    for (r, pd), part in zip(segs, x_parts):
        buf = torch.zeros(P, pd, device=cuda, dtype=torch.bfloat16)
        buf[:, :r] = _pm(part)
        srcs.append(buf)
    g = C.geom(B, H, W, kh, kw, ph, pw)
    wt = C.pack_fwd(w, segs)
    # forward, written into a channel slice of a wider buffer
    outbuf = torch.zeros(P, (cout + 7) // 8 * 8 + 8, device=cuda, dtype=torch.bfloat16)
    C.conv_fwd(srcs, wt, g, cout, outbuf[:, :cout], bias=bias, act=act)
    got = _from_pm(outbuf[:, :cout], B, H, W)
    assert _rel(got, y) < 1e-2, _rel(got, y)
    assert (outbuf[:, cout:] == 0).all()

    # backward
    gy = torch.randn_like(y)
    if act:
        gy = gy * (y > 0)
    y.backward(gy)
    cout_p = (cout + 7) // 8 * 8
    dy = torch.zeros(P, cout_p, device=cuda, dtype=torch.bfloat16)
    dy[:, :cout] = _pm(gy)
    # data grad
    cin_p = sum(p for _, p in segs)
    wtd = C.pack_dgrad(w, segs, cout_p)
    dx = torch.zeros(P, cin_p, device=cuda, dtype=torch.float32)
    C.conv_fwd([dy], wtd, C.geom(B, H, W, kh, kw, kh - 1 - ph, kw - 1 - pw), cin_p, dx, epi=C.EPI_GRAD)
    dx_real = torch.cat([dx[:, o:o + r] for o, (r, _) in zip(
        [sum(p for _, p in segs[:i]) for i in range(len(segs))], segs)], dim=1)
    assert _rel(_from_pm(dx_real, B, H, W), xr.grad) < 1e-2
    # weight + bias grad (accumulated twice -> 2x)
    dw = torch.zeros(cout, wt.shape[1], device=cuda)
    db = torch.zeros(cout, device=cuda)
    C.conv_wgrad(srcs, dy, g, cout, dw, db)
    C.conv_wgrad(srcs, dy, g, cout, dw, db)
    gw = C.unpack_grad(dw, w.shape, segs)
    assert _rel(gw, 2 * wr.grad) < 1e-2, _rel(gw, 2 * wr.grad)
    assert _rel(db, 2 * dy.float().sum(0)[:cout]) < 1e-4


@pytest.mark.parametrize("segs,cout,kh,kw", [([(128, 128), (128, 128), (128, 128)], 256, 1, 5),
                                              ([(324, 328)], 256, 1, 1), ([(128, 128)], 64, 3, 3)])
def test_wgrad_full_size_split_paths(cuda, segs, cout, kh, kw):
    """RAFT-sized pixel counts take the XCD-grouped split-K mapping and the fused bias sum."""
    torch.manual_seed(3)
    B, H, W = 8, 46, 62
    P = B * H * W
    cin = sum(r for r, _ in segs)
    srcs = [torch.zeros(P, pd, device=cuda, dtype=torch.bfloat16) for _, pd in segs]
    for (r, _), buf in zip(segs, srcs):
        buf[:, :r] = torch.randn(P, r, device=cuda).bfloat16()
    dy = torch.randn(P, cout, device=cuda).bfloat16()
    w = torch.zeros(cout, cin, kh, kw, device=cuda)
    wt = C.pack_fwd(w, segs)
    dw = torch.zeros(cout, wt.shape[1], device=cuda)
    db = torch.zeros(cout, device=cuda)
    C.conv_wgrad(srcs, dy, C.geom(B, H, W, kh, kw, kh // 2, kw // 2), cout, dw, db)
    x = torch.cat([_from_pm(buf[:, :r], B, H, W) for (r, _), buf in zip(segs, srcs)], dim=1)
    wr = torch.zeros(cout, cin, kh, kw, device=cuda, requires_grad=True)
    y = F.conv2d(x, wr, padding=(kh // 2, kw // 2))
    y.backward(_from_pm(dy, B, H, W))
    assert _rel(C.unpack_grad(dw, w.shape, segs), wr.grad) < 1e-3
    assert _rel(db, dy.float().sum(0)) < 1e-4


def test_dgrad_relu_mask_and_partial_accumulate(cuda):
    torch.manual_seed(1)
    B, H, W, cin, cout = 1, 9, 10, 64, 32
    P = B * H * W
    x = torch.randn(P, cin, device=cuda).bfloat16()
    w = torch.randn(cout, cin, 3, 3, device=cuda) * 0.1
    dy = torch.randn(P, cout, device=cuda).bfloat16()
    base = torch.randn(P, cin, device=cuda)
    out = base.clone()
    C.conv_fwd([dy], C.pack_dgrad(w), C.geom(B, H, W, 3, 3, 1, 1), cin, out, epi=C.EPI_GRAD, acc_c0=32, mask=x)
    xr = _from_pm(x, B, H, W).requires_grad_(True)
    y = F.conv2d(xr, w.bfloat16().float(), padding=1)
    y.backward(_from_pm(dy, B, H, W))
    ref = xr.grad.permute(0, 2, 3, 1).reshape(P, cin) * (x.float() > 0)
    ref[:, 32:] += base[:, 32:]
    assert _rel(out, ref) < 1e-2


def test_gru_epilogues(cuda):
    torch.manual_seed(2)
    B, H, W, Ch = 2, 7, 11, 128
    P = B * H * W
    hx = torch.randn(P, 3 * Ch, device=cuda).bfloat16()  # [h | x]
    h = hx[:, :Ch]
    wzr = torch.randn(2 * Ch, 3 * Ch, 1, 5, device=cuda) * 0.05
    bzr = torch.randn(2 * Ch, device=cuda) * 0.1
    g = C.geom(B, H, W, 1, 5, 0, 2)
    zr = torch.empty(P, 2 * Ch, device=cuda, dtype=torch.bfloat16)
    rh = torch.empty(P, Ch, device=cuda, dtype=torch.bfloat16)
    C.conv_fwd([hx], C.pack_fwd(wzr), g, 2 * Ch, zr, bias=bzr, epi=C.EPI_GRU_ZR, h=h, out2=rh)
    hxf = _from_pm(hx, B, H, W)
    pre = F.conv2d(hxf, wzr.bfloat16().float(), bzr, padding=(0, 2))
    sig = torch.sigmoid(pre)
    assert _rel(_from_pm(zr, B, H, W), sig) < 1e-2
    rh_ref = sig[:, Ch:] * hxf[:, :Ch]
    assert _rel(_from_pm(rh, B, H, W), rh_ref) < 1e-2
    # candidate + blend: sources [rh | x]
    wq = torch.randn(Ch, 3 * Ch, 1, 5, device=cuda) * 0.05
    bq = torch.randn(Ch, device=cuda) * 0.1
    hn = torch.empty(P, Ch, device=cuda, dtype=torch.bfloat16)
    q = torch.empty(P, Ch, device=cuda, dtype=torch.bfloat16)
    z = zr[:, :Ch]
    C.conv_fwd([rh, hx[:, Ch:]], C.pack_fwd(wq), g, Ch, hn, bias=bq, epi=C.EPI_GRU_Q, h=h, z=z, out2=q)
    rx = torch.cat([_from_pm(rh, B, H, W), hxf[:, Ch:]], dim=1)
    qr = torch.tanh(F.conv2d(rx, wq.bfloat16().float(), bq, padding=(0, 2)))
    zf = _from_pm(z, B, H, W)
    hn_ref = (1 - zf) * hxf[:, :Ch] + zf * qr
    assert _rel(_from_pm(q, B, H, W), qr) < 1e-2
    assert _rel(_from_pm(hn, B, H, W), hn_ref) < 1e-2


@pytest.mark.parametrize("cfg", [20, 21, 24, 25, 26, 1, 8, 9, 41, 45, 59, 60, 61, 62, 63, 64, 65, 67, 74, 75])
@pytest.mark.parametrize("segs,cout,kh,kw,hw", [
    ([(256, 256)], 192, 3, 3, (46, 62)),
    ([(128, 128), (128, 128), (128, 128)], 256, 1, 5, (46, 62)),
    ([(128, 128), (128, 128), (128, 128)], 128, 5, 1, (46, 62)),
    ([(128, 128)], 512, 3, 3, (23, 31)),
    ([(64, 64)], 128, 3, 3, (17, 21)),
    ([(128, 128), (128, 128), (128, 128)], 128, 5, 1, (27, 120)),
    ([(128, 128)], 256, 3, 3, (27, 120)),
    ([(324, 328)], 256, 1, 1, (46, 62)),   # convc1 (the lookup rows: 324 taps + 4 pad channels)
    ([(256, 256)], 576, 1, 1, (46, 62)),   # mask.2
    ([(576, 576)], 256, 1, 1, (23, 31)),   # mask.2 data gradient
    ([(256, 256)], 328, 1, 1, (27, 120)),  # convc1 data gradient
])
def test_fwd_every_variant_full_size(cuda, cfg, segs, cout, kh, kw, hw):
    """Every forward kernel variant (v6 / v5 halo-strip tiles, v4 tiles, generic) at RAFT
    sizes vs an fp32 conv2d."""
    torch.manual_seed(4)
    B, (H, W) = 8, hw
    P = B * H * W
    cin = sum(r for r, _ in segs)
    srcs = [torch.randn(P, pd, device=cuda).bfloat16() for _, pd in segs]
    w = torch.randn(cout, cin, kh, kw, device=cuda) / (cin * kh * kw) ** 0.5
    bias = torch.randn(cout, device=cuda)
    out = torch.full((P, cout), float("nan"), device=cuda, dtype=torch.bfloat16)
    # v6 flat strips: BM + (kh - 1) W + kw - 1 rows must fit the LDS strip buffer
    v6_flat = {41: (256, 479), 45: (256, 447)}
    if cfg in v6_flat and v6_flat[cfg][0] + (kh - 1) * W + kw - 1 > v6_flat[cfg][1]:
        pytest.skip("v6 flat strip does not fit in LDS at this width (2-D tiles cover it)")
    # v6 tap shapes: 45 = 3x3 / 1x5, 59 (2-D) = 3x3 / 1x5, 60 (2-D) = 5x1, 61 (2-D) = 3x3 / 5x1
    # 62 / 63 (128 x 64 2-D tiles, two workgroups per CU) = every tap shape, 64 = 5x1; 74 / 75
    # (64 x 64 2-D tiles, three workgroups per CU) = every tap shape
    if ((cfg in (60, 64) and (kh, kw) != (5, 1)) or (cfg in (45, 59) and (kh, kw) not in ((3, 3), (1, 5)))
            or (cfg == 65 and (kh, kw) != (1, 5)) or (cfg == 67) != ((kh, kw) == (1, 1)) and cfg >= 41
            or (cfg == 61 and (kh, kw) not in ((3, 3), (5, 1)))):
        pytest.skip("v6 variant built for other tap shapes")
    C.conv_fwd(srcs, C.pack_fwd(w, segs), C.geom(B, H, W, kh, kw, kh // 2, kw // 2), cout, out, bias=bias, act=1,
               cfg=cfg)
    x = torch.cat([_from_pm(s, B, H, W)[:, :r] for s, (r, _) in zip(srcs, segs)], dim=1)  # pad channels unread
    ref = F.relu(F.conv2d(x, w.bfloat16().float(), bias, padding=(kh // 2, kw // 2)))
    assert _rel(_from_pm(out, B, H, W), ref) < 1e-2


@pytest.mark.parametrize("segs,couts,kh,kw", [([(128, 128), (128, 128), (128, 128)], (128, 128), 1, 5),
                                               ([(324, 328)], (256,), 1, 1), ([(2, 8)], (128,), 7, 7),
                                               ([(128, 128)], (256, 256), 3, 3), ([(256, 256)], (2,), 3, 3)])
def test_pack_weights_matches_python_packing(cuda, segs, couts, kh, kw):
    torch.manual_seed(5)
    cin = sum(r for r, _ in segs)
    ws = [torch.randn(c, cin, kh, kw, device=cuda).to(memory_format=torch.channels_last) for c in couts]
    bs = [torch.randn(c, device=cuda) for c in couts]
    wf, wd, b = C.pack_weights(ws, bs, segs, scale=0.25)
    wcat = torch.cat(ws, 0)
    assert torch.equal(wf, C.pack_fwd(wcat, segs, scale=0.25))
    assert torch.equal(wd, C.pack_dgrad(wcat, segs, scale=0.25))
    torch.testing.assert_close(b, torch.cat(bs) * 0.25)


def test_wgrad_params_periodic_source_and_param_layout(cuda):
    """Batched weight gradient over T iterations: a periodic (shared) source equals the
    per-iteration sum; stacked parameters get their own (channels-last) gradients."""
    torch.manual_seed(6)
    T, B, H, W = 3, 2, 11, 13
    P = B * H * W
    segs = [(128, 128), (128, 128), (128, 128)]
    hs = torch.randn(T * P, 128, device=cuda).bfloat16()
    inp = torch.randn(P, 128, device=cuda).bfloat16()  # shared by every iteration
    mo = torch.randn(T * P, 128, device=cuda).bfloat16()
    dy = torch.randn(T * P, 256, device=cuda).bfloat16()
    gz = torch.empty(128, 384, 1, 5, device=cuda).to(memory_format=torch.channels_last)
    gr = torch.empty_like(gz)
    bz = torch.empty(128, device=cuda)
    br = torch.empty(128, device=cuda)
    C.conv_wgrad_params([hs, inp, mo], dy, C.geom(T * B, H, W, 1, 5, 0, 2), [gz, gr], [bz, br], segs, scale=0.5)
    ref_w = torch.zeros(256, 384, 1, 5, device=cuda)
    for t in range(T):
        sl = slice(t * P, (t + 1) * P)
        x = torch.cat([_from_pm(hs[sl], B, H, W), _from_pm(inp, B, H, W), _from_pm(mo[sl], B, H, W)], 1)
        wr = torch.zeros(256, 384, 1, 5, device=cuda, requires_grad=True)
        F.conv2d(x, wr, padding=(0, 2)).backward(_from_pm(dy[sl], B, H, W))
        ref_w += wr.grad
    assert _rel(torch.cat([gz, gr]), 0.5 * ref_w) < 1e-3
    assert _rel(torch.cat([bz, br]), 0.5 * dy.float().sum(0)) < 1e-4
    # deterministic: a second run is bitwise identical
    gz2 = torch.empty_like(gz)
    C.conv_wgrad_params([hs, inp, mo], dy, C.geom(T * B, H, W, 1, 5, 0, 2), [gz2, gr], [bz, br], segs, scale=0.5)
    assert torch.equal(gz, gz2)


@pytest.mark.parametrize("cfg", [0, 8, 25, 26, 41, 59, 62, 74, 75])
def test_gru_backward_epilogues_match_unfused(cuda, cfg):
    """EPI_GRU_BWD_A / _B / _LAST (gate backward fused into the data-gradient epilogue) vs
    the plain EPI_GRAD store followed by the separate gru_bwd_a / gru_bwd_b / masked_cast
    kernels, on a 1x5 conv with 384 output channels (the GRU data-gradient shape)."""
    from raft_ros_amd.ops._ext import ops

    k = ops()
    torch.manual_seed(11)
    B, H, W, HID = 2, 23, 31, 128
    P = B * H * W
    dy = torch.randn(P, 256, device=cuda).bfloat16()
    wt = C.pack_fwd(torch.randn(3 * HID, 256, 1, 5, device=cuda) * 0.05, [(256, 256)])
    g = C.geom(B, H, W, 1, 5, 0, 2)
    G0 = torch.randn(P, 3 * HID, device=cuda)
    rnd = lambda: torch.rand(P, HID, device=cuda).bfloat16()  # noqa: E731
    z, q, h, r = rnd(), (torch.rand(P, HID, device=cuda) * 2 - 1).bfloat16(), rnd(), rnd()
    bf = torch.bfloat16

    def plain(acc_c0):
        out = G0.clone()
        C.conv_fwd([dy], wt, g, 3 * HID, out, epi=C.EPI_GRAD, acc_c0=acc_c0, cfg=cfg)
        return out

    def close(a, b, tol=2e-2):
        assert _rel(a.float(), b.float()) < tol

    # A: dH accumulated into G, gate backward in the epilogue; channels >= 128 as EPI_GRAD
    Gp = plain(0)
    dq_r, dz_r, c_r = (torch.empty(P, HID, device=cuda, dtype=bf), torch.empty(P, HID, device=cuda, dtype=bf),
                       torch.empty(P, HID, device=cuda))
    k.gru_bwd_a(Gp[:, :HID], z, q, h, dq_r, dz_r, c_r)
    Gf = G0.clone()
    dq, dz, carry = torch.empty_like(dq_r), torch.empty_like(dz_r), torch.empty_like(c_r)
    C.conv_fwd([dy], wt, g, 3 * HID, Gf, epi=C.EPI_GRU_BWD_A, acc_c0=0, h=h, z=z, g0=q, out2=dq, out3=dz,
               carry=carry, gru_cols=HID, cfg=cfg)
    close(dq, dq_r)
    close(dz, dz_r)
    close(carry, c_r, 1e-5)
    assert torch.equal(Gf[:, HID:], Gp[:, HID:])
    # A with an incoming bf16 gradient and no accumulation
    add = torch.randn(P, HID, device=cuda).bfloat16()
    Gq = G0.clone()
    C.conv_fwd([dy], wt, g, 3 * HID, Gq, epi=C.EPI_GRU_BWD_A, acc_c0=1 << 30, h=h, z=z, g0=q, out2=dq, out3=dz,
               carry=carry, gru_cols=HID, addsrc=add, cfg=cfg)
    Gp2 = plain(1 << 30)
    k.gru_bwd_a(Gp2[:, :HID] + add.float(), z, q, h, dq_r, dz_r, c_r)
    close(dq, dq_r)
    close(carry, c_r, 1e-5)
    # B: d(r h) fresh in channels < 128, accumulated above
    Gp = plain(HID)
    dr_r = torch.empty(P, HID, device=cuda, dtype=bf)
    c_in = torch.randn(P, HID, device=cuda)
    k.gru_bwd_b(Gp[:, :HID], r, h, c_in, dr_r)
    Gf = G0.clone()
    dr = torch.empty_like(dr_r)
    C.conv_fwd([dy], wt, g, 3 * HID, Gf, epi=C.EPI_GRU_BWD_B, acc_c0=HID, h=h, g0=r, carry=c_in, out3=dr,
               gru_cols=HID, cfg=cfg)
    close(dr, dr_r)
    close(Gf, Gp, 1e-5)
    # LAST: bf16 d net, fp32 d inp, masked bf16 d motion
    Gp = plain(0)
    motion = torch.randn(P, HID, device=cuda).bfloat16()
    dmo_r = torch.empty(P, HID, device=cuda, dtype=bf)
    k.masked_cast(Gp[:, 2 * HID:2 * HID + 126], motion, dmo_r)
    Gf = G0.clone()
    dnet, dmo = torch.empty(P, HID, device=cuda, dtype=bf), torch.full((P, HID), 7.0, device=cuda, dtype=bf)
    C.conv_fwd([dy], wt, g, 3 * HID, Gf, epi=C.EPI_GRU_BWD_LAST, acc_c0=0, out3=dnet, gru_cols=HID, cout=dmo,
               cmask=motion, cm_c0=2 * HID, cm_valid=126, cfg=cfg)
    assert torch.equal(dnet, Gp[:, :HID].bfloat16())
    assert torch.equal(Gf[:, HID:2 * HID], Gp[:, HID:2 * HID])
    assert torch.equal(dmo, dmo_r)


def _split_read(buf, G, n):
    """hi + lo planes of channels [0, n) of a group-G split row buffer -> fp32 (P, n)."""
    parts = []
    for g0 in range(0, n, G):
        base = (g0 // G) * 3 * G
        w = min(G, n - g0)
        parts.append(buf[:, base:base + w].float() + buf[:, base + G:base + G + w].float())
    return torch.cat(parts, 1)


@pytest.mark.parametrize("segs,cout,kh,kw,act,G", [
    ([(256, 256)], 192, 3, 3, 1, 256),   # convc2 into a 256-wide group
    ([(2, 8)], 128, 7, 7, 1, 128),       # convf1 on the padded flow operand
    ([(324, 328)], 256, 1, 1, 1, 256),   # convc1 on the correlation features
    ([(128, 128)], 512, 3, 3, 1, 256),   # the fused heads conv, two 256-groups
])
def test_split_conv_is_fp32_faithful(cuda, segs, cout, kh, kw, act, G):
    """Split-bf16 mode (fp32 inference): a conv over [hi | lo | hi] operands against
    [W_hi | W_hi | W_lo] equals the fp32 conv to ~1e-5 relative (vs ~4e-3 for plain bf16)."""
    torch.manual_seed(0)
    B, H, W = 2, 13, 19
    P = B * H * W
    cin = sum(r for r, _ in segs)
    cpad = sum(p for _, p in segs)
    x = torch.randn(B, cin, H, W, device=cuda)
    w = torch.randn(cout, cin, kh, kw, device=cuda) / (cin * kh * kw) ** 0.5
    bias = torch.randn(cout, device=cuda)
    ref = F.conv2d(x, w, bias, padding=(kh // 2, kw // 2))
    if act:
        ref = F.relu(ref)
    xs = torch.zeros(P, 3 * cpad, device=cuda, dtype=torch.bfloat16)
    C.split_pack(x.permute(0, 2, 3, 1).reshape(P, cin).contiguous(), xs, cpad, 0, cpad)
    wf, b = C.pack_weights_split([w], [bias], [segs])
    out = torch.zeros(P, C.split_planes(cout, G), device=cuda, dtype=torch.bfloat16)
    C.conv_fwd([xs], wf, C.geom(B, H, W, kh, kw, kh // 2, kw // 2), cout, out, bias=b, act=act, split=[G, 0, 0, 0])
    got = _from_pm(_split_read(out, G, cout), B, H, W)
    err = _rel(got, ref)
    assert err < 3e-5, err


def test_split_gru_stage_is_fp32_faithful(cuda):
    """One SepConvGRU stage (z||r 1x5 with sigmoid / r*h epilogue, q 1x5 with tanh + blend)
    in split-bf16 mode vs the fp32 module math (core/update.py:33-60)."""
    torch.manual_seed(1)
    B, H, W, Hd = 2, 11, 23, 128
    P = B * H * W
    h, inp, mo = (torch.randn(B, Hd, H, W, device=cuda) * s for s in (0.5, 1.0, 1.0))
    wz, wr, wq = (torch.randn(Hd, 3 * Hd, 1, 5, device=cuda) * 0.03 for _ in range(3))
    bz, br, bq = (torch.randn(Hd, device=cuda) * 0.1 for _ in range(3))
    hx = torch.cat([h, inp, mo], 1)
    z = torch.sigmoid(F.conv2d(hx, wz, bz, padding=(0, 2)))
    r = torch.sigmoid(F.conv2d(hx, wr, br, padding=(0, 2)))
    q = torch.tanh(F.conv2d(torch.cat([r * h, inp, mo], 1), wq, bq, padding=(0, 2)))
    ref = (1 - z) * h + z * q

    def sp(t):
        buf = torch.empty(P, 3 * Hd, device=cuda, dtype=torch.bfloat16)
        return C.split_pack(t.permute(0, 2, 3, 1).reshape(P, Hd).contiguous(), buf, Hd)

    hs, ins, ms = sp(h), sp(inp), sp(mo)
    src = [[(Hd, Hd)]] * 3
    wzr, bzr = C.pack_weights_split([wz, wr], [bz, br], src)
    wqp, bqp = C.pack_weights_split([wq], [bq], src)
    g = C.geom(B, H, W, 1, 5, 0, 2)
    zr = torch.empty(P, 6 * Hd, device=cuda, dtype=torch.bfloat16)
    rh = torch.empty(P, 3 * Hd, device=cuda, dtype=torch.bfloat16)
    hn = torch.empty(P, 3 * Hd, device=cuda, dtype=torch.bfloat16)
    C.conv_fwd([hs, ins, ms], wzr, g, 2 * Hd, zr, bias=bzr, epi=C.EPI_GRU_ZR, h=hs, out2=rh, split=[Hd, Hd, Hd, 0])
    C.conv_fwd([rh, ins, ms], wqp, g, Hd, hn, bias=bqp, epi=C.EPI_GRU_Q, h=hs, z=zr, split=[Hd, 0, Hd, Hd])
    got = _from_pm(_split_read(hn, Hd, Hd), B, H, W)
    assert (got - ref).abs().max().item() < 5e-5, (got - ref).abs().max().item()
    assert _rel(_from_pm(_split_read(zr, Hd, 2 * Hd), B, H, W), torch.cat([z, r], 1)) < 3e-5


@pytest.mark.parametrize("cfg", [0, 1, 8, 9, 20, 21, 24, 25, 26, 41, 45, 59, 61, 62, 63, 74, 75])
@pytest.mark.parametrize("N,B,hw", [(256, 2, (46, 62)), (512, 1, (27, 120)), (256, 1, (23, 31))])
def test_flow_head_conv2_folded_into_heads_epilogue(cuda, cfg, N, B, hw):
    """heads conv (3x3 128 -> N, ReLU, bf16) with flow_head.conv2 (3x3 256 -> 2) folded into
    its epilogue as per-tap partials, finished by n2_apply (+ apply_delta), vs fp32 convs of
    the bf16 activations -- for every forward kernel variant that can run the heads conv."""
    from raft_ros_amd.ops._ext import ops

    torch.manual_seed(7)
    H, W = hw
    if cfg in (41, 45) and 256 + 2 * W + 2 > {41: 479, 45: 447}[cfg]:
        pytest.skip("v6 flat strip does not fit in LDS at this width")
    P = B * H * W
    x = torch.randn(P, 128, device=cuda).bfloat16()
    w1 = torch.randn(N, 128, 3, 3, device=cuda) / (128 * 9) ** 0.5
    b1 = torch.randn(N, device=cuda) * 0.1
    w2 = torch.randn(2, 256, 3, 3, device=cuda) / (256 * 9) ** 0.5
    b2 = torch.randn(2, device=cuda)
    hd = torch.full((P, N), float("nan"), device=cuda, dtype=torch.bfloat16)
    y = torch.full((4, 18, P), float("nan"), device=cuda)
    g = C.geom(B, H, W, 3, 3, 1, 1)
    C.conv_fwd([x], C.pack_fwd(w1, [(128, 128)]), g, N, hd, bias=b1, act=1, cfg=cfg,
               n2w=C.pack_fwd(w2, [(256, 256)]), n2y=y)
    coords1 = torch.randn(B, 2, H, W, device=cuda) * 3
    coords_out, flow, delta = torch.empty_like(coords1), torch.empty_like(coords1), torch.empty(P, 8, device=cuda)
    ops().n2_apply(y, b2, coords1, coords_out, flow, delta)
    hd_ref = F.relu(F.conv2d(_from_pm(x, B, H, W), w1.bfloat16().float(), b1, padding=1))
    assert _rel(_from_pm(hd, B, H, W), hd_ref) < 1e-2
    # conv2 over the kernel's own bf16 activations: only the summation order differs
    d_ref = F.conv2d(_from_pm(hd[:, :256], B, H, W), w2.bfloat16().float(), b2, padding=1)
    d = _from_pm(delta[:, :2], B, H, W)
    torch.testing.assert_close(d, d_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(coords_out, coords1 + d, rtol=0, atol=1e-5)
    yy, xx = torch.meshgrid(torch.arange(H, device=cuda), torch.arange(W, device=cuda), indexing="ij")
    torch.testing.assert_close(flow, coords_out - torch.stack([xx, yy]).float()[None], rtol=0, atol=1e-5)


@pytest.mark.parametrize("N", [128, 64])
@pytest.mark.parametrize("B,hw", [(8, (46, 62)), (1, (27, 120)), (2, (13, 19)), (1, (135, 240))])
def test_convf1_direct_7x7_kernel(cuda, N, B, hw):
    """convf1 (7x7, the 2 flow channels of flow8 -> N, ReLU) on its direct halo-tile MFMA
    kernel (automatic choice) vs an fp32 conv2d; the pad channels 2..7 are never read."""
    torch.manual_seed(8)
    H, W = hw
    P = B * H * W
    flow8 = torch.randn(P, 8, device=cuda).mul(4).bfloat16()
    w = torch.randn(N, 2, 7, 7, device=cuda) / 98 ** 0.5
    bias = torch.randn(N, device=cuda)
    out = torch.full((P, N), float("nan"), device=cuda, dtype=torch.bfloat16)
    C.conv_fwd([flow8], C.pack_fwd(w, [(2, 8)]), C.geom(B, H, W, 7, 7, 3, 3), N, out, bias=bias, act=1)
    ref = F.relu(F.conv2d(_from_pm(flow8, B, H, W)[:, :2], w.bfloat16().float(), bias, padding=3))
    assert _rel(_from_pm(out, B, H, W), ref) < 1e-2
    out2 = torch.full((P, N), float("nan"), device=cuda, dtype=torch.bfloat16)
    C.conv_fwd([flow8], C.pack_fwd(w, [(2, 8)]), C.geom(B, H, W, 7, 7, 3, 3), N, out2, bias=bias, act=1, cfg=1)
    assert _rel(out.float(), out2.float()) < 1e-2


@pytest.mark.parametrize("N,B,hw", [(256, 8, (46, 62)), (128, 2, (13, 19)), (256, 1, (27, 120))])
def test_cin8_dgrad_direct_kernel(cuda, N, B, hw):
    """The flow head's conv2 data gradient (3x3, an 8-channel gradient row -> N, ReLU' mask,
    EPI_GRAD) on its direct kernel (automatic choice) vs the generic GEMM kernel (cfg 1) and
    an fp32 conv2d of the flipped weights."""
    torch.manual_seed(9)
    H, W = hw
    P = B * H * W
    dy = torch.randn(P, 8, device=cuda).bfloat16()
    w = torch.randn(8, N, 3, 3, device=cuda) / 72 ** 0.5  # forward conv N -> 8: dgrad maps 8 -> N
    mask = torch.randn(P, N, device=cuda).bfloat16()
    wd = C.pack_dgrad(w, [(N, N)])
    outs = []
    for cfg in (0, 1):
        out = torch.full((P, N), float("nan"), device=cuda, dtype=torch.bfloat16)
        C.conv_fwd([dy], wd, C.geom(B, H, W, 3, 3, 1, 1), N, out, epi=C.EPI_GRAD, mask=mask, cfg=cfg)
        outs.append(_from_pm(out, B, H, W))
    ref = F.conv_transpose2d(_from_pm(dy, B, H, W), w.bfloat16().float(), padding=1)
    ref = ref * (_from_pm(mask, B, H, W) > 0)
    assert _rel(outs[0], ref) < 1e-2
    assert _rel(outs[0], outs[1]) < 1e-2
