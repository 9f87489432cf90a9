"""Fake (meta) kernels for every ``torch.ops.raft_amd`` op.

The HIP implementations are registered for the CUDA dispatch key in
``csrc/*bindings.cpp``; these shape/dtype functions let the same ops run on
``FakeTensor`` / the ``meta`` device (shape inference, ``torch.compile`` tracing,
memory planning) without a GPU.  Mutating ops (schemas returning ``()``) get no-op
fakes.  Reference counterpart: the single pybind11 module of
alt_cuda_corr/correlation.cpp:51-54, which has neither.
"""
from __future__ import annotations

import torch

_registered = False


def _cl(t: torch.Tensor, sizes):
    return t.new_empty(sizes).contiguous(memory_format=torch.channels_last)


def register() -> None:
    global _registered
    if _registered:
        return
    _registered = True
    lib = "raft_amd::"
    fake = torch.library.register_fake

    @fake(lib + "gemm_nt")
    def _(A, B, alpha, out_dtype):
        return A.new_empty((A.shape[0], A.shape[1], B.shape[1]), dtype=out_dtype)

    @fake(lib + "pyramid_unpool")
    def _(G, H, W, segs, blocked=False):
        return G.new_empty((G.shape[0], H * W, G.shape[2]))

    @fake(lib + "avgpool2x2")
    def _(x):
        return x.new_empty((x.shape[0], x.shape[1] // 2, x.shape[2] // 2))

    @fake(lib + "corr_lookup")
    def _(pyramid, coords, radius, out_dtype, out_channels=0):
        win = (2 * radius + 1) ** 2
        och = out_channels if out_channels > 0 else len(pyramid) * win
        B, _, H, W = coords.shape
        return coords.new_empty((B, H, W, och), dtype=out_dtype)

    @fake(lib + "pyramid_operand")
    def _(fmap, segs, ld, blocked, nchw, bf16_out=False):
        B, C = fmap.shape[:2]
        return fmap.new_empty((B, C, ld) if nchw else (B, ld, C), dtype=torch.bfloat16 if bf16_out else torch.float32)

    @fake(lib + "convex_upsample")
    def _(flow, mask):
        B, _, H, W = flow.shape
        return flow.new_empty((B, 2, 8 * H, 8 * W))

    @fake(lib + "convex_upsample_backward")
    def _(flow, mask, grad):
        return torch.empty_like(flow), torch.empty_strided(mask.shape, mask.stride(), dtype=mask.dtype,
                                                           device=mask.device)

    @fake(lib + "seq_loss")
    def _(preds, gt, valid, gamma, max_flow):
        return gt.new_empty((6,))

    @fake(lib + "seq_loss_backward")
    def _(preds, gt, valid, dloss, gamma, max_flow):
        return [torch.empty_like(gt) for _ in preds]

    @fake(lib + "local_corr")
    def _(fmap1, fmap2, coords, radius, scale):
        B, H1, W1, _ = fmap1.shape
        return fmap1.new_empty((B, H1, W1, (2 * radius + 1) ** 2), dtype=torch.float32)

    @fake(lib + "local_corr_backward")
    def _(fmap1, fmap2, coords, grad, radius, scale, deterministic=False):
        return fmap1.new_empty(fmap1.shape, dtype=torch.float32), fmap2.new_empty(fmap2.shape, dtype=torch.float32)

    @fake(lib + "gru_gates")
    def _(zr, h):
        return _cl(h, h.shape), _cl(h, h.shape)

    @fake(lib + "gru_gates_backward")
    def _(zr, h, gz, grh):
        return _cl(zr, zr.shape), _cl(h, h.shape)

    @fake(lib + "gru_blend")
    def _(z, q, h):
        return _cl(h, h.shape)

    @fake(lib + "gru_blend_backward")
    def _(z, q, h, g):
        return _cl(z, z.shape), _cl(q, q.shape), _cl(h, h.shape)

    @fake(lib + "instance_norm_fwd")
    def _(x, relu, eps):
        N, C = x.shape[:2]
        return _cl(x, x.shape), x.new_empty((N, C, 2), dtype=torch.float32)

    @fake(lib + "instance_norm_bwd")
    def _(x, dy, stats, relu):
        return _cl(x, x.shape)

    @fake(lib + "pack_conv_weights_split")
    def _(w, b, segs, scale, Kf, Kd, G_dy):
        n = sum(t.shape[0] for t in w)
        cin_pad = sum(segs[1::2])
        wf = w[0].new_empty((n, Kf), dtype=torch.bfloat16)
        wd = w[0].new_empty((cin_pad, Kd), dtype=torch.bfloat16) if Kd > 0 else None
        return wf, wd, w[0].new_empty((n,))

    @fake(lib + "pack_conv_weights_multi")
    def _(w, b, nw, segs, nseg, scale, Kf, Kd, aux, f16=False, split=False):
        dt = torch.float16 if f16 else torch.bfloat16
        out, wi, si = [], 0, 0
        for q in range(len(nw)):
            n = sum(t.shape[0] for t in w[wi:wi + nw[q]])
            cin_pad = sum(segs[si:si + 2 * nseg[q]][1::2])
            wi += nw[q]
            si += 2 * nseg[q]
            out += [w[0].new_empty((n, Kf[q]), dtype=dt),
                    w[0].new_empty((cin_pad, Kd[q]) if Kd[q] > 0 else (0,), dtype=dt), w[0].new_empty((n,))]
        return out

    @fake(lib + "pack_conv_weights")
    def _(w, b, segs, scale, Kf, Kd, cout_pad, f16=False):
        n = sum(t.shape[0] for t in w)
        cin_pad = sum(segs[1::2])
        dt = torch.float16 if f16 else torch.bfloat16
        wf = w[0].new_empty((n, Kf), dtype=dt)
        wd = w[0].new_empty((cin_pad, Kd), dtype=dt) if Kd > 0 else None
        return wf, wd, w[0].new_empty((n,))

    @fake(lib + "enc_conv_fwd")
    def _(x, w, bias, stride, pad, stats, split=False, prepacked=None):
        B, H, W, Cx = x.shape
        N, Cin, KH, KW = w.shape
        Ho, Wo = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
        if split:
            T = -(-(Ho * Wo) // 128)
            st = x.new_empty((B, T, 2, N), dtype=torch.float32) if stats else x.new_empty((0,), dtype=torch.float32)
            return x.new_empty((B, Ho, Wo, 3 * N)), st
        if not stats:
            st = x.new_empty((0,), dtype=torch.float32)
        elif (Cx, Cin, N, KH, KW, stride, pad) == (64, 64, 64, 3, 3, 1, 1):
            # resident-weight 3x3 kernel: 16x16 tiles (csrc/kernel_abi.h enc_conv3_eligible)
            st = x.new_empty((B, -(-Ho // 16), -(-Wo // 16), 2, N), dtype=torch.float32)
        else:
            T = -(-(Ho * Wo) // 128)  # 128-pixel conv tiles (csrc/enc_bindings.cpp kBM)
            st = x.new_empty((B, T, 2, N), dtype=torch.float32)
        return x.new_empty((B, Ho, Wo, N)), st

    @fake(lib + "enc_conv_dgrad")
    def _(dys, ws, strides, pads, H, W, res, mask, split=False, prepacked=None):
        return dys[0].new_empty((dys[0].shape[0], H, W, (3 if split else 1) * ws[0].shape[1]))

    @fake(lib + "enc_prep")
    def _(img0, img1, split=False, f16=False):
        n = img0.shape[0] * (2 if img1 is not None else 1)
        return img0.new_empty((n, img0.shape[2], img0.shape[3], 24 if split else 8),
                              dtype=torch.float16 if f16 else torch.bfloat16)

    @fake(lib + "enc_norm_stats")
    def _(stats, B, HW, N, kind, gamma, beta, rmean, rvar, nbt, momentum, eps, W=0):
        like = stats if stats is not None else rmean
        return like.new_empty((B, 4, N), dtype=torch.float32)

    @fake(lib + "enc_apply")
    def _(a, coef, relu_a, r, coef_r, relu_out, split=False):
        return torch.empty_like(a)

    @fake(lib + "enc_norm_bwd")
    def _(g, a0, c0, relu0, a1, c1, kind, split=False):
        N = g.shape[3] // (3 if split else 1)
        bn = kind in (2, 3)
        two = a1 is not None
        f = lambda: g.new_empty((N,), dtype=torch.float32)  # noqa: E731
        return [torch.empty_like(g), torch.empty_like(g) if two else g.new_empty((0,)),
                f() if bn else g.new_empty((0,)), f() if bn else g.new_empty((0,)),
                f() if bn and two else g.new_empty((0,)), f() if bn and two else g.new_empty((0,))]

    @fake(lib + "enc_norm_bwd_part")
    def _(g, a0, c0, relu0, a1, c1, kind, split=False):
        B, H, W, N = g.shape
        N //= 3 if split else 1
        R = min(64, max(1, H * W // 256))  # csrc kNormChunks
        return g.new_empty((B, R, 4, N), dtype=torch.float32)

    @fake(lib + "enc_norm_bwd_finish")
    def _(g, a0, c0, relu0, a1, c1, kind, part, b_fin, split=False):
        N = g.shape[3] // (3 if split else 1)
        two = a1 is not None
        f = lambda: g.new_empty((N,), dtype=torch.float32)  # noqa: E731
        return [torch.empty_like(g), torch.empty_like(g) if two else g.new_empty((0,)), f(), f(),
                f() if two else g.new_empty((0,)), f() if two else g.new_empty((0,))]

    @fake(lib + "upflow8")
    def _(flow):
        B, _, H, W = flow.shape
        return flow.new_empty((B, 2, 8 * H, 8 * W))

    @fake(lib + "upflow8_backward")
    def _(grad, H, W, rows):
        return grad.new_empty((grad.shape[0], 2, H, W))

    # mutating ops: nothing to infer
    for name in ("conv_fwd", "conv_wgrad", "conv_wgrad_params", "gru_bwd_a", "gru_bwd_b", "masked_cast",
                 "pack_flow", "apply_delta", "n2_apply", "corr_lookup_into", "corr_lookup_split_into", "convex_upsample_backward_into",
                 "corr_lookup_backward_", "corr_lookup_grad_rows", "corr_gemm", "corr_pyramid_bwd", "local_corr_mfma", "local_corr_mfma_backward",
                 "enc_conv_wgrad", "enc_pack_multi"):
        fake(lib + name)(lambda *args, **kwargs: None)
