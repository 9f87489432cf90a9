"""Host side of the implicit-GEMM NHWC conv kernels (``csrc/conv_igemm.hip``).

Activations are *pixel-major* 2-D views ``(P, C)`` (P = B*H*W, unit channel
stride, pixel stride = the row pitch of the buffer they live in), so a conv can
read a channel slice of a wider buffer and write into one.  Weights are packed
once per forward into the GEMM layout the kernels read:

* forward  ``[Cout][Kpad]`` with ``k = tap*Cin_pad + c`` (``pack_fwd``);
* data-grad ``[Cin_pad][Kpad']`` with flipped taps and ``k = tap*Cout_pad + n``
  (``pack_dgrad``) -- the data-gradient of a stride-1 conv is itself a conv.

``segments`` describe how the kernel's input channels map onto (possibly
padded) source channels: a list of ``(real, padded)`` pairs, e.g. the motion
encoder's flow input is ``[(2, 8)]`` (2 real channels stored in an 8-channel
buffer) and the corr features ``[(324, 328)]``.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

from ._ext import ops

KBLK = 64  # K granularity of the kernels (BK)


def _round(n: int, m: int) -> int:
    return (n + m - 1) // m * m


def _expand_cin(w: torch.Tensor, segments: Sequence[Tuple[int, int]]) -> torch.Tensor:
    """(Cout, Cin, kh, kw) -> (Cout, Cin_pad, kh, kw) with zeros in padded slots."""
    real = sum(r for r, _ in segments)
    assert real == w.shape[1], (real, w.shape)
    if all(r == p for r, p in segments):
        return w
    parts, c = [], 0
    for r, p in segments:
        parts.append(w[:, c:c + r])
        if p > r:
            parts.append(w.new_zeros(w.shape[0], p - r, w.shape[2], w.shape[3]))
        c += r
    return torch.cat(parts, dim=1)


def pack_fwd(w: torch.Tensor, segments: Optional[Sequence[Tuple[int, int]]] = None, scale: float = 1.0):
    """(Cout, Cin, kh, kw) fp32 -> bf16 [Cout][Kpad] (k = tap*Cin_pad + c)."""
    cout, cin, kh, kw = w.shape
    segments = segments or [(cin, cin)]
    we = _expand_cin(w.detach(), segments)
    cin_p = we.shape[1]
    k = kh * kw * cin_p
    out = torch.zeros(cout, _round(k, KBLK), device=w.device, dtype=torch.bfloat16)
    out[:, :k] = (we * scale).permute(0, 2, 3, 1).reshape(cout, k).to(torch.bfloat16)
    return out


def pack_dgrad(w: torch.Tensor, segments: Optional[Sequence[Tuple[int, int]]] = None, cout_pad: Optional[int] = None,
               scale: float = 1.0):
    """bf16 [Cin_pad][Kpad] for dX = conv(dY, W flipped/transposed), k = tap*Cout_pad + n."""
    cout, cin, kh, kw = w.shape
    segments = segments or [(cin, cin)]
    we = _expand_cin(w.detach(), segments) * scale  # (Cout, Cin_pad, kh, kw)
    cout_p = cout_pad or _round(cout, 8)
    if cout_p > cout:
        we = torch.cat([we, we.new_zeros(cout_p - cout, *we.shape[1:])], dim=0)
    wt = we.flip(2, 3).permute(1, 2, 3, 0)  # (Cin_pad, kh, kw, Cout_pad)
    cin_p = wt.shape[0]
    k = kh * kw * cout_p
    out = torch.zeros(cin_p, _round(k, KBLK), device=w.device, dtype=torch.bfloat16)
    out[:, :k] = wt.reshape(cin_p, k).to(torch.bfloat16)
    return out


def unpack_grad(dw: torch.Tensor, shape, segments: Optional[Sequence[Tuple[int, int]]] = None) -> torch.Tensor:
    """fp32 [Cout][Kpad] accumulated weight gradient -> (Cout, Cin, kh, kw)."""
    cout, cin, kh, kw = shape
    segments = segments or [(cin, cin)]
    cin_p = sum(p for _, p in segments)
    g = dw[:cout, : kh * kw * cin_p].reshape(cout, kh, kw, cin_p).permute(0, 3, 1, 2)
    if cin_p != cin:
        parts, c = [], 0
        for r, p in segments:
            parts.append(g[:, c:c + r])
            c += p
        g = torch.cat(parts, dim=1)
    return g.contiguous()


def geom(B: int, H: int, W: int, kh: int, kw: int, ph: int, pw: int) -> List[int]:
    return [B, H, W, kh, kw, ph, pw]


EPI_STORE, EPI_GRAD, EPI_GRU_ZR, EPI_GRU_Q, EPI_GRU_BWD_A, EPI_GRU_BWD_B, EPI_GRU_BWD_LAST = 0, 1, 2, 3, 4, 5, 6


def conv_fwd(srcs, wt, g, N, out, bias=None, act=0, alpha=1.0, epi=EPI_STORE, acc_c0=1 << 30, mask=None,
             h=None, z=None, out2=None, cfg: int = 0, g0=None, carry=None, out3=None, gru_cols: int = 0,
             addsrc=None, cout=None, cmask=None, cm_c0: int = 0, cm_valid: int = 0, split=None, n2w=None,
             n2y=None):
    """``cfg`` forces a kernel variant (0 = automatic; tests and microbenchmarks only):
    1 generic, 8/9 v4 64x128/64x64, 20/21 v5 halo strip 64x128/128x128 (4 waves),
    24..26 v5 with 8 waves 256x128/128x128/128x256.

    Data-gradient launches of the GRU can finish the gate backward in the epilogue for the
    output channels [0, gru_cols) (fp32 ``out``; the other channels behave as EPI_GRAD):
      EPI_GRU_BWD_A: g = dH (+= out where acc): out2 = dq = g z (1 - q^2), out3 = dz =
        g (q - h) z (1 - z), carry = g (1 - z); with z, g0 = q, h;
        (+ ``addsrc``, an incoming bf16 gradient);
      EPI_GRU_BWD_B: g = d(r h): out3 = dr = g h r (1 - r), out = carry + g r; g0 = r, h;
      EPI_GRU_BWD_LAST: g = out + acc: [0, gru_cols) -> bf16 out3, [gru_cols, cm_c0) -> out,
        [cm_c0, N) -> bf16 cout = g where cmask > 0 (zero past cm_valid).

    ``split = (G_out, G_out2, S_h, S_z)``: split-bf16 (fp32-faithful) epilogues 0 / 2 / 3, see
    ``split_pack`` and csrc/kernel_abi.h ``ConvFwdArgs::split_g``.

    ``n2w`` / ``n2y``: a narrow 3x3 follow-up conv (2 outputs; the flow head's conv2) folded
    into epilogue 0: ``n2y`` (fp32 [slots, 18, P]) receives the per-tap partial products of
    the first 64 * slots output channels, and ``n2_apply`` finishes the conv (see
    csrc/kernel_abi.h ``ConvFwdArgs::n2y``)."""
    ops().conv_fwd(list(srcs), wt, g, N, bias, epi, act, alpha, out, acc_c0, mask, h, z, out2, cfg, g0, carry,
                   out3, gru_cols, addsrc, cout, cmask, cm_c0, cm_valid, list(split) if split else [], n2w, n2y)
    return out


def conv_wgrad(srcs, dy, g, N, dw, db=None, accumulate: bool = True):
    """dw[N][Kpad] (+)= weight gradient in the packed layout (deterministic split reduction)."""
    ops().conv_wgrad(list(srcs), dy, g, N, dw, db, accumulate)


def flat_segments(segments: Sequence[Tuple[int, int]]) -> List[int]:
    return [v for rp in segments for v in rp]


def conv_wgrad_params(srcs, dy, g, wgrads, bgrads, segments, scale: float = 1.0, accumulate: bool = False,
                      fold: bool = False):
    """Weight (+bias) gradients of 1..2 stacked conv parameters written straight into
    ``wgrads`` / ``bgrads`` (parameter layout, any strides).  A source with fewer rows
    than the pixel count is periodic (row p % rows), e.g. context features shared by
    every refinement iteration of a batched update-block weight gradient.  ``fold``: every
    source holds its segment as [hi | lo] split planes; their columns are summed."""
    ops().conv_wgrad_params(list(srcs), dy, g, list(wgrads), list(bgrads), flat_segments(segments), scale,
                            accumulate, fold)


def split_planes(n: int, G: int) -> int:
    """Channels of a split-bf16 row holding ``n`` channels in groups of ``G`` (hi, lo, hi planes)."""
    return -(-n // G) * 3 * G


def split_pack(src: torch.Tensor, dst: torch.Tensor, G: int, c0: int = 0, cpad: Optional[int] = None):
    """fp32 (P, C) rows -> split-bf16 planes (hi, lo, hi) of group width ``G`` in ``dst`` at
    output channels [c0, c0 + cpad) (zeros past C)."""
    ops().split_pack(src, dst, G, c0, cpad if cpad is not None else src.shape[1])
    return dst


def pack_weights_split(weights, biases, source_segments, scale: float = 1.0):
    """Forward weights of a conv over split-bf16 operands (no data-gradient operand); the torch
    reference of ``pack_weights_split_native`` (tests).

    ``source_segments``: one list of (real, padded) segments per SOURCE tensor (a source is one
    split operand [hi | lo | hi] of its padded width).  The packed K runs over each source's
    planes against [W_hi | W_hi | W_lo], so x_hi W_hi + x_lo W_hi + x_hi W_lo is one GEMM."""
    w = torch.cat([t.detach() for t in weights], 0).float() * scale
    parts, c = [], 0
    for segs in source_segments:
        r = sum(rr for rr, _ in segs)
        ws = w[:, c:c + r]
        hi = ws.to(torch.bfloat16).float()
        parts += [hi, hi, ws - hi]
        c += r
    assert c == w.shape[1], (c, w.shape)
    b = [None if t is None else t.detach().float() * scale for t in biases]
    bias = torch.cat(b) if all(x is not None for x in b) else torch.zeros(w.shape[0], device=w.device)
    return pack_fwd(torch.cat(parts, 1), split_segments_by_source(source_segments)), bias


def pack_weights_split_native(weights, biases, segments, scale: float = 1.0, G_dy: int = 0):
    """One HIP launch (csrc/weights.hip pack_conv_weights_split_kernel): the split-bf16 forward
    operand -- every segment (one per source) as [W_hi | W_hi | W_lo] against its [hi | lo | hi]
    planes -- and, for ``G_dy > 0``, the data-gradient operand over dY planes of width ``G_dy``
    (the layouts of ``pack_weights_split`` / ``ops.update_split.pack_dgrad_split``) plus the
    fp32 scaled bias -> (wf, wd or None, bias)."""
    cout = sum(w.shape[0] for w in weights)
    _, cin, kh, kw = weights[0].shape
    cin_p = sum(p for _, p in segments)
    kf = _round(kh * kw * 3 * cin_p, KBLK)
    kd = _round(kh * kw * 3 * G_dy, KBLK) if G_dy else 0
    return ops().pack_conv_weights_split([t.detach() for t in weights], [None if t is None else t.detach() for t in biases],
                                         flat_segments(segments), scale, kf, kd, G_dy)


def pack_weights_multi(layers, f16: bool = False, split: bool = False):
    """Every layer's operands in ONE launch (csrc/weights.hip pack_conv_weights_multi_kernel).

    ``layers``: [(weights, biases, segments, scale, dgrad_arg)] with ``dgrad_arg`` the bool
    ``dgrad`` of :func:`pack_weights` (bf16 / fp16) or the ``G_dy`` of
    :func:`pack_weights_split_native` (``split=True``; 0 = no data-gradient operand).
    Returns [(wf, wd or None, bias)] in the layouts of those two functions."""
    w, b, nw, segs, nseg, scales, kfs, kds, aux = [], [], [], [], [], [], [], [], []
    for weights, biases, segments, scale, darg in layers:
        cout = sum(t.shape[0] for t in weights)
        _, _, kh, kw = weights[0].shape
        cin_p = sum(p for _, p in segments)
        w += [t.detach() for t in weights]
        b += [None if t is None else t.detach() for t in biases]
        nw.append(len(weights))
        fs = flat_segments(segments)
        segs += fs
        nseg.append(len(fs) // 2)
        scales.append(float(scale))
        if split:
            kfs.append(_round(kh * kw * 3 * cin_p, KBLK))
            kds.append(_round(kh * kw * 3 * darg, KBLK) if darg else 0)
            aux.append(int(darg))
        else:
            cout_p = _round(cout, 8)
            kfs.append(_round(kh * kw * cin_p, KBLK))
            kds.append(_round(kh * kw * cout_p, KBLK) if darg else 0)
            aux.append(cout_p)
    out = ops().pack_conv_weights_multi(w, b, nw, segs, nseg, scales, kfs, kds, aux, f16, split)
    return [(out[3 * i], out[3 * i + 1] if out[3 * i + 1].numel() else None, out[3 * i + 2])
            for i in range(len(layers))]


def split_segments_by_source(source_segments) -> List[Tuple[int, int]]:
    """Segments of the expanded weight [W_hi | W_hi | W_lo] per source, in K order (every
    source's (real, padded) channel groups appear three times: its hi, lo and hi planes)."""
    out: List[Tuple[int, int]] = []
    for segs in source_segments:
        for r, p in list(segs) * 3:
            if out and r == p and out[-1][0] == out[-1][1]:  # unpadded neighbours merge (<= 3 segments)
                out[-1] = (out[-1][0] + r, out[-1][1] + p)
            else:
                out.append((r, p))
    return out


def pack_weights(weights, biases, segments, scale: float = 1.0, dgrad: bool = True, f16: bool = False):
    """One HIP launch: fp32 parameters (1..2 stacked along Cout) -> (wf [N][Kpad] bf16,
    wd [Cin_pad][Kpad'] bf16 or None, bias fp32 [N]) -- the layouts of ``pack_fwd`` /
    ``pack_dgrad``; ``f16``: fp16 operands (fp16 AMP) instead of bf16."""
    cout = sum(w.shape[0] for w in weights)
    _, cin, kh, kw = weights[0].shape
    cin_p = sum(p for _, p in segments)
    cout_p = _round(cout, 8)
    kf = _round(kh * kw * cin_p, KBLK)
    kd = _round(kh * kw * cout_p, KBLK) if dgrad else 0
    w = [t.detach() for t in weights]
    b = [None if t is None else t.detach() for t in biases]
    return ops().pack_conv_weights(w, b, flat_segments(segments), scale, kf, kd, cout_p, f16)
