"""Fused RAFT-base update block on hand-written HIP kernels (forward + backward).

One refinement iteration of ``BasicUpdateBlock`` (reference core/update.py:79-136:
BasicMotionEncoder -> SepConvGRU -> FlowHead + mask head) runs as 11
implicit-GEMM MFMA convolutions with fused epilogues (``csrc/conv_igemm.hip``)
instead of ~300 PyTorch/MIOpen launches:

  corr (P, 328) --convc1 1x1+relu--> c1 --convc2 3x3+relu--> cf[:, :192]
  flow8 (P, 8)  --convf1 7x7+relu--> f1 --convf2 3x3+relu--> cf[:, 192:]
  cf --conv 3x3+relu--> motion[:, :126]   (motion[:, 126:] = flow: fused cat)
  [h | inp | motion] --z||r 1x5 (sigmoid, r*h epilogue)--> zr, rh
  [rh | inp | motion] --q 1x5 (tanh + GRU blend epilogue)--> h1          (x2: 5x1)
  h2 --[flow_head.conv1 || mask.0] 3x3+relu (one 512-wide conv)--> hd
  hd[:, :256] --flow_head.conv2 3x3--> delta (fp32);  hd[:, 256:] --0.25*mask.2 1x1--> mask

The backward is hand-scheduled: dgrad convs (same kernel, flipped weights) with
ReLU' masks and partial accumulation in the epilogue, wgrad kernels that
accumulate every iteration's weight/bias gradients in place into persistent
fp32 buffers, and four small elementwise kernels for the GRU gate derivatives.

Weights are packed (bf16, GEMM layout, forward and data-grad variants) ONCE
per RAFT forward by ``_PackWeights``; its backward -- which autograd runs after
the last iteration's backward because every step consumes its token -- turns
the accumulated fp32 buffers into the parameters' gradients.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch

from . import conv as C
from ._ext import ops

HID = 128
CORR_PAD = 328  # 4 * 81 = 324 lookup channels, padded to a multiple of 8


def _layers(block) -> List[Tuple[str, torch.nn.Conv2d]]:
    enc, gru = block.encoder, block.gru
    return [
        ("convc1", enc.convc1), ("convc2", enc.convc2), ("convf1", enc.convf1), ("convf2", enc.convf2),
        ("conv", enc.conv),
        ("zr1", (gru.convz1, gru.convr1)), ("q1", gru.convq1),
        ("zr2", (gru.convz2, gru.convr2)), ("q2", gru.convq2),
        ("heads", (block.flow_head.conv1, block.mask[0])), ("fh2", block.flow_head.conv2), ("mask2", block.mask[2]),
    ]


# input-channel segment layout (real, padded) of every conv
SEGMENTS: Dict[str, List[Tuple[int, int]]] = {
    "convc1": [(324, CORR_PAD)],
    "convc2": [(256, 256)],
    "convf1": [(2, 8)],
    "convf2": [(128, 128)],
    "conv": [(256, 256)],
    "zr1": [(384, 384)], "q1": [(384, 384)], "zr2": [(384, 384)], "q2": [(384, 384)],
    "heads": [(128, 128)],
    "fh2": [(256, 256)],
    "mask2": [(256, 256)],
}
SCALE = {"mask2": 0.25}


def _params(block) -> List[torch.Tensor]:
    out = []
    for _, m in _layers(block):
        mods = m if isinstance(m, tuple) else (m,)
        for mod in mods:
            out += [mod.weight, mod.bias]
    return out


class _WeightState:
    """Packed weights of one RAFT forward + fp32 gradient accumulators."""

    def __init__(self, block):
        self.wf: Dict[str, torch.Tensor] = {}
        self.wd: Dict[str, torch.Tensor] = {}
        self.bias: Dict[str, torch.Tensor] = {}
        self.shape: Dict[str, tuple] = {}
        self.split: Dict[str, List[int]] = {}
        self.cout: Dict[str, int] = {}
        for name, m in _layers(block):
            mods = m if isinstance(m, tuple) else (m,)
            w = torch.cat([mm.weight for mm in mods], dim=0) if len(mods) > 1 else mods[0].weight
            b = torch.cat([mm.bias for mm in mods], dim=0) if len(mods) > 1 else mods[0].bias
            s = SCALE.get(name, 1.0)
            segs = SEGMENTS[name]
            self.shape[name] = tuple(w.shape)
            self.split[name] = [mm.weight.shape[0] for mm in mods]
            self.cout[name] = w.shape[0]
            self.wf[name] = C.pack_fwd(w, segs, scale=s)
            self.wd[name] = C.pack_dgrad(w, segs, scale=s)
            self.bias[name] = (b.detach().float() * s).contiguous()
        self.dw: Dict[str, torch.Tensor] = {}
        self.db: Dict[str, torch.Tensor] = {}

    def grad_bufs(self, name):
        if name not in self.dw:
            wf = self.wf[name]
            self.dw[name] = torch.zeros(wf.shape, device=wf.device, dtype=torch.float32)
            self.db[name] = torch.zeros(wf.shape[0], device=wf.device, dtype=torch.float32)
        return self.dw[name], self.db[name]


class _PackWeights(torch.autograd.Function):
    @staticmethod
    def forward(ctx, state: _WeightState, *params):
        ctx.state = state
        return params[0].new_zeros(())

    @staticmethod
    def backward(ctx, gtoken):
        st: _WeightState = ctx.state
        grads = []
        for name, _ in _layers_from_state(st):
            s = SCALE.get(name, 1.0)
            if name in st.dw:
                gw = C.unpack_grad(st.dw[name], st.shape[name], SEGMENTS[name]) * s
                gb = st.db[name] * s
            else:
                gw = gb = None
            splits = st.split[name]
            if len(splits) == 1:
                grads += [gw, gb]
            else:
                o = 0
                for n in splits:
                    grads += [None if gw is None else gw[o:o + n].contiguous(),
                              None if gb is None else gb[o:o + n].contiguous()]
                    o += n
        st.dw.clear()
        st.db.clear()
        return (None, *grads)


def _layers_from_state(st):
    return [(n, None) for n in st.wf]


def _pm(t: torch.Tensor) -> torch.Tensor:
    """(B, C, H, W) channels-last tensor -> (P, C) pixel-major view (no copy)."""
    B, Ch, H, W = t.shape
    return t.permute(0, 2, 3, 1).reshape(B * H * W, Ch)


def _nchw(t: torch.Tensor, B: int, H: int, W: int) -> torch.Tensor:
    """(P, C) pixel-major -> (B, C, H, W) channels-last view (no copy)."""
    return t.reshape(B, H, W, t.shape[1]).permute(0, 3, 1, 2)


class _UpdateStep(torch.autograd.Function):
    @staticmethod
    def forward(ctx, token, net, inp32, corr, flow, st: _WeightState, inp_bf):
        B, _, H, W = net.shape
        P = B * H * W
        dev = net.device
        bf = torch.bfloat16
        k = ops()
        g3 = lambda kh, kw: C.geom(B, H, W, kh, kw, kh // 2, kw // 2)  # noqa: E731

        h0 = _pm(net.to(bf).contiguous(memory_format=torch.channels_last))
        corr_pm = corr.reshape(P, CORR_PAD)
        inp = inp_bf
        flow = flow.float().contiguous()
        flow8 = torch.empty(P, 8, device=dev, dtype=bf)
        motion = torch.empty(P, HID, device=dev, dtype=bf)
        k.pack_flow(flow, flow8, motion[:, 126:])

        c1 = torch.empty(P, 256, device=dev, dtype=bf)
        C.conv_fwd([corr_pm], st.wf["convc1"], g3(1, 1), 256, c1, bias=st.bias["convc1"], act=1)
        cf = torch.empty(P, 256, device=dev, dtype=bf)
        C.conv_fwd([c1], st.wf["convc2"], g3(3, 3), 192, cf[:, :192], bias=st.bias["convc2"], act=1)
        f1 = torch.empty(P, 128, device=dev, dtype=bf)
        C.conv_fwd([flow8], st.wf["convf1"], g3(7, 7), 128, f1, bias=st.bias["convf1"], act=1)
        C.conv_fwd([f1], st.wf["convf2"], g3(3, 3), 64, cf[:, 192:], bias=st.bias["convf2"], act=1)
        C.conv_fwd([cf], st.wf["conv"], g3(3, 3), 126, motion, bias=st.bias["conv"], act=1)

        saved_gru = []
        h = h0
        for stage, (kh, kw) in ((1, (1, 5)), (2, (5, 1))):
            zr = torch.empty(P, 2 * HID, device=dev, dtype=bf)
            rh = torch.empty(P, HID, device=dev, dtype=bf)
            C.conv_fwd([h, inp, motion], st.wf[f"zr{stage}"], g3(kh, kw), 2 * HID, zr,
                       bias=st.bias[f"zr{stage}"], epi=C.EPI_GRU_ZR, h=h, out2=rh)
            hn = torch.empty(P, HID, device=dev, dtype=bf)
            q = torch.empty(P, HID, device=dev, dtype=bf)
            C.conv_fwd([rh, inp, motion], st.wf[f"q{stage}"], g3(kh, kw), HID, hn,
                       bias=st.bias[f"q{stage}"], epi=C.EPI_GRU_Q, h=h, z=zr[:, :HID], out2=q)
            saved_gru += [h, zr, rh, q]
            h = hn

        hd = torch.empty(P, 512, device=dev, dtype=bf)
        C.conv_fwd([h], st.wf["heads"], g3(3, 3), 512, hd, bias=st.bias["heads"], act=1)
        delta = torch.empty(P, 8, device=dev, dtype=torch.float32)
        C.conv_fwd([hd[:, :256]], st.wf["fh2"], g3(3, 3), 2, delta, bias=st.bias["fh2"])
        mask = torch.empty(P, 576, device=dev, dtype=bf)
        C.conv_fwd([hd[:, 256:]], st.wf["mask2"], g3(1, 1), 576, mask, bias=st.bias["mask2"])

        ctx.st = st
        ctx.dims = (B, H, W)
        ctx.net_dtype = net.dtype
        ctx.save_for_backward(corr, flow8, c1, cf, f1, motion, inp, h, hd, *saved_gru)
        net_out = _nchw(h, B, H, W)
        mask_out = _nchw(mask, B, H, W)
        delta_out = _nchw(delta[:, :2], B, H, W)
        return net_out, mask_out, delta_out

    @staticmethod
    def backward(ctx, g_net, g_mask, g_delta):
        st: _WeightState = ctx.st
        B, H, W = ctx.dims
        P = B * H * W
        (corr, flow8, c1, cf, f1, motion, inp, h2, hd, *sg) = ctx.saved_tensors
        dev = corr.device
        bf = torch.bfloat16
        k = ops()
        g3 = lambda kh, kw: C.geom(B, H, W, kh, kw, kh // 2, kw // 2)  # noqa: E731
        gd = lambda kh, kw: C.geom(B, H, W, kh, kw, kh - 1 - kh // 2, kw - 1 - kw // 2)  # noqa: E731

        def wgrad(name, srcs, dy, kh, kw):
            dw, db = st.grad_bufs(name)
            C.conv_wgrad(srcs, dy, g3(kh, kw), st.cout[name], dw, db)

        def dgrad(name, dy, kh, kw, out, n, mask=None, acc_c0=1 << 30):
            C.conv_fwd([dy], st.wd[name], gd(kh, kw), n, out, epi=C.EPI_GRAD, mask=mask, acc_c0=acc_c0)

        # ---- heads
        dhd = torch.empty(P, 512, device=dev, dtype=bf)
        if g_mask is not None:
            dmask = _pm(g_mask.to(bf).contiguous(memory_format=torch.channels_last))
            wgrad("mask2", [hd[:, 256:]], dmask, 1, 1)
            dgrad("mask2", dmask, 1, 1, dhd[:, 256:], 256, mask=hd[:, 256:])
        else:
            dhd[:, 256:].zero_()
        ddelta = torch.zeros(P, 8, device=dev, dtype=bf)
        if g_delta is not None:
            ddelta[:, :2] = g_delta.permute(0, 2, 3, 1).reshape(P, 2)
        wgrad("fh2", [hd[:, :256]], ddelta, 3, 3)
        dgrad("fh2", ddelta, 3, 3, dhd[:, :256], 256, mask=hd[:, :256])
        wgrad("heads", [h2], dhd, 3, 3)
        dh = torch.empty(P, HID, device=dev, dtype=torch.float32)
        if g_net is not None:
            dh.copy_(_pm(g_net))
            acc = 0
        else:
            acc = 1 << 30
        dgrad("heads", dhd, 3, 3, dh, HID, acc_c0=acc)

        # ---- GRU stages (reverse order); G = [dh | d inp | d motion] accumulates over stages
        G = torch.empty(P, 3 * HID, device=dev, dtype=torch.float32)
        carry = torch.empty(P, HID, device=dev, dtype=torch.float32)
        dq = torch.empty(P, HID, device=dev, dtype=bf)
        dzr = torch.empty(P, 2 * HID, device=dev, dtype=bf)
        first = True
        for stage, (kh, kw) in ((2, (5, 1)), (1, (1, 5))):
            h, zr, rh, q = sg[(stage - 1) * 4:(stage - 1) * 4 + 4]
            dH = dh if stage == 2 else G[:, :HID]
            k.gru_bwd_a(dH, zr[:, :HID], q, h, dq, dzr[:, :HID], carry)
            wgrad(f"q{stage}", [rh, inp, motion], dq, kh, kw)
            # fresh write of d(rh); x part fresh on the first stage, accumulated afterwards
            dgrad(f"q{stage}", dq, kh, kw, G, 3 * HID, acc_c0=(3 * HID if first else HID))
            k.gru_bwd_b(G[:, :HID], zr[:, HID:], h, carry, dzr[:, HID:])
            wgrad(f"zr{stage}", [h, inp, motion], dzr, kh, kw)
            dgrad(f"zr{stage}", dzr, kh, kw, G, 3 * HID, acc_c0=0)
            first = False

        # ---- motion encoder
        dmo = torch.empty(P, HID, device=dev, dtype=bf)
        k.masked_cast(G[:, 2 * HID:2 * HID + 126], motion, dmo)  # relu' ; flow channels -> 0
        wgrad("conv", [cf], dmo, 3, 3)
        dcf = torch.empty(P, 256, device=dev, dtype=bf)
        dgrad("conv", dmo, 3, 3, dcf, 256, mask=cf)
        wgrad("convc2", [c1], dcf[:, :192], 3, 3)
        dc1 = torch.empty(P, 256, device=dev, dtype=bf)
        dgrad("convc2", dcf[:, :192], 3, 3, dc1, 256, mask=c1)
        wgrad("convc1", [corr.reshape(P, CORR_PAD)], dc1, 1, 1)
        dcorr = torch.empty(P, CORR_PAD, device=dev, dtype=bf)
        dgrad("convc1", dc1, 1, 1, dcorr, CORR_PAD)
        wgrad("convf2", [f1], dcf[:, 192:], 3, 3)
        df1 = torch.empty(P, 128, device=dev, dtype=bf)
        dgrad("convf2", dcf[:, 192:], 3, 3, df1, 128, mask=f1)
        wgrad("convf1", [flow8], df1, 7, 7)

        d_net = _nchw(G[:, :HID].to(ctx.net_dtype), B, H, W)
        d_inp = _nchw(G[:, HID:2 * HID].contiguous(), B, H, W)
        d_corr = dcorr.reshape(B, H, W, CORR_PAD)
        return torch.zeros((), device=dev), d_net, d_inp, d_corr, None, None, None


class FusedBasicUpdate:
    """Per-forward driver: packs weights once, then runs fused iterations."""

    def __init__(self, block, inp: torch.Tensor):
        self.state = _WeightState(block)
        self.token = _PackWeights.apply(self.state, *_params(block))
        # the context features are constant over iterations: one bf16 pixel-major copy,
        # while the fp32 ``inp`` keeps autograd's cross-iteration gradient sum in fp32
        self.inp32 = inp.float().contiguous(memory_format=torch.channels_last)
        self.inp_bf = _pm(inp.detach().to(torch.bfloat16).contiguous(memory_format=torch.channels_last))

    def __call__(self, net, corr_padded, flow):
        return _UpdateStep.apply(self.token, net, self.inp32, corr_padded, flow, self.state, self.inp_bf)


def supported(block) -> bool:
    from ..models.update import BasicUpdateBlock

    return isinstance(block, BasicUpdateBlock)
