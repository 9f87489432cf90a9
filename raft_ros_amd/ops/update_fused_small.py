"""Fused RAFT-small refinement step on the hand-written HIP kernels (forward + backward).

Same design as ``update_fused.py`` (one autograd node per iteration, weight gradients
batched over all iterations by a token node), for the small update operator
(reference core/update.py:16-31 ConvGRU, :62-77 SmallMotionEncoder, :99-112
SmallUpdateBlock; core/raft.py:131-134 upflow8):

  lookup (4 levels x 49 taps, radius 3)   -> corr (P, 200)                [corr_lookup_into, which also
  coords1 - grid                          -> flow8 (P, 8), motion[:, 80:82]      packs the flow operand]
  corr --convc1 1x1+relu--> cf[:, :96]
  flow8 --convf1 7x7+relu--> f1 --convf2 3x3+relu--> cf[:, 96:]
  cf --conv 3x3+relu--> motion[:, :80]           (motion = 88 channels, 82..87 zero)
  [h | inp | motion] --z||r 3x3 (sigmoid, r*h epilogue)--> zr, rh
  [rh | inp | motion] --q 3x3 (tanh + GRU blend epilogue)--> h'
  h' --flow_head.conv1 3x3+relu--> hd --flow_head.conv2 3x3--> delta
  coords1 + delta [apply_delta];  8x bilinear upsampling [upflow8]

Input channel segments are padded to multiples of 8 (196 corr taps -> 200, 82 motion
channels -> 88); the packed weights hold zeros in the padded slots.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from . import conv as C
from ._ext import ops
from .update_fused import _I32, _Arena, _nchw, _pm

HID, CTX = 96, 64
MOT, MOT_PAD = 82, 88
CORR_PAD = 200  # 4 * 49 = 196 lookup channels, padded to a multiple of 8
GX = HID + CTX + MOT_PAD  # [h | inp | motion] channels of the GRU convs (248)

# name -> (modules getter, input segments (real, padded), needs a dgrad operand)
_LAYERS = [
    ("convc1", lambda b: (b.encoder.convc1,), [(196, CORR_PAD)], True),
    ("convf1", lambda b: (b.encoder.convf1,), [(2, 8)], False),
    ("convf2", lambda b: (b.encoder.convf2,), [(64, 64)], True),
    ("conv", lambda b: (b.encoder.conv,), [(128, 128)], True),
    ("zr", lambda b: (b.gru.convz, b.gru.convr), [(HID, HID), (CTX, CTX), (MOT, MOT_PAD)], True),
    ("q", lambda b: (b.gru.convq,), [(HID, HID), (CTX, CTX), (MOT, MOT_PAD)], True),
    ("fh1", lambda b: (b.flow_head.conv1,), [(HID, HID)], True),
    ("fh2", lambda b: (b.flow_head.conv2,), [(128, 128)], True),
]
_DY = ("dd8", "dhd", "dq", "dzr", "dmo", "dcf", "df1")


def _params(block) -> List[torch.Tensor]:
    out = []
    for _, mods, _, _ in _LAYERS:
        for m in mods(block):
            out += [m.weight, m.bias]
    return out


class _Run:
    def __init__(self, block, inp: torch.Tensor, iters: int, pyramid=None, keep: bool = True,
                 dt16=torch.bfloat16):
        B, _, H, W = inp.shape
        self.dt16 = dt16  # 16-bit operand dtype: bf16, or fp16 (fp16 AMP)
        self.dims = (B, H, W)
        self.P = B * H * W
        self.iters = iters
        self.block = block
        self.pyr = pyramid
        self.arena = _Arena(iters, self.P, inp.device, keep, dt16)
        self.done = set()
        self.g_all: Optional[torch.Tensor] = None  # [iters, P, GX] data-gradient rows (backward)
        self.coords = {}
        self.wf, self.wd, self.bias = {}, {}, {}
        packed = C.pack_weights_multi([([m.weight for m in mods(block)], [m.bias for m in mods(block)], segs, 1.0, dgrad)
                                       for name, mods, segs, dgrad in _LAYERS], f16=dt16 == torch.float16)
        for (name, _, _, _), (wf, wd, b) in zip(_LAYERS, packed):
            self.wf[name], self.wd[name], self.bias[name] = wf, wd, b
        self.inp_bf = _pm(inp.detach().to(dt16).contiguous(memory_format=torch.channels_last))
        self._motion_zeroed = False

    def geom(self, kh, kw, T: int = 1):
        B, H, W = self.dims
        return C.geom(T * B, H, W, kh, kw, kh // 2, kw // 2)

    def geom_d(self, kh, kw):
        B, H, W = self.dims
        return C.geom(B, H, W, kh, kw, kh - 1 - kh // 2, kw - 1 - kw // 2)

    def motion(self, t: int) -> torch.Tensor:
        m = self.arena.take("motion", t, MOT_PAD)
        if self.arena.keep:
            if not self._motion_zeroed:  # padding channels 82..87 stay zero in every slot
                self.arena.bufs["motion"][:, MOT:].zero_()
                self._motion_zeroed = True
        else:
            m[:, MOT:].zero_()
        return m

    def weight_grads(self) -> List[Optional[torch.Tensor]]:
        T, P, ar = self.iters, self.P, self.arena
        for t in range(T):
            if t not in self.done:
                for name in _DY:
                    if name in ar.bufs:
                        ar.rows(name, t, t + 1).zero_()
        inp = self.inp_bf

        def srcs_dy(name, t0, t1):
            r = lambda n: ar.rows(n, t0, t1)  # noqa: E731
            if name == "convc1":
                return [r("corr")], r("dcf")[:, :96]
            if name == "convf1":
                return [r("flow8")], r("df1")
            if name == "convf2":
                return [r("f1")], r("dcf")[:, 96:]
            if name == "conv":
                return [r("cf")], r("dmo")
            if name == "zr":
                return [ar.rows("h", t0, t1), inp, r("motion")], r("dzr")
            if name == "q":
                return [r("rh"), inp, r("motion")], r("dq")
            if name == "fh1":
                return [ar.rows("h", t0 + 1, t1 + 1)], r("dhd")
            return [r("hd")], r("dd8")  # fh2

        grads: List[Optional[torch.Tensor]] = []
        for name, mods, segs, _ in _LAYERS:
            ms = mods(self.block)
            wg = [torch.empty_like(m.weight) for m in ms]
            bg = [torch.empty_like(m.bias) for m in ms]
            kh, kw = ms[0].weight.shape[2:]
            srcs, dy = srcs_dy(name, 0, T)
            per_iter = max([s.stride(0) * 2 * P for s in srcs] + [dy.stride(0) * 2 * P])
            chunk = max(1, min(T, _I32 // max(per_iter, 1)))
            for t0 in range(0, T, chunk):
                t1 = min(T, t0 + chunk)
                srcs, dy = srcs_dy(name, t0, t1)
                if len(srcs) > 1:
                    # the batched wgrad kernels take multi-source inputs only in 128-channel
                    # segments; the small GRU's [96 | 64 | 88] input is materialised instead
                    n = (t1 - t0) * P
                    srcs = [torch.cat([s if s.shape[0] == n else s.repeat((t1 - t0), 1) for s in srcs], dim=1)]
                C.conv_wgrad_params(srcs, dy, self.geom(kh, kw, t1 - t0), wg, bg, segs, 1.0, accumulate=t0 > 0)
            for w, b in zip(wg, bg):
                grads += [w, b]
        return grads


class _PackWeights(torch.autograd.Function):
    @staticmethod
    def forward(ctx, run: _Run, *params):
        ctx.run = run
        ctx.set_materialize_grads(False)  # the steps send no token gradient (None): no zero fills
        return params[0].new_empty(())  # ordering token: its value is never read (no fill launch)

    @staticmethod
    def backward(ctx, gtoken):
        run: _Run = ctx.run
        grads = run.weight_grads()
        run.arena.bufs.clear()
        return (None, *grads)


class _Step(torch.autograd.Function):
    @staticmethod
    def forward(ctx, wtoken, ptoken, net, inp32, corr_in, coords1, run: _Run, t: int, up: bool = True):
        B, H, W = run.dims
        P = run.P
        k = ops()
        ar = run.arena
        g = run.geom

        net_pm = _pm(net)
        if not ar.keep and net_pm.dtype == run.dt16 and net_pm.is_contiguous():
            h0 = net_pm  # inference: the previous step's output rows, no copy per iteration
        else:
            h0 = ar.take("h", t, HID, slots=run.iters + 1)
            if net_pm.data_ptr() != h0.data_ptr():
                h0.copy_(net_pm)
        corr = ar.take("corr", t, CORR_PAD)
        flow8 = ar.take("flow8", t, 8)
        motion = run.motion(t)
        if run.pyr is not None:  # the lookup launch also packs the flow operand
            k.corr_lookup_into(run.pyr.levels, coords1, run.pyr.radius, corr.view(B, H, W, CORR_PAD), flow8,
                               motion[:, 80:82])
        else:
            corr.copy_(corr_in.reshape(P, CORR_PAD))
            k.pack_flow(coords1, flow8, motion[:, 80:82], True)

        cf = ar.take("cf", t, 128)
        C.conv_fwd([corr], run.wf["convc1"], g(1, 1), 96, cf[:, :96], bias=run.bias["convc1"], act=1)
        f1 = ar.take("f1", t, 64)
        C.conv_fwd([flow8], run.wf["convf1"], g(7, 7), 64, f1, bias=run.bias["convf1"], act=1)
        C.conv_fwd([f1], run.wf["convf2"], g(3, 3), 32, cf[:, 96:], bias=run.bias["convf2"], act=1)
        C.conv_fwd([cf], run.wf["conv"], g(3, 3), 80, motion, bias=run.bias["conv"], act=1)

        inp = run.inp_bf
        zr = ar.take("zr", t, 2 * HID)
        rh = ar.take("rh", t, HID)
        C.conv_fwd([h0, inp, motion], run.wf["zr"], g(3, 3), 2 * HID, zr, bias=run.bias["zr"],
                   epi=C.EPI_GRU_ZR, h=h0, out2=rh)
        hn = ar.take("h", t + 1, HID, slots=run.iters + 1)
        q = ar.take("q", t, HID)
        C.conv_fwd([rh, inp, motion], run.wf["q"], g(3, 3), HID, hn, bias=run.bias["q"],
                   epi=C.EPI_GRU_Q, h=h0, z=zr[:, :HID], out2=q)

        hd = ar.take("hd", t, 128)
        C.conv_fwd([hn], run.wf["fh1"], g(3, 3), 128, hd, bias=run.bias["fh1"], act=1)
        delta = torch.empty(P, 8, device=net.device, dtype=torch.float32)
        C.conv_fwd([hd], run.wf["fh2"], g(3, 3), 2, delta, bias=run.bias["fh2"])

        coords_out = torch.empty_like(coords1)
        flow = torch.empty_like(coords1)
        k.apply_delta(coords1, delta, coords_out, flow)
        flow_up = k.upflow8(flow) if up else None  # inference: only the last step's is read

        ctx.run, ctx.t = run, t
        ctx.net_dtype = net.dtype
        ctx.has_corr_in = corr_in is not None
        run.coords[t] = coords1
        ctx.mark_non_differentiable(coords_out)
        # no zero fills for the gradients that never arrive (coords_out; the last step's net)
        ctx.set_materialize_grads(False)
        return _nchw(hn, B, H, W), flow_up, coords_out

    @staticmethod
    def backward(ctx, g_net, g_flow_up, _g_coords):
        run: _Run = ctx.run
        t = ctx.t
        B, H, W = run.dims
        P = run.P
        dev = run.inp_bf.device
        k = ops()
        ar = run.arena
        gd = run.geom_d

        def R(name):
            return ar.rows(name, t, t + 1)

        def dgrad(name, dy, kh, kw, out, n, mask=None, acc_c0=1 << 30):
            C.conv_fwd([dy], run.wd[name], gd(kh, kw), n, out, epi=C.EPI_GRAD, mask=mask, acc_c0=acc_c0)

        dd8 = ar.take("dd8", t, 8)
        if g_flow_up is not None and run.dt16 == torch.bfloat16:
            k.upflow8_backward(g_flow_up.float().contiguous(), H, W, dd8)
        elif g_flow_up is not None:  # fp16 rows: from the fp32 flow gradient
            dflow = k.upflow8_backward(g_flow_up.float().contiguous(), H, W, None)
            dd8.zero_()
            dd8[:, :2] = _pm(dflow)
        else:
            dd8.zero_()
        hd = R("hd")
        dhd = ar.take("dhd", t, 128)
        dgrad("fh2", dd8, 3, 3, dhd, 128, mask=hd)
        # ConvGRU; the gate backward runs in the data-gradient epilogues (ops/update_fused.py):
        # fh1's data gradient = dH (+ incoming d net) -> dq, dz, carry; q's -> dr, d h; z||r's ->
        # bf16 d net, d inp, ReLU'-masked d motion.  G = [d h | d inp | d motion] (fp32)
        h = ar.rows("h", t, t + 1)
        zr, q = R("zr"), R("q")
        # per-forward [iters, P, GX] rows: the d inp columns are summed once by step 0's backward
        if run.g_all is None:
            run.g_all = torch.empty(run.iters, P, GX, device=dev, dtype=torch.float32)
        G = run.g_all[t]
        carry = torch.empty(P, HID, device=dev, dtype=torch.float32)
        dq = ar.take("dq", t, HID)
        dzr = ar.take("dzr", t, 2 * HID)
        C.conv_fwd([dhd], run.wd["fh1"], gd(3, 3), HID, carry, epi=C.EPI_GRU_BWD_A, h=h, z=zr[:, :HID], g0=q,
                   out2=dq, out3=dzr[:, :HID], carry=carry, gru_cols=HID,
                   addsrc=_pm(g_net).to(run.dt16).contiguous() if g_net is not None else None)
        C.conv_fwd([dq], run.wd["q"], gd(3, 3), GX, G, epi=C.EPI_GRU_BWD_B, h=h, g0=zr[:, HID:], carry=carry,
                   out3=dzr[:, HID:], gru_cols=HID)
        motion, cf, f1 = R("motion"), R("cf"), R("f1")
        dmo = ar.take("dmo", t, 80)
        d_net = torch.empty(P, HID, device=dev, dtype=run.dt16)
        # relu' of the motion features; the flow channels -> coords (detached)
        C.conv_fwd([dzr], run.wd["zr"], gd(3, 3), GX, G, epi=C.EPI_GRU_BWD_LAST, acc_c0=0, out3=d_net, gru_cols=HID,
                   cout=dmo, cmask=motion, cm_c0=HID + CTX, cm_valid=80)

        # motion encoder
        dcf = ar.take("dcf", t, 128)
        dgrad("conv", dmo, 3, 3, dcf, 128, mask=cf)
        dcorr = torch.empty(P, CORR_PAD, device=dev, dtype=run.dt16)
        dgrad("convc1", dcf[:, :96], 1, 1, dcorr, CORR_PAD)
        df1 = ar.take("df1", t, 64)
        dgrad("convf2", dcf[:, 96:], 3, 3, df1, 64, mask=f1)
        run.done.add(t)

        d_corr_in = None
        if ctx.has_corr_in:
            d_corr_in = dcorr.reshape(B, H, W, CORR_PAD)
        elif run.pyr is not None and run.pyr.levels:
            run.pyr.add_grad(run.coords[t], dcorr.reshape(B, H, W, CORR_PAD))
        d_net = _nchw(d_net if ctx.net_dtype == run.dt16 else d_net.to(ctx.net_dtype), B, H, W)
        d_inp = None
        if t == 0:  # the last step backward to run (every other step's d net feeds it)
            done = sorted(run.done)
            gall = run.g_all if len(done) == run.iters else run.g_all[done]
            d_inp = _nchw(gall[:, :, HID:HID + CTX].sum(0), B, H, W)
            run.g_all = None
        # the tokens only order the autograd graph (their nodes run after every step's backward
        # whatever they receive): no gradient, no fill / accumulate kernels
        return None, None, d_net, d_inp, d_corr_in, None, None, None, None


class FusedSmallUpdate:
    """Per-forward driver of the fused RAFT-small refinement steps."""

    corr_pad = CORR_PAD

    def __init__(self, block, inp: torch.Tensor, iters: int, pyramid=None, dt16=torch.bfloat16):
        keep = torch.is_grad_enabled()
        self.run = _Run(block, inp, iters, pyramid=pyramid, keep=keep, dt16=dt16)
        self.token = _PackWeights.apply(self.run, *_params(block))
        self.inp32 = inp.float().contiguous(memory_format=torch.channels_last)

    def step(self, t: int, net, coords1, ptoken=None, corr=None,
             upsample: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor], torch.Tensor]:
        if ptoken is None:
            ptoken = self.token.new_zeros(())
        up = upsample or torch.is_grad_enabled()  # skipping needs a forward nobody backpropagates
        return _Step.apply(self.token, ptoken, net, self.inp32, corr, coords1.detach().float().contiguous(),
                           self.run, t, up)


def supported(block) -> bool:
    from ..models.update import SmallUpdateBlock

    return isinstance(block, SmallUpdateBlock)
