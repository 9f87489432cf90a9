"""fp32 RAFT-small refinement step on the hand-written kernels (split-bf16 mode), training and
inference.

The small-model counterpart of ``ops/update_split.py`` (same operand planes, packing and
two-GEMM weight gradients; see there) for the reference's SmallUpdateBlock
(core/update.py:16-31 ConvGRU, :62-77 SmallMotionEncoder, :99-112; core/raft.py:131-134
upflow8) -- the ``is_small: true`` configuration of the ROS node (ros/config/config.yaml:3)
and ``demo.py --small`` / ``evaluate.py --small`` without ``--mixed_precision``:

  lookup (4 x 49 taps, fp32)            -> corr  [hi|lo|hi] of 200 (196 real)
  coords1 - grid                        -> flow8 [8], motion[:, 80:82]
  corr --convc1 1x1--> cf[:, :96];  flow8 --convf1 7x7--> f1 --convf2 3x3--> cf[:, 96:]
  cf --conv 3x3--> motion[:, :80]       (motion planes of 88: 82 real, zero padded)
  [h | inp | motion] --z||r 3x3 (fp32 sigmoid, r*h)--> zr, rh
  [rh | inp | motion] --q 3x3 (fp32 tanh + blend)--> h'
  h' --flow_head.conv1 3x3--> hd --flow_head.conv2 3x3--> delta (fp32);  upflow8
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

from . import conv as C
from ._ext import ops
from .update_fused import _Arena, _nchw, _pm
from .update_split import _I32, SplitWeightToken, _SplitToken, _sp, wgrad_split_params

HID, CTX = 96, 64
MOT_PAD = 88
CORR_PAD = 200
GX = HID + CTX + MOT_PAD  # [d h | d inp | d motion] rows of the GRU data gradients (248)
_GRU_SRC = [[(HID, HID)], [(CTX, CTX)], [(82, MOT_PAD)]]

# name -> (modules getter, forward source segments, data-gradient output segments or None,
# dY split groups (c0, n, G))
_LAYERS = [
    ("convc1", lambda b: (b.encoder.convc1,), [[(196, CORR_PAD)]], [(196, CORR_PAD)], [(0, 96, 96)]),
    ("convf1", lambda b: (b.encoder.convf1,), [[(2, 8)]], None, [(0, 64, 64)]),
    ("convf2", lambda b: (b.encoder.convf2,), [[(64, 64)]], [(64, 64)], [(0, 32, 32)]),
    ("conv", lambda b: (b.encoder.conv,), [[(128, 128)]], [(128, 128)], [(0, 80, 80)]),
    ("zr", lambda b: (b.gru.convz, b.gru.convr), _GRU_SRC, [s for src in _GRU_SRC for s in src], [(0, 192, 192)]),
    ("q", lambda b: (b.gru.convq,), _GRU_SRC, [s for src in _GRU_SRC for s in src], [(0, HID, HID)]),
    ("fh1", lambda b: (b.flow_head.conv1,), [[(HID, HID)]], [(HID, HID)], [(0, 128, 128)]),
    ("fh2", lambda b: (b.flow_head.conv2,), [[(128, 128)]], [(128, 128)], [(0, 2, 8)]),
]
# weight-gradient operands: (split sources (arena name, plane width), split dY (name, plane width))
_WGRAD = {
    "convc1": ([("corr", CORR_PAD)], ("dcfc", 96)),
    "convf1": ([("flow8", 8)], ("df1", 64)),
    "convf2": ([("f1", 64)], ("dcff", 32)),
    "conv": ([("cf", 128)], ("dmo", 80)),
    "zr": ([("h", HID), ("inp", CTX), ("motion", MOT_PAD)], ("dzr", 192)),
    "q": ([("rh", HID), ("inp", CTX), ("motion", MOT_PAD)], ("dq", HID)),
    "fh1": ([("h+", HID)], ("dhd", 128)),
    "fh2": ([("hd", 128)], ("dd8", 8)),
}
_DY_NAMES = ("dd8", "dhd", "dq", "dzr", "dmo", "dcfc", "dcff", "df1")


def _params(block) -> List[torch.Tensor]:
    out = []
    for _, mods, *_ in _LAYERS:
        for m in mods(block):
            out += [m.weight, m.bias]
    return out


class _SRun:
    def __init__(self, block, inp: torch.Tensor, coords0: torch.Tensor, iters: int, pyramid=None, keep: bool = True):
        B, _, H, W = inp.shape
        self.dims = (B, H, W)
        self.P = P = B * H * W
        self.iters = iters
        self.block = block
        self.pyr = pyramid
        self.keep = keep
        self.arena = _Arena(iters, P, inp.device, keep)
        self.coords0 = coords0
        self.done = set()
        self.grad_out: Optional[List[torch.Tensor]] = None
        self.g_all: Optional[torch.Tensor] = None
        self.dnet: Dict[int, torch.Tensor] = {}
        self.coords: Dict[int, torch.Tensor] = {}
        self.wf, self.bias, self.wd = {}, {}, {}
        gdys = [dyg[0][2] if (keep and dsegs is not None) else 0 for _, _, _, dsegs, dyg in _LAYERS]
        packed = C.pack_weights_multi(
            [([m.weight for m in mods(block)], [m.bias for m in mods(block)], [s for src in fsrc for s in src], 1.0,
              gdy) for (_, mods, fsrc, _, _), gdy in zip(_LAYERS, gdys)], split=True)
        for (name, *_), gdy, (wf, wd, b) in zip(_LAYERS, gdys, packed):
            self.wf[name], self.bias[name] = wf, b
            if gdy:
                self.wd[name] = wd
        self.inp_s = C.split_pack(_pm(inp.detach().float()).contiguous(),
                                  torch.empty(P, 3 * CTX, device=inp.device, dtype=torch.bfloat16), CTX)

    def geom(self, kh, kw, T: int = 1):
        B, H, W = self.dims
        return C.geom(T * B, H, W, kh, kw, kh // 2, kw // 2)

    def geom_d(self, kh, kw):
        B, H, W = self.dims
        return C.geom(B, H, W, kh, kw, kh - 1 - kh // 2, kw - 1 - kw // 2)

    def take(self, name, t, width, dtype=torch.bfloat16, slots=None):
        if name == "h" and not self.keep:  # without autograd: a ping-pong pair of hidden states
            ring = self.arena.bufs.get("h")
            if ring is None:
                ring = self.arena.bufs["h"] = torch.empty(2, self.P, width, device=self.arena.device, dtype=dtype)
            return ring[t % 2]
        return self.arena.take(name, t, width, dtype=dtype, slots=slots)

    def alloc_weight_grads(self) -> List[torch.Tensor]:
        """Empty parameter gradients in ``weight_grads`` order, on the current stream."""
        out: List[torch.Tensor] = []
        for _, mods, *_ in _LAYERS:
            for m in mods(self.block):
                out += [torch.empty_like(m.weight), torch.empty_like(m.bias)]
        return out

    def weight_grads(self, out_bufs: Optional[List[torch.Tensor]] = None) -> List[torch.Tensor]:
        T, P, ar = self.iters, self.P, self.arena
        for t in range(T):
            if t not in self.done:
                for name in _DY_NAMES:
                    if name in ar.bufs:
                        ar.rows(name, t, t + 1).zero_()

        def rows(name, t0, t1):
            if name == "inp":
                return self.inp_s
            if name == "h+":
                return ar.rows("h", t0 + 1, t1 + 1)
            return ar.rows(name, t0, t1)

        out: List[torch.Tensor] = []
        gi = 0
        for name, mods, fsrc, _dsegs, _dyg in _LAYERS:
            ms = mods(self.block)
            if out_bufs is not None:
                wg = [out_bufs[gi + 2 * i] for i in range(len(ms))]
                bg = [out_bufs[gi + 2 * i + 1] for i in range(len(ms))]
            else:
                wg = [torch.empty_like(m.weight) for m in ms]
                bg = [torch.empty_like(m.bias) for m in ms]
            gi += 2 * len(ms)
            kh, kw = ms[0].weight.shape[2:]
            segs = [s for src in fsrc for s in src]
            srcs_spec, (dyn, gdy) = _WGRAD[name]
            multi = len(srcs_spec) > 1
            per_iter = 6 * P * (sum(w for _, w in srcs_spec) if multi else max(w for _, w in srcs_spec) + gdy)
            chunk = max(1, min(T, _I32 // max(per_iter, 1)))
            for t0 in range(0, T, chunk):
                t1 = min(T, t0 + chunk)
                srcs = [(rows(n, t0, t1)[:, :3 * w], w) for n, w in srcs_spec]
                wgrad_split_params(srcs, rows(dyn, t0, t1), gdy, self.geom(kh, kw, t1 - t0), wg, bg, segs,
                                   concat=multi, accumulate=t0 > 0)
            for w, b in zip(wg, bg):
                out += [w, b]
        return out


def weight_token(block):
    """The early-created weight-gradient token (ops/update_split.py SplitWeightToken)."""
    return SplitWeightToken(block, _params)


class _Step(torch.autograd.Function):
    @staticmethod
    def forward(ctx, wtoken, ptoken, net, inp32, corr_in, coords1, run: _SRun, t: int, up: bool = True):
        B, H, W = run.dims
        P = run.P
        dev = coords1.device
        k = ops()
        g = run.geom

        h0 = run.take("h", t, 3 * HID, slots=run.iters + 1)
        if net.data_ptr() != h0.data_ptr():
            C.split_pack(_pm(net.float()).contiguous(), h0, HID)
        corr = run.take("corr", t, 3 * CORR_PAD)
        flow8 = run.take("flow8", t, 24)
        motion = run.take("motion", t, 3 * MOT_PAD)
        if run.pyr is not None:  # one launch: split features + the split flow operand
            k.corr_lookup_split_into(run.pyr.levels, coords1, run.pyr.radius, corr, CORR_PAD, flow8, motion[:, 80:],
                                     MOT_PAD)
            motion[:, 82:MOT_PAD].zero_()
            motion[:, MOT_PAD + 82:2 * MOT_PAD].zero_()
            motion[:, 2 * MOT_PAD + 82:].zero_()
        else:
            C.split_pack(corr_in.reshape(P, -1).float().contiguous(), corr, CORR_PAD, 0, CORR_PAD)
            flow = (coords1 - run.coords0).permute(0, 2, 3, 1).reshape(P, 2).contiguous()
            C.split_pack(flow, flow8, 8, 0, 8)
            C.split_pack(flow, motion, MOT_PAD, 80, 8)  # flow at 80..81, zeros 82..87

        cf = run.take("cf", t, 384)
        f1 = run.take("f1", t, 192)
        C.conv_fwd([corr], run.wf["convc1"], g(1, 1), 96, cf, bias=run.bias["convc1"], act=1, split=_sp(128))
        C.conv_fwd([flow8], run.wf["convf1"], g(7, 7), 64, f1, bias=run.bias["convf1"], act=1, split=_sp(64))
        C.conv_fwd([f1], run.wf["convf2"], g(3, 3), 32, cf[:, 96:], bias=run.bias["convf2"], act=1, split=_sp(128))
        C.conv_fwd([cf], run.wf["conv"], g(3, 3), 80, motion, bias=run.bias["conv"], act=1, split=_sp(MOT_PAD))

        inp = run.inp_s
        zr = run.take("zr", t, 576)
        rh = run.take("rh", t, 3 * HID)
        C.conv_fwd([h0, inp, motion], run.wf["zr"], g(3, 3), 2 * HID, zr, bias=run.bias["zr"], epi=C.EPI_GRU_ZR,
                   h=h0, out2=rh, split=_sp(HID, HID, HID))
        hn = run.take("h", t + 1, 3 * HID, slots=run.iters + 1)
        q = run.take("q", t, 3 * HID)
        C.conv_fwd([rh, inp, motion], run.wf["q"], g(3, 3), HID, hn, bias=run.bias["q"], epi=C.EPI_GRU_Q, h=h0,
                   z=zr, out2=q, split=_sp(HID, HID, HID, HID))

        hd = run.take("hd", t, 384)
        C.conv_fwd([hn], run.wf["fh1"], g(3, 3), 128, hd, bias=run.bias["fh1"], act=1, split=_sp(128))
        delta = torch.empty(P, 8, device=dev, dtype=torch.float32)
        C.conv_fwd([hd], run.wf["fh2"], g(3, 3), 2, delta, bias=run.bias["fh2"])
        coords_out = torch.empty_like(coords1)
        flow_lo = torch.empty_like(coords1)
        k.apply_delta(coords1, delta, coords_out, flow_lo)
        flow_up = k.upflow8(flow_lo) if up else None

        ctx.run, ctx.t = run, t
        ctx.corr_shape = None if corr_in is None else corr_in.shape
        run.coords[t] = coords1
        ctx.mark_non_differentiable(coords_out)
        ctx.set_materialize_grads(False)
        return _nchw(hn, B, H, W)[:, :HID], flow_up, coords_out

    @staticmethod
    def backward(ctx, g_net, g_flow_up, _g_coords):
        run: _SRun = ctx.run
        t = ctx.t
        B, H, W = run.dims
        P = run.P
        dev = run.inp_s.device
        k = ops()
        gd = run.geom_d
        R = lambda name: run.arena.rows(name, t, t + 1)  # noqa: E731

        dd8 = run.take("dd8", t, 24)
        if g_flow_up is not None:
            dflow = k.upflow8_backward(g_flow_up.float().contiguous(), H, W, None)
            C.split_pack(_pm(dflow).contiguous(), dd8, 8, 0, 8)
        else:
            dd8.zero_()
        hd = R("hd")
        dhd = run.take("dhd", t, 384)
        C.conv_fwd([dd8], run.wd["fh2"], gd(3, 3), 128, dhd, epi=C.EPI_GRAD, mask=hd[:, :128], split=_sp(128))

        h, zr, q = run.arena.rows("h", t, t + 1), R("zr"), R("q")
        if run.g_all is None:
            run.g_all = torch.empty(run.iters, P, GX, device=dev, dtype=torch.float32)
        G = run.g_all[t]
        carry = torch.empty(P, HID, device=dev, dtype=torch.float32)
        dq = run.take("dq", t, 3 * HID)
        dzr = run.take("dzr", t, 576)
        dnext = run.dnet.pop(t + 1, None)
        if dnext is None and g_net is not None:
            dnext = C.split_pack(_pm(g_net.float()).contiguous(),
                                 torch.empty(P, 3 * HID, device=dev, dtype=torch.bfloat16), HID)
        C.conv_fwd([dhd], run.wd["fh1"], gd(3, 3), HID, carry, epi=C.EPI_GRU_BWD_A, h=h, z=zr, g0=q, out2=dq,
                   out3=dzr, carry=carry, gru_cols=HID, addsrc=dnext,
                   split=_sp(0, HID, HID, HID, HID, 192, HID if dnext is not None else 0))
        C.conv_fwd([dq], run.wd["q"], gd(3, 3), GX, G, epi=C.EPI_GRU_BWD_B, h=h, g0=zr[:, 3 * HID:], carry=carry,
                   out3=dzr[:, HID:], gru_cols=HID, split=_sp(0, 0, HID, 0, HID, 192))
        motion, cf, f1 = R("motion"), R("cf"), R("f1")
        dmo = run.take("dmo", t, 240)
        d_net = torch.empty(P, 3 * HID, device=dev, dtype=torch.bfloat16)
        C.conv_fwd([dzr], run.wd["zr"], gd(3, 3), GX, G, epi=C.EPI_GRU_BWD_LAST, acc_c0=0, out3=d_net, gru_cols=HID,
                   cout=dmo, cmask=motion[:, :MOT_PAD], cm_c0=HID + CTX, cm_valid=80, split=_sp(0, 0, 0, 0, 0, HID, 0, 80))

        dcfc = run.take("dcfc", t, 288)
        dcff = run.take("dcff", t, 96)
        wdc = run.wd["conv"]
        C.conv_fwd([dmo], wdc[:96], gd(3, 3), 96, dcfc, epi=C.EPI_GRAD, mask=cf[:, :96], split=_sp(96))
        C.conv_fwd([dmo], wdc[96:128], gd(3, 3), 32, dcff, epi=C.EPI_GRAD, mask=cf[:, 96:128], split=_sp(32))
        dcorr = torch.empty(P, CORR_PAD, device=dev, dtype=torch.float32)
        C.conv_fwd([dcfc], run.wd["convc1"], gd(1, 1), CORR_PAD, dcorr, epi=C.EPI_GRAD)
        df1 = run.take("df1", t, 192)
        C.conv_fwd([dcff], run.wd["convf2"], gd(3, 3), 64, df1, epi=C.EPI_GRAD, mask=f1[:, :64], split=_sp(64))

        d_corr_in = None
        if ctx.corr_shape is not None:
            d_corr_in = dcorr[:, :ctx.corr_shape[-1]].reshape(ctx.corr_shape)
        elif run.pyr is not None and run.pyr.levels:
            run.pyr.add_grad(run.coords[t], dcorr.view(B, H, W, CORR_PAD))
        run.dnet[t] = d_net
        run.done.add(t)
        d_net_out = d_inp = None
        if t == 0:
            # the parameter gradients the tail stream writes: main-stream memory taken before the
            # event it waits for (ops/update_split.py _SplitToken.backward)
            run.grad_out = run.alloc_weight_grads()
            run.steps_done = torch.cuda.Event()
            run.steps_done.record(torch.cuda.current_stream(dev))
            d_net_out = _nchw(d_net[:, :HID].float() + d_net[:, HID:2 * HID].float(), B, H, W)
            done = sorted(run.done)
            gall = run.g_all if len(done) == run.iters else run.g_all[done]
            d_inp = _nchw(gall[:, :, HID:HID + CTX].sum(0), B, H, W)
            run.g_all = None
            run.dnet.clear()
        return None, None, d_net_out, d_inp, d_corr_in, None, None, None, None


class SplitSmallUpdate:
    """Per-forward driver of the fp32 (split-bf16) RAFT-small refinement step (training: with
    autograd; inference: ``torch.no_grad`` / ``inference_mode``)."""

    def __init__(self, block, inp: torch.Tensor, coords0: torch.Tensor, iters: int, pyramid=None,
                 token: Optional[SplitWeightToken] = None):
        self.run = _SRun(block, inp, coords0, iters, pyramid=pyramid, keep=torch.is_grad_enabled())
        if token is not None and self.run.keep:
            token.run = self.run
            self.token = token.tensor
        else:
            self.token = _SplitToken.apply(self.run, *_params(block))
        self.inp32 = inp.float().contiguous(memory_format=torch.channels_last)

    def step(self, t: int, net, coords1, ptoken=None, corr=None,
             upsample: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor], torch.Tensor]:
        if ptoken is None:
            ptoken = self.token.new_zeros(())
        up = upsample or torch.is_grad_enabled()
        return _Step.apply(self.token, ptoken, net, self.inp32, corr, coords1.detach().float().contiguous(),
                           self.run, t, up)


def supported(block) -> bool:
    from ..models.update import SmallUpdateBlock

    return isinstance(block, SmallUpdateBlock)
