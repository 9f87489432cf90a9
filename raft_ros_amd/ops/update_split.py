"""fp32 RAFT-base refinement step for TRAINING on the hand-written kernels (split-bf16 mode).

Without AMP the reference trains every conv in fp32 (``train.py:230`` has no autocast unless
``--mixed_precision``; ``train_standard.sh:3-6``).  This module runs that recipe on the same
implicit-GEMM kernels as the bf16 fused step (``ops/update_fused.py``) in split-bf16 mode:

* every activation, and every data gradient that feeds a GEMM, is stored as ``[hi | lo | hi]``
  bf16 planes of a group width ``G`` (``ops.conv.split_pack``, the kernels' ``split_*``
  epilogue stores; csrc/kernel_abi.h ``ConvFwdArgs::split_g``);
* forward convs pack ``[W_hi | W_hi | W_lo]`` along K and data-gradient convs the same split
  of the flipped / transposed weight along the dY planes, so each bf16 MFMA GEMM computes
  ``x_hi W_hi + x_lo W_hi + x_hi W_lo`` with fp32 accumulation: the fp32 product up to the
  dropped ``x_lo W_lo`` term (~2^-16 relative, finer than the TF32 convolutions cuDNN runs for
  "fp32" training by default);
* weight gradients: two GEMMs per conv over all iterations at once (the weights are shared by
  every iteration, core/raft.py:122-139), ``[X_hi | X_lo]^T dY_hi`` and ``X_hi^T dY_lo``, folded
  into the fp32 parameter layout;
* the GRU gate math, the coordinates, the correlation features, the mask logits and every
  gradient row that accumulates (the GRU's ``[d h | d inp | d motion]``) stay fp32.

Per iteration (reference core/raft.py:122-139, core/update.py:79-136) one autograd node
``_SplitStep``; one ``_SplitToken`` node whose backward (after every step's) computes the
batched weight gradients.  The hidden-state gradient between steps travels out of band
(``_SRun.dnet``) as split planes, so it is never rounded to the dtype of an autograd edge.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

from . import conv as C
from ._ext import ops
from .streams import aux_stream
from .update_fused import _Arena, _nchw, _pm, _side_stream

HID = 128
CORR_PAD = 328
_I32 = (1 << 31) - 1
# (B, H, W) pixels per step above which the weight gradients run in iteration chunks
# (32-bit byte offsets of the kernels' buffer descriptors)

# name -> (modules getter, forward source segments (one list per split source), data-gradient
# output segments (None: no data gradient), dY split groups (c0, n, G), output scale)
_LAYERS = [
    ("convc1", lambda b: (b.encoder.convc1,), [[(324, CORR_PAD)]], [(324, CORR_PAD)], [(0, 256, 256)], 1.0),
    ("convc2", lambda b: (b.encoder.convc2,), [[(256, 256)]], [(256, 256)], [(0, 192, 192)], 1.0),
    ("convf1", lambda b: (b.encoder.convf1,), [[(2, 8)]], None, [(0, 128, 128)], 1.0),
    ("convf2", lambda b: (b.encoder.convf2,), [[(128, 128)]], [(128, 128)], [(0, 64, 64)], 1.0),
    ("conv", lambda b: (b.encoder.conv,), [[(256, 256)]], [(256, 256)], [(0, 126, HID)], 1.0),
    ("zr1", lambda b: (b.gru.convz1, b.gru.convr1), [[(HID, HID)]] * 3, [(HID, HID)] * 3, [(0, 256, 256)], 1.0),
    ("q1", lambda b: (b.gru.convq1,), [[(HID, HID)]] * 3, [(HID, HID)] * 3, [(0, HID, HID)], 1.0),
    ("zr2", lambda b: (b.gru.convz2, b.gru.convr2), [[(HID, HID)]] * 3, [(HID, HID)] * 3, [(0, 256, 256)], 1.0),
    ("q2", lambda b: (b.gru.convq2,), [[(HID, HID)]] * 3, [(HID, HID)] * 3, [(0, HID, HID)], 1.0),
    ("heads", lambda b: (b.flow_head.conv1, b.mask[0]), [[(HID, HID)]], [(HID, HID)], [(0, 512, 512)], 1.0),
    ("fh2", lambda b: (b.flow_head.conv2,), [[(256, 256)]], [(256, 256)], [(0, 2, 8)], 1.0),
    ("mask2", lambda b: (b.mask[2],), [[(256, 256)]], [(256, 256)], [(0, 576, 576)], 0.25),  # core/update.py:135
]
_BY_NAME = {name: spec for name, *spec in _LAYERS}

# weight-gradient operands: name -> (split sources (arena name, plane width, first column),
# split dY (arena name, plane width)).  "h" = the step's input hidden state, "h+" its output,
# "inp" the iteration-shared context features (a periodic source).
_WGRAD = {
    "convc1": ([("corr", CORR_PAD, 0)], ("dc1", 256)),
    "convc2": ([("c1", 256, 0)], ("dcfc", 192)),
    "convf1": ([("flow8", 8, 0)], ("df1", HID)),
    "convf2": ([("f1", HID, 0)], ("dcff", 64)),
    "conv": ([("cf", 256, 0)], ("dmo", HID)),
    "zr1": ([("h", HID, 0), ("inp", HID, 0), ("motion", HID, 0)], ("dzr1", 256)),
    "q1": ([("rh1", HID, 0), ("inp", HID, 0), ("motion", HID, 0)], ("dq1", HID)),
    "zr2": ([("h1", HID, 0), ("inp", HID, 0), ("motion", HID, 0)], ("dzr2", 256)),
    "q2": ([("rh2", HID, 0), ("inp", HID, 0), ("motion", HID, 0)], ("dq2", HID)),
    "heads": ([("h+", HID, 0)], ("dhd", 512)),
    "fh2": ([("hd", 256, 0)], ("dd8", 8)),
    "mask2": ([("hd", 256, 768)], ("dmask", 576)),
}
# backward arena rows a step that fed no loss leaves unwritten (zeroed before the weight grads)
_DY_NAMES = ("dmask", "dd8", "dhd", "dq1", "dq2", "dzr1", "dzr2", "dmo", "dcfc", "dcff", "dc1", "df1")


def _params(block) -> List[torch.Tensor]:
    out = []
    for _, mods, *_ in _LAYERS:
        for m in mods(block):
            out += [m.weight, m.bias]
    return out


def _hi_lo(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    hi = w.to(torch.bfloat16).float()
    return hi, w - hi


def pack_dgrad_split(weights, cin_segments, dy_groups, scale: float = 1.0) -> torch.Tensor:
    """Data-gradient operand of a conv whose dY is stored as split planes: the rows of the
    (stacked, scaled) weight in dY column order -- per dY group (c0, n, G): W_hi, W_hi, W_lo, each
    zero-padded from n to G rows -- packed like ``ops.conv.pack_dgrad`` (flipped taps, k = tap *
    Cout' + n'), so dX = conv(dY_split, .) is dY_hi W_hi + dY_lo W_hi + dY_hi W_lo."""
    w = torch.cat([t.detach() for t in weights], 0).float() * scale
    hi, lo = _hi_lo(w)
    rows = []
    for c0, n, G in dy_groups:
        for part in (hi, hi, lo):
            blk = part[c0:c0 + n]
            if G > n:
                blk = torch.cat([blk, blk.new_zeros(G - n, *blk.shape[1:])], 0)
            rows.append(blk)
    we = torch.cat(rows, 0)
    return C.pack_dgrad(we, cin_segments, cout_pad=we.shape[0])


def _fold_planes(dw: torch.Tensor, N: int, taps: int, widths: List[int], planes: int) -> torch.Tensor:
    """(N, >=K) packed weight gradient over ``planes`` split planes per source -> (N, taps,
    sum(widths)) with the planes summed."""
    tot = planes * sum(widths)
    g = dw[:N, :taps * tot].reshape(N, taps, tot)
    if planes == 1:
        return g
    parts, c = [], 0
    for w in widths:
        parts.append(g[:, :, c:c + w] + g[:, :, c + w:c + 2 * w])
        c += 2 * w
    return torch.cat(parts, 2)


def wgrad_split(srcs, dy: torch.Tensor, G_dy: int, geom, shape, segments, scale: float = 1.0,
                concat: bool = False):
    """fp32-faithful weight / bias gradient of a conv over split operands.

    ``srcs``: (tensor, plane width) per split source (rows [hi | lo | hi]); ``dy``: split rows of
    plane width ``G_dy``.  Two GEMMs -- [X_hi | X_lo]^T dY_hi and X_hi^T dY_lo -- into packed fp32
    buffers, folded into ``shape`` (Cout, Cin, kh, kw) (``segments``: the real / padded input
    channels of each source) -> (dW, db), both times ``scale``.  ``concat``: materialise the
    sources as one operand per GEMM (multi-source layouts the kernels do not take: segments
    that are not multiples of 128 channels); periodic sources are repeated."""
    N, _, kh, kw = shape
    taps = kh * kw
    widths = [w for _, w in srcs]
    dev = dy.device
    out = []
    for planes, dyv in ((2, dy[:, :G_dy]), (1, dy[:, G_dy:2 * G_dy])):
        views = [t[:, :planes * w] for t, w in srcs]
        if concat and len(views) > 1:
            n = dy.shape[0]
            views = [torch.cat([v if v.shape[0] == n else v.repeat(n // v.shape[0], 1) for v in views], dim=1)]
        K = taps * planes * sum(widths)
        dw = torch.empty(N, -(-K // C.KBLK) * C.KBLK, device=dev, dtype=torch.float32)
        db = torch.empty(N, device=dev, dtype=torch.float32)
        C.conv_wgrad(views, dyv, geom, N, dw, db, accumulate=False)
        out.append((_fold_planes(dw, N, taps, widths, planes), db))
    g = out[0][0] + out[1][0]  # (N, taps, sum widths)
    dW = C.unpack_grad(g.reshape(N, -1), shape, segments)
    db = out[0][1] + out[1][1]
    if scale != 1.0:
        dW, db = dW * scale, db * scale
    return dW, db


def wgrad_split_params(srcs, dy: torch.Tensor, G_dy: int, geom, wgrads, bgrads, segments, scale: float = 1.0,
                       concat: bool = False, accumulate: bool = False) -> None:
    """``wgrad_split`` reduced straight into the parameter gradients ``wgrads`` / ``bgrads``
    (1..2 stacked parameters, any strides): [X_hi | X_lo]^T dY_hi with the hi / lo plane columns
    summed by the reduction (csrc/weights.hip, ConvParamDesc::fold), then X_hi^T dY_lo
    accumulated -- two GEMMs and two reductions per conv, no fold / unpack / add kernels."""
    v1 = [t[:, :2 * w] for t, w in srcs]
    v2 = [t[:, :w] for t, w in srcs]
    if concat and len(srcs) > 1:
        n = dy.shape[0]
        rep = lambda v: v if v.shape[0] == n else v.repeat(n // v.shape[0], 1)  # noqa: E731
        v1 = [torch.cat([rep(v) for v in v1], dim=1)]
        v2 = [torch.cat([rep(v) for v in v2], dim=1)]
    C.conv_wgrad_params(v1, dy[:, :G_dy], geom, wgrads, bgrads, segments, scale, accumulate=accumulate, fold=True)
    C.conv_wgrad_params(v2, dy[:, G_dy:2 * G_dy], geom, wgrads, bgrads, segments, scale, accumulate=True)


class _SRun:
    """Everything one RAFT forward's split steps share."""

    def __init__(self, block, inp: torch.Tensor, coords0: torch.Tensor, iters: int, pyramid=None,
                 keep: bool = True):
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
        self.g_all: Optional[torch.Tensor] = None
        self.grad_out: Optional[List[torch.Tensor]] = None
        self.dnet: Dict[int, torch.Tensor] = {}  # step -> split d(hidden state in) rows
        self.coords: Dict[int, torch.Tensor] = {}
        self.flows: Dict[int, torch.Tensor] = {}
        self.wf: Dict[str, torch.Tensor] = {}
        self.bias: Dict[str, torch.Tensor] = {}
        self.wd: Dict[str, torch.Tensor] = {}
        # one HIP launch for every conv: forward + (training) data-gradient operands, biases
        gdys = [dyg[0][2] if (keep and dsegs is not None) else 0 for _, _, _, dsegs, dyg, _ in _LAYERS]
        packed = C.pack_weights_multi(
            [([m.weight for m in mods(block)], [m.bias for m in mods(block)], [s for src in fsrc for s in src], scale,
              gdy) for (_, mods, fsrc, _, _, scale), gdy in zip(_LAYERS, gdys)], split=True)
        for (name, *_), gdy, (wf, wd, b) in zip(_LAYERS, gdys, packed):
            self.wf[name], self.bias[name] = wf, b
            if gdy:
                self.wd[name] = wd
        self.inp_s = C.split_pack(_pm(inp.detach().float()).contiguous(),
                                  torch.empty(P, 3 * HID, device=inp.device, dtype=torch.bfloat16), HID)

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

    # ------------------------------------------------------------ batched weight gradients
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
            if name == "h":
                return ar.rows("h", t0, t1)
            if name == "h+":
                return ar.rows("h", t0 + 1, t1 + 1)
            return ar.rows(name, t0, t1)

        out: List[torch.Tensor] = []
        gi = 0
        for name, mods, fsrc, _dsegs, _dyg, scale in _LAYERS:
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
            per_iter = max([3 * w * 2 * P for _, w, _ in srcs_spec] + [3 * gdy * 2 * P, 1536 * 2 * P])
            chunk = max(1, min(T, _I32 // per_iter))
            for t0 in range(0, T, chunk):
                t1 = min(T, t0 + chunk)
                srcs = [(rows(n, t0, t1)[:, c0:c0 + 3 * w], w) for n, w, c0 in srcs_spec]
                wgrad_split_params(srcs, rows(dyn, t0, t1), gdy, self.geom(kh, kw, t1 - t0), wg, bg, segs, scale,
                                   accumulate=t0 > 0)
            for w, b in zip(wg, bg):
                out += [w, b]
        return out


class SplitWeightToken:
    """Weight-gradient token created before the encoders (see ops/update_fused.py WeightToken):
    the batched split weight gradients run on the tail stream beside the encoders' backward."""

    def __init__(self, block, params_fn=None):
        self.run = None
        self.tensor = _SplitToken.apply(self, *(params_fn or _params)(block))


class _SplitToken(torch.autograd.Function):
    """Token node: its backward (after every step's backward) runs the batched weight grads."""

    @staticmethod
    def forward(ctx, holder, *params):
        ctx.holder = holder  # a run, or a SplitWeightToken whose run is filled in later
        ctx.set_materialize_grads(False)
        return params[0].new_empty(())  # ordering token: its value is never read (no fill launch)

    @staticmethod
    def backward(ctx, gtoken):
        h = ctx.holder
        run = h.run if isinstance(h, SplitWeightToken) else h
        ctx.holder = None  # break the token <-> graph cycle (see ops/update_fused.py _PackWeights)
        if isinstance(h, SplitWeightToken):
            h.run = None
        if run is None:
            return (None,) * len(ctx.needs_input_grad)
        ev = getattr(run, "steps_done", None)
        if ev is not None:
            cur = torch.cuda.current_stream(run.inp_s.device)
            ws = aux_stream(cur.device, "tail")
            ws.wait_event(ev)
            with torch.cuda.stream(ws):
                # straight into main-stream gradients allocated before the event ws waited for
                # (ops/update_fused.py _PackWeights.backward): no record_stream, no copies
                grads = run.weight_grads(out_bufs=run.grad_out)
            cur.wait_stream(ws)
            run.grad_out = None
            # the arena is this stream's memory, released after this stream waited for ws
        else:
            grads = run.weight_grads()
        run.arena.bufs.clear()
        run.dnet.clear()
        return (None, *grads)


def _one_block(grads):
    from .encoder import _one_block as ob

    return ob(grads)


def _sp(g=0, g2=0, h=0, z=0, g0=0, g3=0, add=0, cout=0):
    """Split descriptor of one conv launch (csrc/kernel_abi.h ConvFwdArgs::split_*)."""
    return [g, g2, h, z, g0, g3, add, cout]


class _SplitStep(torch.autograd.Function):
    @staticmethod
    def forward(ctx, wtoken, ptoken, net, inp32, corr_in, coords1, run: _SRun, t: int, up: bool = True):
        B, H, W = run.dims
        P = run.P
        dev = coords1.device
        k = ops()
        g = run.geom
        S1 = lambda G: _sp(G)  # noqa: E731

        h0 = run.take("h", t, 3 * HID, slots=run.iters + 1)
        if net.data_ptr() != h0.data_ptr():  # the first step: fp32 hidden state from the context encoder
            C.split_pack(_pm(net.float()).contiguous(), h0, HID)
        corr = run.take("corr", t, 3 * CORR_PAD)
        flow8 = run.take("flow8", t, 24)
        motion = run.take("motion", t, 3 * HID)
        if run.pyr is not None:  # one launch: split features + the split flow operand
            k.corr_lookup_split_into(run.pyr.levels, coords1, run.pyr.radius, corr, CORR_PAD, flow8, motion[:, 126:],
                                     HID)
        else:
            C.split_pack(corr_in.reshape(P, -1).float().contiguous(), corr, CORR_PAD, 0, CORR_PAD)
            flow = (coords1 - run.coords0).permute(0, 2, 3, 1).reshape(P, 2).contiguous()
            C.split_pack(flow, flow8, 8, 0, 8)
            C.split_pack(flow, motion, HID, 126, 2)

        c1 = run.take("c1", t, 768)
        cf = run.take("cf", t, 768)
        f1 = run.take("f1", t, 3 * HID)
        main = torch.cuda.current_stream(dev)
        side = _side_stream(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            C.conv_fwd([flow8], run.wf["convf1"], g(7, 7), 128, f1, bias=run.bias["convf1"], act=1, split=S1(128))
            C.conv_fwd([f1], run.wf["convf2"], g(3, 3), 64, cf[:, 192:], bias=run.bias["convf2"], act=1,
                       split=S1(256))
        C.conv_fwd([corr], run.wf["convc1"], g(1, 1), 256, c1, bias=run.bias["convc1"], act=1, split=S1(256))
        C.conv_fwd([c1], run.wf["convc2"], g(3, 3), 192, cf, bias=run.bias["convc2"], act=1, split=S1(256))
        main.wait_stream(side)
        C.conv_fwd([cf], run.wf["conv"], g(3, 3), 126, motion, bias=run.bias["conv"], act=1, split=S1(HID))

        inp = run.inp_s
        h = h0
        for stage, (kh, kw) in ((1, (1, 5)), (2, (5, 1))):
            zr = run.take(f"zr{stage}", t, 768)
            rh = run.take(f"rh{stage}", t, 3 * HID)
            C.conv_fwd([h, inp, motion], run.wf[f"zr{stage}"], g(kh, kw), 2 * HID, zr, bias=run.bias[f"zr{stage}"],
                       epi=C.EPI_GRU_ZR, h=h, out2=rh, split=_sp(HID, HID, HID))
            hn = run.take("h1", t, 3 * HID) if stage == 1 else run.take("h", t + 1, 3 * HID, slots=run.iters + 1)
            q = run.take(f"q{stage}", t, 3 * HID)
            C.conv_fwd([rh, inp, motion], run.wf[f"q{stage}"], g(kh, kw), HID, hn, bias=run.bias[f"q{stage}"],
                       epi=C.EPI_GRU_Q, h=h, z=zr, out2=q, split=_sp(HID, HID, HID, HID))
            h = hn

        hd = run.take("hd", t, 1536)
        nh = 512 if up else 256
        C.conv_fwd([h], run.wf["heads"][:nh], g(3, 3), nh, hd, bias=run.bias["heads"][:nh], act=1, split=S1(256))
        delta = torch.empty(P, 8, device=dev, dtype=torch.float32)
        C.conv_fwd([hd[:, :768]], run.wf["fh2"], g(3, 3), 2, delta, bias=run.bias["fh2"])
        coords_out = torch.empty_like(coords1)
        flow_lo = torch.empty_like(coords1)
        k.apply_delta(coords1, delta, coords_out, flow_lo)
        flow_up = None
        if up:
            mask = run.take("mask", t, 576, dtype=torch.float32)
            C.conv_fwd([hd[:, 768:]], run.wf["mask2"], g(1, 1), 576, mask, bias=run.bias["mask2"])
            flow_up = k.convex_upsample(flow_lo, _nchw(mask, B, H, W))
        ctx.run, ctx.t = run, t
        ctx.corr_shape = None if corr_in is None else corr_in.shape
        run.coords[t] = coords1
        run.flows[t] = flow_lo
        ctx.mark_non_differentiable(coords_out)
        ctx.set_materialize_grads(False)
        return _nchw(h, B, H, W)[:, :HID], flow_up, coords_out

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

        hd = R("hd")
        dmask = run.take("dmask", t, 3 * 576)
        dd8 = run.take("dd8", t, 24)
        if g_flow_up is not None:
            mask = R("mask")
            dflow, dm = k.convex_upsample_backward(run.flows[t], _nchw(mask, B, H, W), g_flow_up)
            C.split_pack(_pm(dm), dmask, 576)
            C.split_pack(_pm(dflow).contiguous(), dd8, 8, 0, 8)
        else:
            dmask.zero_()
            dd8.zero_()
        dhd = run.take("dhd", t, 1536)
        C.conv_fwd([dd8], run.wd["fh2"], gd(3, 3), 256, dhd, epi=C.EPI_GRAD, mask=hd[:, :256], split=_sp(512))
        C.conv_fwd([dmask], run.wd["mask2"], gd(1, 1), 256, dhd[:, 256:], epi=C.EPI_GRAD, mask=hd[:, 768:1024],
                   split=_sp(512))

        # ---- GRU stages in reverse (gate backward in the data-gradient epilogues, fp32 gates)
        stages = ((2, (5, 1)), (1, (1, 5)))
        gates = {}
        for stage, _ in stages:
            gates[stage] = (run.arena.rows("h", t, t + 1) if stage == 1 else R("h1"), R(f"zr{stage}"), R(f"q{stage}"),
                            run.take(f"dq{stage}", t, 3 * HID), run.take(f"dzr{stage}", t, 768))
        carry = torch.empty(P, HID, device=dev, dtype=torch.float32)

        def gate_a(stage, add=0):
            h, zr, q, dq, dzr = gates[stage]
            return dict(epi=C.EPI_GRU_BWD_A, h=h, z=zr, g0=q, out2=dq, out3=dzr, carry=carry, gru_cols=HID,
                        split=_sp(0, HID, HID, HID, HID, 256, add))

        dnext = run.dnet.pop(t + 1, None)
        if dnext is None and g_net is not None:  # the last step's hidden state fed a loss (external use)
            dnext = C.split_pack(_pm(g_net.float()).contiguous(),
                                 torch.empty(P, 3 * HID, device=dev, dtype=torch.bfloat16), HID)
        C.conv_fwd([dhd], run.wd["heads"], gd(3, 3), HID, carry, addsrc=dnext,
                   **gate_a(2, HID if dnext is not None else 0))

        if run.g_all is None:
            run.g_all = torch.empty(run.iters, P, 3 * HID, device=dev, dtype=torch.float32)
        G = run.g_all[t]
        motion = R("motion")
        dmo = run.take("dmo", t, 3 * HID)
        d_net = torch.empty(P, 3 * HID, device=dev, dtype=torch.bfloat16)
        for i, (stage, (kh, kw)) in enumerate(stages):
            h, zr, q, dq, dzr = gates[stage]
            C.conv_fwd([dq], run.wd[f"q{stage}"], gd(kh, kw), 3 * HID, G, epi=C.EPI_GRU_BWD_B,
                       acc_c0=(3 * HID if i == 0 else HID), h=h, g0=zr[:, 3 * HID:], carry=carry, out3=dzr[:, HID:],
                       gru_cols=HID, split=_sp(0, 0, HID, 0, HID, 256))
            if i + 1 < len(stages):
                C.conv_fwd([dzr], run.wd[f"zr{stage}"], gd(kh, kw), 3 * HID, G, acc_c0=0, **gate_a(stages[i + 1][0]))
            else:
                C.conv_fwd([dzr], run.wd[f"zr{stage}"], gd(kh, kw), 3 * HID, G, epi=C.EPI_GRU_BWD_LAST, acc_c0=0,
                           out3=d_net, gru_cols=HID, cout=dmo, cmask=motion[:, :HID], cm_c0=2 * HID, cm_valid=126,
                           split=_sp(0, 0, 0, 0, 0, HID, 0, HID))

        # ---- motion encoder
        cf, c1, f1 = R("cf"), R("c1"), R("f1")
        dcfc = run.take("dcfc", t, 576)
        dcff = run.take("dcff", t, 192)
        wdc = run.wd["conv"]
        C.conv_fwd([dmo], wdc[:192], gd(3, 3), 192, dcfc, epi=C.EPI_GRAD, mask=cf[:, :192], split=_sp(192))
        C.conv_fwd([dmo], wdc[192:256], gd(3, 3), 64, dcff, epi=C.EPI_GRAD, mask=cf[:, 192:256], split=_sp(64))
        df1 = run.take("df1", t, 3 * HID)
        dc1 = run.take("dc1", t, 768)
        C.conv_fwd([dcff], run.wd["convf2"], gd(3, 3), 128, df1, epi=C.EPI_GRAD, mask=f1[:, :HID], split=_sp(HID))
        C.conv_fwd([dcfc], run.wd["convc2"], gd(3, 3), 256, dc1, epi=C.EPI_GRAD, mask=c1[:, :256], split=_sp(256))
        dcorr = torch.empty(P, CORR_PAD, device=dev, dtype=torch.float32)
        C.conv_fwd([dc1], run.wd["convc1"], gd(1, 1), CORR_PAD, dcorr, epi=C.EPI_GRAD)
        d_corr_in = None
        if ctx.corr_shape is not None:
            n = ctx.corr_shape[-1]
            d_corr_in = dcorr[:, :n].reshape(ctx.corr_shape)
        elif run.pyr is not None and run.pyr.levels:
            run.pyr.add_grad(run.coords[t], dcorr.view(B, H, W, CORR_PAD))
        run.dnet[t] = d_net
        run.done.add(t)

        d_net_out = d_inp = None
        if t == 0:  # the last step backward to run
            # the parameter gradients the tail stream writes: main-stream memory taken before the
            # event it waits for (ops/update_split.py _SplitToken.backward)
            run.grad_out = run.alloc_weight_grads()
            run.steps_done = torch.cuda.Event()
            run.steps_done.record(torch.cuda.current_stream(dev))
            d_net_out = _nchw(d_net[:, :HID].float() + d_net[:, HID:2 * HID].float(), B, H, W)
            done = sorted(run.done)
            gi = run.g_all[:, :, HID:2 * HID] if len(done) == run.iters else run.g_all[done][:, :, HID:2 * HID]
            d_inp = _nchw(gi.sum(0), B, H, W)
            run.g_all = None
            run.dnet.clear()
        return None, None, d_net_out, d_inp, d_corr_in, None, None, None, None


class SplitTrainBasicUpdate:
    """Per-forward driver of the fp32 (split-bf16) fused refinement step, with autograd."""

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
        """-> (net (B, 128, H, W) hi-plane view, flow_up (B, 2, 8H, 8W) fp32, coords1 after the update)."""
        if ptoken is None:
            ptoken = self.token.new_zeros(())
        up = upsample or torch.is_grad_enabled()
        return _SplitStep.apply(self.token, ptoken, net, self.inp32, corr, coords1.detach().float().contiguous(),
                                self.run, t, up)


def supported(block) -> bool:
    from ..models.update import BasicUpdateBlock

    return isinstance(block, BasicUpdateBlock)
