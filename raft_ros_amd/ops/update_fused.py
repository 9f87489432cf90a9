"""Fused RAFT-base refinement step on hand-written HIP kernels (forward + backward).

One refinement iteration (reference core/raft.py:122-139 + core/update.py:79-136:
corr lookup -> BasicMotionEncoder -> SepConvGRU -> FlowHead + mask head ->
coords update -> convex upsampling) is ONE autograd node, ``_Step``, whose
forward runs 16 HIP launches:

  lookup (4 levels x 81 taps)          -> corr (P, 328)             [corr_lookup_into, which also
  coords1 - grid                       -> flow8 (P, 8), motion[:, 126:]   packs the flow operand]
  corr --convc1 1x1+relu--> c1 --convc2 3x3+relu--> cf[:, :192]
  flow8 --convf1 7x7+relu--> f1 --convf2 3x3+relu--> cf[:, 192:]
  cf --conv 3x3+relu--> motion[:, :126]
  [h | inp | motion] --z||r 1x5 (sigmoid, r*h epilogue)--> zr, rh
  [rh | inp | motion] --q 1x5 (tanh + GRU blend epilogue)--> h1          (x2: 5x1)
  h2 --[flow_head.conv1 || mask.0] 3x3+relu (one 512-wide conv)--> hd
  hd[:, :256] --flow_head.conv2 3x3--> delta;  hd[:, 256:] --0.25*mask.2 1x1--> mask
  coords1 + delta, flow = coords1 - grid   [apply_delta];  convex 8x upsample

Weight gradients are NOT computed per iteration.  The weights are shared by
every iteration (core/raft.py:122-139), so each step's backward only stores its
output gradients dY (bf16) in a per-forward arena, next to the activations its
forward stored there; ``_PackWeights.backward`` -- which autograd runs after
the last step's backward, since every step consumes its token -- then runs ONE
weight-gradient GEMM per conv over all ``iters * P`` pixels (the context
features, shared by all iterations, are a periodic source) and writes the
parameter gradients directly (csrc/weights.hip: fixed-order split reduction,
so the result is deterministic).  The dgrad chain stays per iteration.

Weights are packed (bf16 GEMM operands, forward and data-grad variants) by one
HIP launch per conv per RAFT forward (``ops.conv.pack_weights``).
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, List, Optional, Tuple

import torch

from . import conv as C
from .streams import aux_stream
from ._ext import ops

HID = 128
CORR_PAD = 328  # 4 * 81 = 324 lookup channels, padded to a multiple of 8
_I32 = (1 << 31) - 1

# name -> (modules getter, input segments (real, padded), output scale, needs a dgrad operand)
_LAYERS = [
    ("convc1", lambda b: (b.encoder.convc1,), [(324, CORR_PAD)], 1.0, True),
    ("convc2", lambda b: (b.encoder.convc2,), [(256, 256)], 1.0, True),
    ("convf1", lambda b: (b.encoder.convf1,), [(2, 8)], 1.0, False),
    ("convf2", lambda b: (b.encoder.convf2,), [(128, 128)], 1.0, True),
    ("conv", lambda b: (b.encoder.conv,), [(256, 256)], 1.0, True),
    ("zr1", lambda b: (b.gru.convz1, b.gru.convr1), [(128, 128)] * 3, 1.0, True),
    ("q1", lambda b: (b.gru.convq1,), [(128, 128)] * 3, 1.0, True),
    ("zr2", lambda b: (b.gru.convz2, b.gru.convr2), [(128, 128)] * 3, 1.0, True),
    ("q2", lambda b: (b.gru.convq2,), [(128, 128)] * 3, 1.0, True),
    ("heads", lambda b: (b.flow_head.conv1, b.mask[0]), [(128, 128)], 1.0, True),
    ("fh2", lambda b: (b.flow_head.conv2,), [(256, 256)], 1.0, True),
    ("mask2", lambda b: (b.mask[2],), [(256, 256)], 0.25, True),  # core/update.py:135
]
SEGMENTS = {name: segs for name, _, segs, _, _ in _LAYERS}


def _params(block) -> List[torch.Tensor]:
    out = []
    for _, mods, _, _, _ in _LAYERS:
        for m in mods(block):
            out += [m.weight, m.bias]
    return out


def _pm(t: torch.Tensor) -> torch.Tensor:
    """(B, C, H, W) channels-last tensor -> (P, C) pixel-major view (no copy)."""
    B, Ch, H, W = t.shape
    return t.permute(0, 2, 3, 1).reshape(B * H * W, Ch)


def _nchw(t: torch.Tensor, B: int, H: int, W: int) -> torch.Tensor:
    """(P, C) pixel-major -> (B, C, H, W) channels-last view (no copy)."""
    return t.reshape(B, H, W, t.shape[1]).permute(0, 3, 1, 2)


# backward arena buffers (name, channels) and the buffer order of fused_step_bwd (csrc/bindings.cpp
# step_exec::BwdBuf)
_BWD_ARENA = (("dmask", 576), ("dd8", 8), ("dhd", 512), ("dq1", HID), ("dq2", HID), ("dzr1", 2 * HID),
              ("dzr2", 2 * HID), ("dmo", HID), ("dcf", 256), ("dc1", 256), ("df1", 128))
_BWD_BUFS = ("hd", "mask", "h", "h1", "zr1", "zr2", "q1", "q2", "motion", "cf", "c1", "f1", "dmask", "dd8", "dhd",
             "dq1", "dq2", "dzr1", "dzr2", "dmo", "dcf", "dc1", "df1")


class _Arena:
    """Per-forward storage: one (slots * P, C) buffer per name, slot t at rows [t*P, (t+1)*P).

    While training every activation a step's backward or the batched weight gradient
    reads, and every deferred weight-gradient dY, lives here.  Without autograd
    (``keep=False``) ``take`` hands out per-call temporaries instead.
    """

    def __init__(self, iters: int, P: int, device, keep: bool, dtype=torch.bfloat16):
        self.iters, self.P, self.device, self.keep = iters, P, device, keep
        self.dtype = dtype  # the 16-bit activation dtype (bf16, or fp16 under fp16 AMP)
        self.bufs: Dict[str, torch.Tensor] = {}

    def take(self, name: str, t: int, C: int, dtype=None, slots: Optional[int] = None) -> torch.Tensor:
        dtype = dtype or self.dtype
        if not self.keep:
            return torch.empty(self.P, C, device=self.device, dtype=dtype)
        buf = self.bufs.get(name)
        if buf is None:
            buf = torch.empty((slots or self.iters) * self.P, C, device=self.device, dtype=dtype)
            self.bufs[name] = buf
        return buf[t * self.P:(t + 1) * self.P]

    def rows(self, name: str, t0: int, t1: int) -> torch.Tensor:
        return self.bufs[name][t0 * self.P:t1 * self.P]


class _Run:
    """Everything one RAFT forward's fused steps share."""

    def __init__(self, block, inp: torch.Tensor, iters: int, pyramid=None, keep: bool = True,
                 dt16=torch.bfloat16):
        B, _, H, W = inp.shape
        self.dt16 = dt16  # 16-bit operand dtype: bf16, or fp16 (fp16 AMP, v_mfma_f32_32x32x16_f16)
        self.dims = (B, H, W)
        self.P = P = B * H * W
        self.iters = iters
        self.block = block
        self.pyr = pyramid  # ops.corr._PyramidState or None (local correlation supplies corr)
        self.arena = _Arena(iters, P, inp.device, keep, dt16)
        self.done = set()  # steps whose backward stored their dY
        self.g_all: Optional[torch.Tensor] = None  # [iters, P, 3*HID] data-gradient rows (backward)
        self.tail: Optional[torch.cuda.Stream] = None  # stream of the motion-encoder backward
        self.wgrads: Optional[List[torch.Tensor]] = None  # weight gradients of iterations [wg_lo, iters)
        self.grad_out: Optional[List[torch.Tensor]] = None  # preallocated (main-stream) parameter gradients
        self.wg_lo = iters
        self.coords: Dict[int, torch.Tensor] = {}
        self.flows: Dict[int, torch.Tensor] = {}
        self.wf: Dict[str, torch.Tensor] = {}
        self.wd: Dict[str, Optional[torch.Tensor]] = {}
        self.bias: Dict[str, torch.Tensor] = {}
        self.cout: Dict[str, int] = {}
        self.n2y: Optional[torch.Tensor] = None  # folded flow-head partials (native step), per run
        self.bwd_bufs: Optional[List[torch.Tensor]] = None  # arena bases handed to fused_step_bwd
        # every layer's operands in one launch
        mods_of = [(name, mods(block)) for name, mods, _, _, _ in _LAYERS]
        packed = C.pack_weights_multi([([m.weight for m in ms], [m.bias for m in ms], segs, scale, dgrad)
                                       for (_, ms), (_, _, segs, scale, dgrad) in zip(mods_of, _LAYERS)],
                                      f16=dt16 == torch.float16)
        for (name, ms), (wf, wd, b) in zip(mods_of, packed):
            self.wf[name], self.wd[name], self.bias[name] = wf, wd, b
            self.cout[name] = sum(m.weight.shape[0] for m in ms)
        # context features: constant over the iterations -> one bf16 pixel-major copy
        self.inp_bf = _pm(inp.detach().to(dt16).contiguous(memory_format=torch.channels_last))

    def release(self):
        """Drop the arena (and the native backward's references to its buffers) once the batched
        weight gradients are queued: the run object itself may live on (autograd contexts,
        reference cycles) until a later collection."""
        self.arena.bufs.clear()
        self.bwd_bufs = None
        self.wd_list = None

    def geom(self, kh, kw, T: int = 1):
        B, H, W = self.dims
        return C.geom(T * B, H, W, kh, kw, kh // 2, kw // 2)

    def fork(self):
        """Side stream for the independent conv branches of a step (it first waits for the
        main stream; every buffer it touches is allocated on the main stream beforehand).
        With ``CONCURRENT = False`` both branches run on the main stream."""
        main = torch.cuda.current_stream()
        if not CONCURRENT:
            return main, main
        side = _side_stream(main.device)
        side.wait_stream(main)
        return main, side

    def geom_d(self, kh, kw):
        B, H, W = self.dims
        return C.geom(B, H, W, kh, kw, kh - 1 - kh // 2, kw - 1 - kw // 2)

    # ------------------------------------------------------------ batched weight gradients
    def alloc_weight_grads(self) -> List[torch.Tensor]:
        """Empty parameter-gradient tensors in ``weight_grads`` order, on the current stream."""
        out: List[torch.Tensor] = []
        for _, mods, _, _, _ in _LAYERS:
            for m in mods(self.block):
                out += [torch.empty_like(m.weight), torch.empty_like(m.bias)]
        return out

    def weight_grads(self, t_lo: int = 0, t_hi: Optional[int] = None,
                     grads: Optional[List[torch.Tensor]] = None,
                     out_bufs: Optional[List[torch.Tensor]] = None,
                     only: Optional[set] = None) -> List[Optional[torch.Tensor]]:
        """Parameter gradients summed over iterations [t_lo, t_hi); ``grads``: the tensors of an
        earlier range to accumulate into (None: fresh ones, or ``out_bufs`` to write);
        ``only``: compute just these layers (the others' entries are passed through)."""
        T, P, ar = self.iters, self.P, self.arena
        t_hi = T if t_hi is None else t_hi
        for t in range(t_lo, t_hi):  # steps whose outputs fed no loss: zero dY
            if t not in self.done and only is None:
                for name in ("dmask", "dd8", "dhd", "dq1", "dq2", "dzr1", "dzr2", "dmo", "dcf", "dc1", "df1"):
                    if name in ar.bufs:
                        ar.rows(name, t, t + 1).zero_()
        inp = self.inp_bf

        def srcs_dy(name, t0, t1):
            r = lambda n: ar.rows(n, t0, t1)  # noqa: E731
            if name == "convc1":
                return [r("corr")], r("dc1")
            if name == "convc2":
                return [r("c1")], r("dcf")[:, :192]
            if name == "convf1":
                return [r("flow8")], r("df1")
            if name == "convf2":
                return [r("f1")], r("dcf")[:, 192:]
            if name == "conv":
                return [r("cf")], r("dmo")
            if name == "zr1":
                return [ar.rows("h", t0, t1), inp, r("motion")], r("dzr1")
            if name == "q1":
                return [r("rh1"), inp, r("motion")], r("dq1")
            if name == "zr2":
                return [r("h1"), inp, r("motion")], r("dzr2")
            if name == "q2":
                return [r("rh2"), inp, r("motion")], r("dq2")
            if name == "heads":
                return [ar.rows("h", t0 + 1, t1 + 1)], r("dhd")
            if name == "fh2":
                return [r("hd")[:, :256]], r("dd8")
            return [r("hd")[:, 256:]], r("dmask")  # mask2

        out: List[Optional[torch.Tensor]] = []
        gi = 0
        for name, mods, segs, scale, _ in _LAYERS:
            ms = mods(self.block)
            dst = grads if grads is not None else out_bufs
            if dst is None:
                wg = [torch.empty_like(m.weight) for m in ms]
                bg = [torch.empty_like(m.bias) for m in ms]
            else:
                wg = [dst[gi + 2 * i] for i in range(len(ms))]
                bg = [dst[gi + 2 * i + 1] for i in range(len(ms))]
            gi += 2 * len(ms)
            if only is not None and name not in only:
                for w, b in zip(wg, bg):
                    out += [w, b]
                continue
            kh, kw = ms[0].weight.shape[2:]
            # one launch over the range, unless an operand would exceed the kernels' 32-bit
            # byte offsets (very large batches / resolutions): then chunks of iterations
            srcs, dy = srcs_dy(name, t_lo, t_hi)
            per_iter = max([s.stride(0) * 2 * P for s in srcs] + [dy.stride(0) * 2 * P])
            chunk = max(1, min(t_hi - t_lo, _I32 // max(per_iter, 1)))
            for t0 in range(t_lo, t_hi, chunk):
                t1 = min(t_hi, t0 + chunk)
                srcs, dy = srcs_dy(name, t0, t1)
                C.conv_wgrad_params(srcs, dy, self.geom(kh, kw, t1 - t0), wg, bg, segs, scale,
                                    accumulate=t0 > t_lo or grads is not None)
            for w, b in zip(wg, bg):
                out += [w, b]
        return out

    def early_weight_grads(self, t: int) -> None:
        """Called once step ``t``'s backward has stored its dY: when [t, t_hi) is a complete
        range of WGRAD_SPLIT, queue its weight gradients on the ``wgrad`` stream, where they
        run beside the backward of the earlier iterations (the data-gradient chain is serial
        and leaves most of the GPU idle)."""
        if WGRAD_SPLIT <= 1 or not self.arena.keep or t == 0:
            return
        T = self.iters
        bounds = [T * k // WGRAD_SPLIT for k in range(1, WGRAD_SPLIT)]
        if t not in bounds:
            return
        t_hi = min([b for b in bounds if b > t], default=T)
        dev = self.inp_bf.device
        ws = aux_stream(dev, "wgrad")
        ws.wait_stream(torch.cuda.current_stream(dev))
        if self.tail is not None:  # the motion-encoder backward wrote its dY there
            ws.wait_stream(self.tail)
        with torch.cuda.stream(ws):
            self.wgrads = self.weight_grads(t, t_hi, self.wgrads)
        self.wg_lo = t


TAIL_STREAM = True  # motion-encoder backward on its own stream (see _Step.backward)
# the batched weight gradients in WGRAD_SPLIT iteration ranges: all but the first start on the
# wgrad stream as soon as their iterations' backward is done (_Run.early_weight_grads)
WGRAD_SPLIT = int(os.environ.get("RAFT_WGRAD_SPLIT", "1"))  # 2: -1.5 % (gpurun_out r3 A/B), kept off
HEAD_STREAM = True  # upsampler / head backward ahead of the d-net chain (see _Step.backward)
# flow_head.conv2 folded into the heads conv's epilogue (per-tap partials) + n2_apply, instead of
# a separate 3x3 256 -> 2 conv that re-reads the 256-channel activation 9 times
FOLD_N2 = os.environ.get("RAFT_FOLD_N2", "1") != "0"
# the step's forward issued by one native op (csrc/bindings.cpp fused_step_fwd) instead of ~17
# Python-side op calls (neutral on the GPU, profiles/r5o_bench_native*.json: the launches, not
# Python, are the host cost); tests set it False to compare with the Python body bitwise
NATIVE_STEP = True
# the step's backward issued by one native op (csrc/bindings.cpp fused_step_bwd) instead of ~11
# conv_fwd calls and ~30 arena views from Python (~0.28 ms of host time per iteration, which is
# step time at batch 1-2 per GPU); tests set it False to compare with the Python body bitwise
NATIVE_BWD = os.environ.get("RAFT_NATIVE_BWD", "1") != "0"
# batched weight gradients on the tail stream beside the encoders' backward (see WeightToken)
EARLY_WGRAD = os.environ.get("RAFT_EARLY_WGRAD", "1") != "0"
# (Measured and dropped: the batched weight gradients split over two streams, neutral,
# profiles/r4_bench_wgrad_mt_ab.log; issued from the last step's backward instead of the weight
# token's, neutral, profiles/r5x_bench*.json -- the tail of the step is throughput-bound.)
# (Measured and dropped: the batched weight gradients on a CU-masked stream -- 128 / 64 / 32 of
# the 256 CUs: 374 / 290 / 210 vs 450 pairs/s, profiles/r6j_*.json.  They share the encoders'
# backward window as throughput work; starving them lengthens the step.)
# diagnostics: a list collects (main-stream event at the token's backward, weight-gradient
# start, end) event triples on the tail stream (scripts/host_lead.py --wgrad_timing)
WGRAD_TIMING: Optional[list] = None


def _head_stream(device) -> torch.cuda.Stream:
    return aux_stream(device, "side")  # idle during the loop's backward (ops/streams.py)


def keep_tail(run) -> bool:
    """Forward tail work needs a caller that joins the tail stream (FusedBasicUpdate.join)."""
    return run.arena.keep


def _tail_stream(device) -> torch.cuda.Stream:
    return aux_stream(device, "tail")
# the step's flow / correlation conv branches on the side and main streams (+0.7 %,
# profiles/r2_concurrent_branches_ab.log; it lost while the process used more streams than
# hardware queues)
CONCURRENT = True


def _side_stream(device) -> torch.cuda.Stream:
    return aux_stream(device, "side")


class WeightToken:
    """The autograd token of the batched weight gradients, created BEFORE the encoders run.

    Autograd executes ready nodes in decreasing creation order, so a token created before the
    encoders has its backward run only after the encoders' backward (and the pyramid's) have
    been issued.  It then computes the weight gradients on the tail stream, starting from the
    event the last refinement step's backward recorded (``_Run.steps_done``): they overlap the
    encoders' backward on the main and side streams instead of running before it (both are
    far from filling the GPU alone).  The current stream waits for them before the gradients
    are handed back, i.e. behind the already-issued encoder backward."""

    def __init__(self, block):
        self.run = None
        self.tensor = _PackWeights.apply(self, *_params(block))


class _PackWeights(torch.autograd.Function):
    """Token node: its backward (after every step's backward) runs the batched weight grads."""

    @staticmethod
    def forward(ctx, holder, *params):
        ctx.holder = holder  # a _Run, or a WeightToken whose run is filled in later
        ctx.set_materialize_grads(False)  # the steps send no token gradient (None): no zero fills
        return params[0].new_empty(())  # ordering token: its value is never read (no fill launch)

    @staticmethod
    def backward(ctx, gtoken):
        h = ctx.holder
        run: _Run = h.run if isinstance(h, WeightToken) else h
        # break the token <-> graph reference cycle (token.tensor.grad_fn holds this ctx, whose
        # holder is the token): without it every step's run (~28 MB of device tensors at config #2)
        # stayed reachable until the next cyclic garbage collection (scripts/mem_growth.py)
        ctx.holder = None
        if isinstance(h, WeightToken):
            h.run = None
        if run is None:  # the token's forward pass never reached the update loop
            return (None,) * (len(ctx.needs_input_grad))
        cur = torch.cuda.current_stream() if run.inp_bf.is_cuda else None
        ev = getattr(run, "steps_done", None)
        if ev is not None and run.wgrads is None and cur is not None:
            ws = _tail_stream(cur.device)
            ws.wait_event(ev)  # the steps' backward on the main stream (the tail stream is ordered)
            with torch.cuda.stream(ws):
                if WGRAD_TIMING is not None:  # scripts/host_lead.py --wgrad_timing
                    evs = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                    evs[0].record(cur)  # main stream: the encoder backward queued before this point
                    evs[1].record(ws)
                grads = run.weight_grads(out_bufs=run.grad_out)
                if WGRAD_TIMING is not None:
                    evs[2].record(ws)
                    WGRAD_TIMING.append(evs)
            cur.wait_stream(ws)
            # no record_stream: the gradients were allocated on this stream before the event the
            # tail stream waited for, and the arena (this stream's memory too) is released only
            # after this stream waited for the tail stream -- every later reuse of those blocks is
            # ordered behind the weight gradients.  (A record_stream'ed block costs an event on
            # the recorded stream when it is freed: ~70 of them, ~0.5 ms of GPU time, used to
            # land on the main stream at every optimizer.zero_grad.)
            run.grad_out = None
            run.release()
            run.tail = None
            return (None, *grads)
        if run.tail is not None:  # the steps' motion-encoder backward wrote dY on the tail stream
            cur.wait_stream(run.tail)
        if run.wgrads is not None:
            # the later iterations' gradients were computed on the wgrad stream during the
            # loop's backward (_Run.early_weight_grads): add the remaining iterations there too
            # (same stream: ordered after them), then join
            ws = aux_stream(cur.device, "wgrad")
            ws.wait_stream(cur)
            with torch.cuda.stream(ws):
                grads = run.weight_grads(0, run.wg_lo, run.wgrads)
            cur.wait_stream(ws)
            for g in grads:
                g.record_stream(cur)
            for b in run.arena.bufs.values():
                b.record_stream(ws)
        else:
            grads = run.weight_grads()
        run.release()
        run.wgrads = None
        return (None, *grads)


class _Step(torch.autograd.Function):
    @staticmethod
    def forward(ctx, wtoken, ptoken, net, inp32, corr_in, coords1, run: _Run, t: int, up: bool = True):
        B, H, W = run.dims
        P = run.P
        dev = net.device
        bf = run.dt16
        k = ops()
        ar = run.arena
        g = run.geom

        # hidden state: slot t of the "h" arena (slot t+1 = this step's output).  Without the
        # arena (inference) the previous step's output rows are used as they are: a fresh slot
        # would cost a copy of the hidden state per iteration (32 copies of 8 MB per 1080p pair)
        net_pm = _pm(net)
        if not ar.keep and net_pm.dtype == run.dt16 and net_pm.is_contiguous():
            h0 = net_pm
        else:
            h0 = ar.take("h", t, HID, slots=run.iters + 1)
            if net_pm.data_ptr() != h0.data_ptr():
                h0.copy_(net_pm)
        if NATIVE_STEP and dev.type == "cuda":
            return _Step._native_forward(ctx, run, t, up, h0, coords1, corr_in, net.dtype)
        # correlation features
        corr = ar.take("corr", t, CORR_PAD)
        flow8 = ar.take("flow8", t, 8)
        motion = ar.take("motion", t, HID)
        if run.pyr is not None:  # the lookup launch also packs the flow operand (flow8, motion[:, 126:])
            k.corr_lookup_into(run.pyr.levels, coords1, run.pyr.radius, corr.view(B, H, W, CORR_PAD), flow8,
                               motion[:, 126:])
        else:
            corr.copy_(corr_in.reshape(P, CORR_PAD))
            k.pack_flow(coords1, flow8, motion[:, 126:], True)

        c1 = ar.take("c1", t, 256)
        cf = ar.take("cf", t, 256)
        f1 = ar.take("f1", t, 128)
        # the flow branch (convf1 -> convf2) runs beside the correlation branch (convc1 -> convc2):
        # neither launch fills the 256 CUs on its own
        main, side = run.fork()
        with torch.cuda.stream(side):
            C.conv_fwd([flow8], run.wf["convf1"], g(7, 7), 128, f1, bias=run.bias["convf1"], act=1)
            C.conv_fwd([f1], run.wf["convf2"], g(3, 3), 64, cf[:, 192:], bias=run.bias["convf2"], act=1)
        C.conv_fwd([corr], run.wf["convc1"], g(1, 1), 256, c1, bias=run.bias["convc1"], act=1)
        C.conv_fwd([c1], run.wf["convc2"], g(3, 3), 192, cf[:, :192], bias=run.bias["convc2"], act=1)
        main.wait_stream(side)
        C.conv_fwd([cf], run.wf["conv"], g(3, 3), 126, motion, bias=run.bias["conv"], act=1)

        inp = run.inp_bf
        h = h0
        for stage, (kh, kw) in ((1, (1, 5)), (2, (5, 1))):
            zr = ar.take(f"zr{stage}", t, 2 * HID)
            rh = ar.take(f"rh{stage}", t, HID)
            C.conv_fwd([h, inp, motion], run.wf[f"zr{stage}"], g(kh, kw), 2 * HID, zr,
                       bias=run.bias[f"zr{stage}"], epi=C.EPI_GRU_ZR, h=h, out2=rh)
            hn = ar.take("h1", t, HID) if stage == 1 else ar.take("h", t + 1, HID, slots=run.iters + 1)
            q = ar.take(f"q{stage}", t, HID)
            C.conv_fwd([rh, inp, motion], run.wf[f"q{stage}"], g(kh, kw), HID, hn,
                       bias=run.bias[f"q{stage}"], epi=C.EPI_GRU_Q, h=h, z=zr[:, :HID], out2=q)
            h = hn

        hd = ar.take("hd", t, 512)
        coords_out = torch.empty_like(coords1)
        flow = torch.empty_like(coords1)
        # flow_head.conv2: folded into the heads conv (its per-tap partials, 4 slots of 64
        # channels) and finished with apply_delta by n2_apply -- or a conv of its own
        n2 = dict(n2w=run.wf["fh2"], n2y=torch.empty(4, 18, P, device=dev, dtype=torch.float32)) if FOLD_N2 else {}

        def flow_head_out():
            if FOLD_N2:
                k.n2_apply(n2["n2y"], run.bias["fh2"], coords1, coords_out, flow)
            else:
                delta = torch.empty(P, 8, device=dev, dtype=torch.float32)
                C.conv_fwd([hd[:, :256]], run.wf["fh2"], g(3, 3), 2, delta, bias=run.bias["fh2"])
                k.apply_delta(coords1, delta, coords_out, flow)

        if not up:
            # inference step whose upsampled flow nobody reads (test_mode keeps only the last):
            # the flow head alone -- the first 256 rows of the fused heads weight -- no mask
            # head, no convex upsampling
            C.conv_fwd([h], run.wf["heads"], g(3, 3), 256, hd, bias=run.bias["heads"], act=1, **n2)
            flow_head_out()
            return _nchw(h, B, H, W), None, coords_out
        mask = ar.take("mask", t, 576)
        # the mask head (its 3x3 half of the fused heads conv, the 1x1) and the convex upsampling
        # feed only the loss, not the next step: they run on the tail stream beside the next
        # step's lookup / motion encoder / GRU (the caller joins the tail stream before the loss
        # reads the flows); the main stream keeps the flow head alone
        tail = _tail_stream(dev) if TAIL_STREAM and dev.type == "cuda" and keep_tail(run) else None
        C.conv_fwd([h], run.wf["heads"], g(3, 3), 256 if tail is not None else 512, hd, bias=run.bias["heads"],
                   act=1, **n2)
        flow_head_out()
        if tail is not None:
            tail.wait_stream(torch.cuda.current_stream(dev))
            run.tail = tail
        with torch.cuda.stream(tail) if tail is not None else contextlib.nullcontext():
            if tail is not None:  # mask.0: rows [256, 512) of the fused heads weight
                C.conv_fwd([h], run.wf["heads"][256:], g(3, 3), 256, hd[:, 256:], bias=run.bias["heads"][256:],
                           act=1)
            C.conv_fwd([hd[:, 256:]], run.wf["mask2"], g(1, 1), 576, mask, bias=run.bias["mask2"])
            flow_up = k.convex_upsample(flow, _nchw(mask, B, H, W))
        if tail is not None:
            flow_up.record_stream(torch.cuda.current_stream(dev))

        ctx.run, ctx.t = run, t
        ctx.net_dtype = net.dtype
        ctx.has_corr_in = corr_in is not None
        run.coords[t] = coords1
        run.flows[t] = flow
        ctx.mark_non_differentiable(coords_out)
        # no zero fills for the gradients that never arrive (coords_out; the last step's net)
        ctx.set_materialize_grads(False)
        return _nchw(h, B, H, W), flow_up, coords_out

    @staticmethod
    def _native_forward(ctx, run, t, up, h0, coords1, corr_in, net_dtype):
        """The forward above as one native op call (csrc/bindings.cpp fused_step_fwd): the same
        launches, streams and arena slots, issued from C++."""
        B, H, W = run.dims
        ar = run.arena
        take = ar.take
        dev = h0.device
        if run.n2y is None:
            run.n2y = torch.empty(4, 18, run.P, device=dev, dtype=torch.float32)
            run.wf_list = [run.wf[name] for name, _, _, _, _ in _LAYERS]
            run.bias_list = [run.bias[name] for name, _, _, _, _ in _LAYERS]
            run.none16 = torch.empty(0, device=dev, dtype=run.dt16)
        h_out = take("h", t + 1, HID, slots=run.iters + 1)
        bufs = [h0, take("corr", t, CORR_PAD), take("flow8", t, 8), take("motion", t, HID), take("c1", t, 256),
                take("cf", t, 256), take("f1", t, 128), take("zr1", t, 2 * HID), take("rh1", t, HID),
                take("q1", t, HID), take("h1", t, HID), take("zr2", t, 2 * HID), take("rh2", t, HID),
                take("q2", t, HID), h_out, take("hd", t, 512), take("mask", t, 576) if up else run.none16, run.n2y,
                coords1, run.inp_bf]
        tail = _tail_stream(dev) if TAIL_STREAM and up and keep_tail(run) else None
        cfg = [B, H, W, run.pyr.radius if run.pyr is not None else 0, int(up),
               _side_stream(dev).cuda_stream if CONCURRENT else 0, tail.cuda_stream if tail is not None else 0,
               int(FOLD_N2), 0]
        res = ops().fused_step_fwd(bufs, run.wf_list, run.bias_list, run.pyr.levels if run.pyr is not None else [],
                                   corr_in if run.pyr is None else None, cfg)
        coords_out, flow = res[0], res[1]
        if not up:
            return _nchw(h_out, B, H, W), None, coords_out
        if tail is not None:
            run.tail = tail
        ctx.run, ctx.t = run, t
        ctx.net_dtype = net_dtype
        ctx.has_corr_in = corr_in is not None
        run.coords[t] = coords1
        run.flows[t] = flow
        ctx.mark_non_differentiable(coords_out)
        ctx.set_materialize_grads(False)
        return _nchw(h_out, B, H, W), res[2], coords_out

    @staticmethod
    def _native_backward(ctx, g_net, g_flow_up):
        """The backward below as one native op call (csrc/bindings.cpp fused_step_bwd): the same
        launches, streams and arena slots, issued from C++."""
        run: _Run = ctx.run
        t = ctx.t
        B, H, W = run.dims
        ar = run.arena
        dev = run.inp_bf.device
        main = torch.cuda.current_stream(dev)
        head = _head_stream(dev) if HEAD_STREAM else None
        if head is not None:
            ready = getattr(g_flow_up, "_raft_ready", None) if g_flow_up is not None else None
            if ready is not None:
                head.wait_event(ready)
            else:
                head.wait_stream(main)
            if g_flow_up is not None:
                g_flow_up.record_stream(head)
        if run.bwd_bufs is None:  # every backward arena buffer at once, then the views' bases
            for name, C in _BWD_ARENA:
                ar.take(name, 0, C)
            run.bwd_bufs = [ar.bufs[n] for n in _BWD_BUFS]
            none16 = torch.empty(0, device=dev, dtype=run.dt16)
            run.wd_list = [run.wd[name] if run.wd[name] is not None else none16 for name, _, _, _, _ in _LAYERS]
            run.g_all = torch.empty(run.iters, run.P, 3 * HID, device=dev, dtype=torch.float32)
        dense = not ctx.has_corr_in and run.pyr is not None and bool(run.pyr.levels)
        if dense and not run.pyr.deferrable():
            run.pyr.grad_buffers()  # allocated (zeroed) on the main stream
        tail = _tail_stream(dev) if dense and TAIL_STREAM else None
        if tail is not None:
            run.tail = run.pyr.tail = tail
        d_net, dcorr = ops().fused_step_bwd(run.bwd_bufs, run.wd_list, run.g_all, run.flows[t], g_net, g_flow_up,
                                            [B, H, W, t, head.cuda_stream if head is not None else 0,
                                             tail.cuda_stream if tail is not None else 0])
        if dense:
            if run.pyr.deferrable():
                run.pyr.pending.append((run.coords[t], dcorr.view(B, H, W, CORR_PAD)))
            else:
                with torch.cuda.stream(tail) if tail is not None else contextlib.nullcontext():
                    run.pyr.add_grad(run.coords[t], dcorr.view(B, H, W, CORR_PAD))
        return d_net, dcorr

    @staticmethod
    def backward(ctx, g_net, g_flow_up, _g_coords):
        run: _Run = ctx.run
        t = ctx.t
        B, H, W = run.dims
        P = run.P
        dev = g_flow_up.device if g_flow_up is not None else run.inp_bf.device
        bf = run.dt16
        k = ops()
        ar = run.arena
        gd = run.geom_d
        if NATIVE_BWD and dev.type == "cuda" and ar.keep:
            d_net, dcorr = _Step._native_backward(ctx, g_net, g_flow_up)
            return _Step._backward_tail(ctx, d_net, dcorr)

        def R(name):  # this step's slot of a forward arena
            return ar.rows(name, t, t + 1)

        def dgrad(name, dy, kh, kw, out, n, mask=None, acc_c0=1 << 30):
            C.conv_fwd([dy], run.wd[name], gd(kh, kw), n, out, epi=C.EPI_GRAD, mask=mask, acc_c0=acc_c0)

        hd, mask = R("hd"), R("mask")
        dmask = ar.take("dmask", t, 576)
        dd8 = ar.take("dd8", t, 8)
        dhd = ar.take("dhd", t, 512)
        # ---- upsampler + head data gradients.  They need only this step's loss gradient and
        # forward activations, not the d net of the later step: on the head stream they start
        # from the loss gradient's ready event while the main stream still runs the later
        # step's GRU backward (without such an event: after everything queued so far)
        main = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
        head = _head_stream(dev) if HEAD_STREAM and main is not None and ar.keep else None
        if head is not None:
            ready = getattr(g_flow_up, "_raft_ready", None) if g_flow_up is not None else None
            if ready is not None:
                head.wait_event(ready)
            else:
                head.wait_stream(main)
            if g_flow_up is not None:
                g_flow_up.record_stream(head)
        with torch.cuda.stream(head) if head is not None else contextlib.nullcontext():
            if g_flow_up is not None:
                k.convex_upsample_backward_into(run.flows[t], _nchw(mask, B, H, W), g_flow_up,
                                                _nchw(dmask, B, H, W), dd8)
            else:
                dmask.zero_()
                dd8.zero_()
            dgrad("fh2", dd8, 3, 3, dhd[:, :256], 256, mask=hd[:, :256])
            dgrad("mask2", dmask, 1, 1, dhd[:, 256:], 256, mask=hd[:, 256:])
        if head is not None:
            main.wait_stream(head)
        # ---- GRU stages (reverse order).  The gate backward runs in the epilogues of the data
        # gradients: the conv producing a stage's dH finishes (dq, dz, carry) of that stage
        # (EPI_GRU_BWD_A), the q conv's data gradient finishes dr and d h (EPI_GRU_BWD_B); the
        # last one writes d net (bf16), d inp and the ReLU'-masked d motion (EPI_GRU_BWD_LAST).
        # G = [d h | d inp | d motion] (fp32) accumulates over the stages.
        stages = ((2, (5, 1)), (1, (1, 5)))
        gates = {}
        for stage, _ in stages:
            gates[stage] = (ar.rows("h", t, t + 1) if stage == 1 else R("h1"), R(f"zr{stage}"), R(f"q{stage}"),
                            ar.take(f"dq{stage}", t, HID), ar.take(f"dzr{stage}", t, 2 * HID))
        carry = torch.empty(P, HID, device=dev, dtype=torch.float32)

        def gate_a(stage):
            h, zr, q, dq, dzr = gates[stage]
            return dict(epi=C.EPI_GRU_BWD_A, h=h, z=zr[:, :HID], g0=q, out2=dq, out3=dzr[:, :HID], carry=carry,
                        gru_cols=HID)

        # heads data gradient = dH of stage 2 (+ the incoming d net); `carry` stands in for the
        # fp32 output, which this epilogue does not write
        C.conv_fwd([dhd], run.wd["heads"], gd(3, 3), HID, carry,
                   addsrc=_pm(g_net).to(bf).contiguous() if g_net is not None else None, **gate_a(2))

        # this step's slot of a per-forward [iters, P, 3*HID] buffer: the d inp columns of every
        # step stay there and are summed once by the last backward (step 0) -- no per-step
        # gradient copy / add kernels for the iteration-shared context features
        if run.g_all is None:
            run.g_all = torch.empty(run.iters, P, 3 * HID, device=dev, dtype=torch.float32)
        G = run.g_all[t]
        motion = R("motion")
        dmo = ar.take("dmo", t, HID)
        d_net = torch.empty(P, HID, device=dev, dtype=bf)
        for i, (stage, (kh, kw)) in enumerate(stages):
            h, zr, q, dq, dzr = gates[stage]
            # d(r h) -> dr and d h = carry + d(rh) r; the other channels fresh on the first stage,
            # accumulated afterwards
            C.conv_fwd([dq], run.wd[f"q{stage}"], gd(kh, kw), 3 * HID, G, epi=C.EPI_GRU_BWD_B,
                       acc_c0=(3 * HID if i == 0 else HID), h=h, g0=zr[:, HID:], carry=carry, out3=dzr[:, HID:],
                       gru_cols=HID)
            if i + 1 < len(stages):  # -> dH of the next (earlier) stage
                C.conv_fwd([dzr], run.wd[f"zr{stage}"], gd(kh, kw), 3 * HID, G, acc_c0=0,
                           **gate_a(stages[i + 1][0]))
            else:  # d net (bf16), d inp, d motion masked by the ReLU' (flow channels -> 0)
                C.conv_fwd([dzr], run.wd[f"zr{stage}"], gd(kh, kw), 3 * HID, G, epi=C.EPI_GRU_BWD_LAST, acc_c0=0,
                           out3=d_net, gru_cols=HID, cout=dmo, cmask=motion, cm_c0=2 * HID, cm_valid=126)

        # ---- motion encoder.  With the dense pyramid its backward is a side branch: it feeds only
        # the pyramid gradient and the batched weight gradients, not the d net the next (earlier)
        # step waits for.  It runs on the tail stream, beside that step's head / GRU backward;
        # the pyramid and weight-gradient backward join the tail stream before they read.
        cf, c1, f1 = R("cf"), R("c1"), R("f1")
        dcf = ar.take("dcf", t, 256)
        dc1 = ar.take("dc1", t, 256)
        df1 = ar.take("df1", t, 128)
        dcorr = torch.empty(P, CORR_PAD, device=dev, dtype=bf)
        dense = not ctx.has_corr_in and run.pyr is not None and bool(run.pyr.levels)
        if dense and not run.pyr.deferrable():
            run.pyr.grad_buffers()  # allocated (zeroed) on the main stream
        tail = _tail_stream(dev) if dense and TAIL_STREAM and dev.type == "cuda" else None
        if tail is not None:
            tail.wait_stream(torch.cuda.current_stream(dev))
            dcorr.record_stream(tail)
            run.tail = run.pyr.tail = tail
        with torch.cuda.stream(tail) if tail is not None else contextlib.nullcontext():
            dgrad("conv", dmo, 3, 3, dcf, 256, mask=cf)
            dgrad("convf2", dcf[:, 192:], 3, 3, df1, 128, mask=f1)
            dgrad("convc2", dcf[:, :192], 3, 3, dc1, 256, mask=c1)
            dgrad("convc1", dc1, 1, 1, dcorr, CORR_PAD)
            if dense:
                run.pyr.add_grad(run.coords[t], dcorr.reshape(B, H, W, CORR_PAD))
        return _Step._backward_tail(ctx, d_net, dcorr)

    @staticmethod
    def _backward_tail(ctx, d_net, dcorr):
        run: _Run = ctx.run
        t = ctx.t
        B, H, W = run.dims
        dev = d_net.device
        ar = run.arena
        run.done.add(t)
        run.early_weight_grads(t)

        d_corr_in = dcorr.reshape(B, H, W, CORR_PAD) if ctx.has_corr_in else None
        d_net = _nchw(d_net if ctx.net_dtype == run.dt16 else d_net.to(ctx.net_dtype), B, H, W)
        d_inp = None
        if t == 0:  # the last step backward to run (every other step's d net feeds it)
            if EARLY_WGRAD and dev.type == "cuda" and ar.keep:
                # the parameter gradients the tail stream will write: main-stream memory, taken
                # before the event the tail stream waits for (see _PackWeights.backward)
                run.grad_out = run.alloc_weight_grads()
                run.steps_done = torch.cuda.Event()
                run.steps_done.record(torch.cuda.current_stream(dev))
            done = sorted(run.done)
            gi = run.g_all[:, :, HID:2 * HID] if len(done) == run.iters else run.g_all[done][:, :, HID:2 * HID]
            d_inp = _nchw(gi.sum(0), B, H, W)
            run.g_all = None
        # the tokens only order the autograd graph (their nodes run after every step's backward
        # whatever they receive): no gradient, no fill / accumulate kernels
        return None, None, d_net, d_inp, d_corr_in, None, None, None, None


class FusedBasicUpdate:
    """Per-forward driver: packs the weights once, then runs fused refinement steps."""

    def __init__(self, block, inp: torch.Tensor, iters: int, pyramid=None, token: Optional[WeightToken] = None,
                 dt16=torch.bfloat16):
        keep = torch.is_grad_enabled()
        self.run = _Run(block, inp, iters, pyramid=pyramid, keep=keep, dt16=dt16)
        if token is not None and keep:
            token.run = self.run  # created before the encoders (see WeightToken)
            self.token = token.tensor
        else:
            self.token = _PackWeights.apply(self.run, *_params(block))
        # the fp32 ``inp`` keeps autograd's cross-iteration gradient sum in fp32
        self.inp32 = inp.float().contiguous(memory_format=torch.channels_last)

    def join(self):
        """Make the current stream wait for the steps' tail-stream work (their upsampled flows)."""
        if self.run.tail is not None:
            torch.cuda.current_stream().wait_stream(self.run.tail)

    def step(self, t: int, net, coords1, ptoken=None, corr=None,
             upsample: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor], torch.Tensor]:
        """One refinement iteration -> (net, flow_up (B, 2, 8H, 8W) fp32, coords1 after the
        update (no grad)).  ``ptoken``: the correlation pyramid's autograd token (dense path);
        ``corr``: (B, H, W, 328) bf16 features (local-correlation path).  ``upsample=False``
        (honoured without autograd only): flow_up is None and the mask head is skipped."""
        if ptoken is None:
            ptoken = self.token.new_zeros(())
        up = upsample or torch.is_grad_enabled()  # skipping needs a forward nobody backpropagates
        return _Step.apply(self.token, ptoken, net, self.inp32, corr, coords1.detach().float().contiguous(),
                           self.run, t, up)


def supported(block) -> bool:
    from ..models.update import BasicUpdateBlock

    return isinstance(block, BasicUpdateBlock)


# ------------------------------------------------------------------ fp32-faithful inference
# Without AMP (the reference's default for demo.py / evaluate.py / the ROS node) the
# refinement step runs on the same HIP kernels in split-bf16 mode: every activation is
# stored as hi / lo / hi bf16 planes and every conv packs [W_hi | W_hi | W_lo], so each
# bf16 MFMA GEMM computes x_hi W_hi + x_lo W_hi + x_hi W_lo with fp32 accumulation -- the
# fp32 product up to the dropped x_lo W_lo term (~2^-16 relative); gates, GRU blend and
# coordinates stay fp32 (csrc/kernel_abi.h ConvFwdArgs::split_g).  Inference only.

# name -> input segments per SOURCE operand (each a split [hi | lo | hi] tensor)
_SPLIT_SOURCES = {
    "convc1": [[(324, CORR_PAD)]],
    "convc2": [[(256, 256)]],
    "convf1": [[(2, 8)]],
    "convf2": [[(128, 128)]],
    "conv": [[(256, 256)]],
    "zr1": [[(128, 128)]] * 3,
    "q1": [[(128, 128)]] * 3,
    "zr2": [[(128, 128)]] * 3,
    "q2": [[(128, 128)]] * 3,
    "heads": [[(128, 128)]],
    "fh2": [[(256, 256)]],
    "mask2": [[(256, 256)]],
}


class SplitBasicUpdate:
    """Per-forward driver of the fp32-faithful (split-bf16) fused refinement step."""

    def __init__(self, block, inp: torch.Tensor, iters: int, pyramid=None):
        B, _, H, W = inp.shape
        self.dims = (B, H, W)
        self.P = P = B * H * W
        self.pyr = pyramid
        dev = inp.device
        self.wf, self.bias = {}, {}
        packed = C.pack_weights_multi(
            [([m.weight for m in mods(block)], [m.bias for m in mods(block)],
              [s for src in _SPLIT_SOURCES[name] for s in src], scale, 0) for name, mods, _, scale, _ in _LAYERS],
            split=True)
        for (name, _, _, _, _), (wf, _, b) in zip(_LAYERS, packed):
            self.wf[name], self.bias[name] = wf, b
        bf = torch.bfloat16
        e = lambda n: torch.empty(P, n, device=dev, dtype=bf)  # noqa: E731
        self.inp = C.split_pack(_pm(inp.float()), e(384), HID)
        self.h = [e(384), e(384), e(384)]  # h (in), h1, h (out) ping-pong
        self.corr, self.flow8, self.motion = e(3 * CORR_PAD), e(24), e(384)
        self.c1, self.cf, self.f1 = e(768), e(768), e(384)
        self.zr, self.rh, self.hd = e(768), e(384), e(1536)
        self.delta = torch.empty(P, 8, device=dev, dtype=torch.float32)
        self.mask = torch.empty(P, 576, device=dev, dtype=torch.float32)

    def geom(self, kh, kw):
        B, H, W = self.dims
        return C.geom(B, H, W, kh, kw, kh // 2, kw // 2)

    def step(self, t: int, net, coords1, coords0, corr=None, upsample: bool = True):
        """-> (net (B, 128, H, W) fp32 channels-last, flow_up or None, coords1 after the update).
        ``corr``: (P, >=324) fp32 lookup rows (local correlation); else the dense pyramid."""
        B, H, W = self.dims
        P, g, k = self.P, self.geom, ops()
        h0 = self.h[0]
        if t == 0 or net is not None:
            C.split_pack(_pm(net.float()), h0, HID)
        if corr is None:
            st = self.pyr
            corr = k.corr_lookup(st.levels, coords1.contiguous(), st.radius, torch.float32, CORR_PAD).view(P, CORR_PAD)
        C.split_pack(corr, self.corr, CORR_PAD, 0, CORR_PAD)
        flow = (coords1 - coords0).permute(0, 2, 3, 1).reshape(P, 2).contiguous()
        C.split_pack(flow, self.flow8, 8, 0, 8)
        C.split_pack(flow, self.motion, HID, 126, 2)
        S1 = lambda G: [G, 0, 0, 0]  # noqa: E731
        C.conv_fwd([self.flow8], self.wf["convf1"], g(7, 7), 128, self.f1, bias=self.bias["convf1"], act=1,
                   split=S1(128))
        C.conv_fwd([self.f1], self.wf["convf2"], g(3, 3), 64, self.cf[:, 192:], bias=self.bias["convf2"], act=1,
                   split=S1(256))
        C.conv_fwd([self.corr], self.wf["convc1"], g(1, 1), 256, self.c1, bias=self.bias["convc1"], act=1,
                   split=S1(256))
        C.conv_fwd([self.c1], self.wf["convc2"], g(3, 3), 192, self.cf, bias=self.bias["convc2"], act=1,
                   split=S1(256))
        C.conv_fwd([self.cf], self.wf["conv"], g(3, 3), 126, self.motion, bias=self.bias["conv"], act=1,
                   split=S1(128))
        h = h0
        for stage, (kh, kw) in ((1, (1, 5)), (2, (5, 1))):
            C.conv_fwd([h, self.inp, self.motion], self.wf[f"zr{stage}"], g(kh, kw), 2 * HID, self.zr,
                       bias=self.bias[f"zr{stage}"], epi=C.EPI_GRU_ZR, h=h, out2=self.rh, split=[HID, HID, HID, 0])
            hn = self.h[1] if stage == 1 else self.h[2]
            C.conv_fwd([self.rh, self.inp, self.motion], self.wf[f"q{stage}"], g(kh, kw), HID, hn,
                       bias=self.bias[f"q{stage}"], epi=C.EPI_GRU_Q, h=h, z=self.zr, split=[HID, 0, HID, HID])
            h = hn
        self.h[0], self.h[2] = self.h[2], self.h[0]  # the next step's input
        nh = 512 if upsample else 256
        C.conv_fwd([h], self.wf["heads"][:nh], g(3, 3), nh, self.hd, bias=self.bias["heads"][:nh], act=1,
                   split=S1(256))
        C.conv_fwd([self.hd[:, :768]], self.wf["fh2"], g(3, 3), 2, self.delta, bias=self.bias["fh2"])
        coords_out = torch.empty_like(coords1)
        flow_lo = torch.empty_like(coords1)
        k.apply_delta(coords1, self.delta, coords_out, flow_lo)
        flow_up = None
        if upsample:
            C.conv_fwd([self.hd[:, 768:]], self.wf["mask2"], g(1, 1), 576, self.mask, bias=self.bias["mask2"])
            flow_up = k.convex_upsample(flow_lo, _nchw(self.mask, B, H, W))
        return None, flow_up, coords_out

    def net(self) -> torch.Tensor:
        """The current hidden state as fp32 (B, 128, H, W) (hi + lo planes)."""
        B, H, W = self.dims
        h = self.h[0]
        return _nchw((h[:, :HID].float() + h[:, HID:2 * HID].float()), B, H, W)
