"""Native (HIP) execution of the residual CNN encoders, one autograd node per encoder.

The encoder modules (``models/extractor.py``, reference core/extractor.py:6-267) keep
their parameters and names; on the GPU bf16 path ``encode(module, img1, img2)`` runs
the whole network on the kernels of ``csrc/encoder.hip``:

* activations are NHWC bf16 ``[B, H, W, C]`` end to end; the stem reads the raw 0..255
  fp32 images and normalises them on the fly (``2 * img / 255 - 1``, channels padded
  3 -> 8), both frames of the feature encoder as one batch;
* every conv epilogue emits per-tile (sum, M2) statistics, so InstanceNorm / BatchNorm
  need no statistics pass: a tiny finalize (Chan combine, fixed order; BatchNorm running
  statistics updated in place) and one apply pass that also fuses the ReLU and, at the
  end of a residual block, the downsample norm, the residual add and the final ReLU;
* backward: stride-parity-split data gradients (the first conv of a block and its
  downsample share one launch; the epilogue adds the identity-residual gradient and
  applies the ReLU' of the block input), three-pass norm backward (both tail branches
  at once), split-pixel weight gradients reduced into the fp32 parameter layout.

Nothing here goes through MIOpen, so the encoder is also safe inside a captured HIP
graph (``runtime/train_graph.py``): MIOpen convolutions produced non-finite gradients
from the second replay of a captured training step.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from ..parallel import sync_bn
from ._ext import ops, use_native
from .norm import InstanceNorm2dNHWC

# norm kinds shared with csrc/encoder.hip
_NONE, _INSTANCE, _BATCH_TRAIN, _BATCH_EVAL = 0, 1, 2, 3

# pack every conv's weight operand (forward, and the data-gradient operands of the backward) with
# two launches at the start of the encoder forward instead of one packing launch in front of each
# conv (RAFT_ENC_PREPACK=0: per-conv packing; the two launches on an auxiliary stream measured
# -1.6 % and were removed, profiles/r4_enc_prepack_ab.log)
PREPACK = os.environ.get("RAFT_ENC_PREPACK", "1") != "0"
# fp32 training: three-plane (fp32-exact) encoder forward; RAFT_ENC_SPLIT3=0 keeps the round-4
# two-plane forward (A/B, tests)
SPLIT3 = os.environ.get("RAFT_ENC_SPLIT3", "1") != "0"


def _norm_kind(m: nn.Module):
    if isinstance(m, InstanceNorm2dNHWC):
        return _INSTANCE
    if isinstance(m, nn.BatchNorm2d):
        return _BATCH_TRAIN if m.training else _BATCH_EVAL
    if isinstance(m, nn.Sequential) and len(m) == 0:
        return _NONE
    return None


def _unit_convs(block):
    """(conv, norm) chain of a residual / bottleneck block, plus its downsample pair."""
    if hasattr(block, "conv3"):  # BottleneckBlock
        units = [(block.conv1, block.norm1), (block.conv2, block.norm2), (block.conv3, block.norm3)]
        down = (block.downsample[0], block.norm4) if block.downsample is not None else None
    else:  # ResidualBlock
        units = [(block.conv1, block.norm1), (block.conv2, block.norm2)]
        down = (block.downsample[0], block.norm3) if block.downsample is not None else None
    return units, down


def supported(enc: nn.Module, image: torch.Tensor) -> bool:
    """True when ``enc`` can run on the native encoder kernels for this input."""
    if not image.is_cuda or not use_native(image):
        return False
    if enc.training and enc.dropout is not None:
        return False
    norms = [enc.norm1]
    for layer in (enc.layer1, enc.layer2, enc.layer3):
        for blk in layer:
            units, down = _unit_convs(blk)
            norms += [n for _, n in units] + ([down[1]] if down else [])
    return all(_norm_kind(n) is not None for n in norms)


class _Layout:
    """Flat parameter order of one encoder (the autograd inputs) and its norm kinds."""

    def __init__(self, enc):
        self.params = []
        self.index = {}

        def add(t):
            if t is None:
                return -1
            self.index[id(t)] = len(self.params)
            self.params.append(t)
            return self.index[id(t)]

        def conv(c):
            return {"w": add(c.weight), "b": add(c.bias), "stride": c.stride[0], "pad": c.padding[0],
                    "module": c}

        def norm(n):
            k = _norm_kind(n)
            d = {"kind": k, "module": n}
            if k in (_BATCH_TRAIN, _BATCH_EVAL):
                d["g"], d["bt"] = add(n.weight), add(n.bias)
            return d

        self.stem = (conv(enc.conv1), norm(enc.norm1))
        self.blocks = []
        for layer in (enc.layer1, enc.layer2, enc.layer3):
            for blk in layer:
                units, down = _unit_convs(blk)
                self.blocks.append(([(conv(c), norm(n)) for c, n in units],
                                    (conv(down[0]), norm(down[1])) if down else None))
        self.out = conv(enc.conv2)


def _stats(a, st, nd, P, split: bool = False):
    """coef [B, 4, N] of the norm ``nd`` for the conv output ``a``."""
    m = nd["module"]
    B, H, W, N = a.shape
    N = N // 3 if split else N
    k = nd["kind"]
    if k in (_BATCH_TRAIN, _BATCH_EVAL):
        Bs = B
        if k == _BATCH_TRAIN and sync_bn.is_synced(m):  # --sync_bn: every rank's images (parallel/sync_bn.py)
            st, Bs = sync_bn.native_norm_stats(st, m.process_group)
        coef = ops().enc_norm_stats(st if k == _BATCH_TRAIN else None, Bs, H * W, N, k, P[nd["g"]], P[nd["bt"]],
                                    m.running_mean, m.running_var,
                                    m.num_batches_tracked if k == _BATCH_TRAIN else None,
                                    m.momentum if m.momentum is not None else 0.1, m.eps, W)
        return coef[:B] if Bs != B else coef
    eps = getattr(m, "eps", 1e-5)
    return ops().enc_norm_stats(st, B, H * W, N, k, None, None, None, None, None, 0.0, eps, W)


def _conv(x, cd, P, stats, split: bool = False, pk=None):
    b = P[cd["b"]] if cd["b"] >= 0 else None
    # split: the fp32 weight is split into [W_hi | W_hi | W_lo] by the packing kernel, every step
    # (no cached copy: an optimizer step -- fused AdamW does not bump the parameter versions --
    # must never leave a stale split weight behind); ``pk``: the operands packed ahead (_Prepack)
    packed = pk.fwd.get(id(cd)) if pk is not None else None
    return ops().enc_conv_fwd(x, P[cd["w"]], b, cd["stride"], cd["pad"], stats, split, packed)


def _conv_hw(h, w, cd):
    m = cd["module"]
    s, p = cd["stride"], cd["pad"]
    return (h + 2 * p - m.kernel_size[0]) // s + 1, (w + 2 * p - m.kernel_size[1]) // s + 1


class _Prepack:
    """Weight operands of one encoder packed ahead, in one persistent buffer per input shape.

    ``issue()`` packs every conv's forward operand with ONE launch (csrc/encoder.hip
    enc_pack_multi_kernel) at the start of the forward, and every data-gradient operand of
    the backward with a second one (the weights do not change before the optimizer step),
    instead of one small packing launch in front of each of the ~58 convs of the two encoders
    (config #2: 761 -> ~705 kernels per step).  The stem conv still packs its own weights.
    The job plans (the kernel arguments of every job, uploaded once) hold the parameters' data
    pointers and are rebuilt when those change.

    The launches run on the consumer stream.  The buffer is
    allocated on the consuming stream and kept, so no allocator event is recorded per step;
    each step's packing follows the consumer's queued work, which includes every earlier read
    of the buffer."""

    _MAX_SHAPES = 4

    def __init__(self, L, P, H, W, split, f16, need_bwd, device):
        mul = 3 if split else 1
        self.fwd_jobs, self.bwd_jobs = [], []  # (cd, Cx) / (cds, H, W)
        h, w = _conv_hw(H, W, L.stem[0])
        for units, down in L.blocks:
            for ui, (cd, _nd) in enumerate(units):
                self.fwd_jobs.append((cd, mul * P[cd["w"]].shape[1]))
                cds = [cd] + ([down[0]] if ui == 0 and down is not None else [])
                self.bwd_jobs.append((cds, h, w))
                if ui == 0 and down is not None:
                    self.fwd_jobs.append((down[0], mul * P[down[0]["w"]].shape[1]))
                h, w = _conv_hw(h, w, cd)
        self.fwd_jobs.append((L.out, mul * P[L.out["w"]].shape[1]))
        self.bwd_jobs.append(([L.out], h, w))
        if not need_bwd:
            self.bwd_jobs = []
        self.split, self.f16, self.need_bwd = split, f16, need_bwd
        self.device = device
        self.buf = None
        self.ptrs = None

    def _build(self, P):
        """Job plans and the packed buffer (first use, and whenever a parameter moved)."""
        o = ops()
        fj = [o.enc_pack_fwd_job(P[cd["w"]], cx, cd["pad"], self.split, self.f16) for cd, cx in self.fwd_jobs]
        bj = [o.enc_pack_dgrad_job([P[c["w"]] for c in cds], [c["stride"] for c in cds], [c["pad"] for c in cds],
                                   h, w, self.split, self.f16) for cds, h, w in self.bwd_jobs]
        offs, total = [], 0
        for _, n, _ in fj + bj:
            offs.append(total)
            total += -(-n // 256) * 256
        if self.buf is None or self.buf.numel() != total:
            self.buf = torch.empty(total, device=self.device, dtype=torch.float16 if self.f16 else torch.bfloat16)

        def plan(jobs, ofs):
            blk = [0]
            for _, _, nb in jobs:
                blk.append(blk[-1] + nb)
            raw = torch.cat([t for t, _, _ in jobs] + [torch.tensor(ofs, dtype=torch.int64).view(torch.uint8),
                                                        torch.tensor(blk, dtype=torch.int32).view(torch.uint8)])
            return raw.to(self.device), len(jobs), blk[-1]

        self.fwd_plan = plan(fj, offs[:len(fj)])
        self.fwd = {id(cd): self.buf[a:a + n] for (cd, _), a, (_, n, _) in zip(self.fwd_jobs, offs, fj)}
        self.bwd = {}
        if bj:
            self.bwd_plan = plan(bj, offs[len(fj):])
            self.bwd = {id(cds[0]): self.buf[a:a + n] for (cds, _, _), a, (_, n, _) in
                        zip(self.bwd_jobs, offs[len(fj):], bj)}

    def issue(self, P):
        o = ops()
        ptrs = tuple(p.data_ptr() for p in P)
        if ptrs != self.ptrs:
            self._build(P)
            self.ptrs = ptrs
        # on the consumer stream: ordered by the stream itself
        o.enc_pack_multi(self.fwd_plan[0], self.fwd_plan[1], self.fwd_plan[2], self.buf)
        if self.bwd_jobs:
            o.enc_pack_multi(self.bwd_plan[0], self.bwd_plan[1], self.bwd_plan[2], self.buf)
        return self


def _prepack(L, x0, split: bool, f16: bool, stream_name: str):
    """Issue the ahead-of-time packing of ``L``'s weight operands (None: disabled / too many
    input shapes seen).  Inside a HIP-graph capture only an already-built plan is used (a
    rebuild uploads the job table, a host copy that cannot be captured; the warm-up forward
    before the capture builds it).  (Per-conv packing inside the graph was ~32 serial 6 us
    launches per 1080p pair.)"""
    capturing = torch.cuda.is_current_stream_capturing() if x0.device.type == "cuda" else False
    if not PREPACK or x0.device.type != "cuda":
        return None

    need_bwd = torch.is_grad_enabled()
    key = (x0.shape[1], x0.shape[2], split, f16, need_bwd)
    cache = L.__dict__.setdefault("prepacks", {})
    pk = cache.get(key)
    if pk is None:
        if capturing or len(cache) >= _Prepack._MAX_SHAPES:
            return None
        pk = cache[key] = _Prepack(L, L.params, x0.shape[1], x0.shape[2], split, f16, need_bwd, x0.device)
    if capturing and tuple(p.data_ptr() for p in L.params) != pk.ptrs:
        return None
    return pk.issue(L.params)


def _forward(L, x0, P, split: bool = False, pk=None):
    """Run the encoder; returns (output NHWC, saved records).  ``split``: every activation as
    split-bf16 planes (fp32-faithful, see below).  ``pk``: weight operands packed ahead."""
    o = ops()
    sc, sn = L.stem
    a0, st = _conv(x0, sc, P, True, split)
    c0 = _stats(a0, st, sn, P, split)
    h = o.enc_apply(a0, c0, True, None, None, False, split)
    stem_rec = (x0, a0, c0, h)
    recs = []
    for units, down in L.blocks:
        hin = h
        ins, acts, coefs = [], [], []
        cur = hin
        for ui, (cd, nd) in enumerate(units):
            a, st = _conv(cur, cd, P, nd["kind"] != _BATCH_EVAL, split, pk)
            c = _stats(a, st, nd, P, split)
            ins.append(cur)
            acts.append(a)
            coefs.append(c)
            if ui + 1 < len(units):
                cur = o.enc_apply(a, c, True, None, None, False, split)
        drec = None
        if down is not None:
            dcd, dnd = down
            ad, st = _conv(hin, dcd, P, dnd["kind"] != _BATCH_EVAL, split, pk)
            cdn = _stats(ad, st, dnd, P, split)
            h = o.enc_apply(acts[-1], coefs[-1], True, ad, cdn, True, split)
            drec = (ad, cdn)
        else:
            h = o.enc_apply(acts[-1], coefs[-1], True, hin, None, True, split)
        recs.append((ins, acts, coefs, drec, h))
    y, _ = _conv(h, L.out, P, False, split, pk)
    return y, stem_rec, recs


# ------------------------------------------------------------------ fp32-faithful (split) mode
# Without AMP (the reference's default for training, demo.py, evaluate.py and the ROS node) the
# encoders run on the same kernels in split-bf16 mode: activations -- and in training every
# data gradient -- are stored as [hi | lo | hi] bf16 planes and each conv packs [W_hi | W_hi |
# W_lo] (split while packing, csrc/encoder.hip enc_pack_kernel; the data-gradient convs split
# along Cout against split dY planes), so a bf16 MFMA GEMM computes x_hi W_hi + x_lo W_hi +
# x_hi W_lo with fp32 accumulation; norm statistics come from the fp32 accumulators, the norm
# apply / backward passes read and write the planes in fp32, and each weight gradient is two
# GEMMs ([X_hi | X_lo]^T dY_hi + X_hi^T dY_lo) folded into the fp32 parameter layout.
#
# Training (mode 2, round 5): the planes are [hi | mid | lo] -- the fp32 value exactly -- and
# the forward convs run six K planes (x hi, mid, hi, lo, hi, mid against W H, H, M, H, L, M:
# every product down to ~2^-24 of x W), so the forward is the fp32 conv; the backward keeps the
# two-plane GEMMs (its operands' first two planes are the same in both layouts; the data-
# gradient decode tables read hi where mode 1 read the duplicate hi plane).  CPU emulation on
# the reference's gradients (scripts/emulate_split_precision.py): rounding the encoder's
# FORWARD operands / outputs to 16 bits costs RMS 4.0e-3 (base) / 8.3e-3 (small) over all
# parameters, the gradient operands 4-5e-6, the update block's forward 7e-4 / 1.4e-4 -- MIOpen's
# own fp32 deviation is 1.8e-3.  The six-plane forward doubles the encoders' forward MFMA work.

def _forward_split(L, x0, P, pk=None, mode: int = 1):
    """``_forward`` on split-bf16 planes without records (inference); the split output rows."""
    return _forward(L, x0, P, mode, pk)[0]


def _split_rows(g: torch.Tensor, mode: int = 1) -> torch.Tensor:
    """fp32 [..., C] -> bf16 [..., 3C] split planes: [hi | lo | hi] (mode 1) or [hi | mid | lo]
    (mode 2, the three-plane layout: see ``encode``)."""
    g = g.float()
    hi = g.to(torch.bfloat16)
    r = g - hi.float()
    lo = r.to(torch.bfloat16)
    third = (r - lo.float()).to(torch.bfloat16) if mode == 2 else hi
    return torch.cat([hi, lo, third], dim=-1).contiguous()


def _unsplit(y: torch.Tensor, mode: int) -> torch.Tensor:
    """Split rows [..., 3N] -> the fp32 value [..., N] (hi + lo, + the third plane in mode 2)."""
    N = y.shape[-1] // 3
    out = y[..., :N].float() + y[..., N:2 * N].float()
    return out + y[..., 2 * N:].float() if mode == 2 else out


def _wgrad(x, dy, cd, P, grads, nd=None, split: bool = False):
    """Weight / bias gradient of conv ``cd``; ``nd``: the norm it feeds.  InstanceNorm and
    training-mode BatchNorm subtract the per-channel mean, so a conv bias in front of them
    has an exactly zero gradient (written as 0, not as bf16 rounding noise).  ``split``: x and
    dy are split rows; two GEMMs [X_hi | X_lo]^T dY_hi and X_hi^T dY_lo, planes folded."""
    w = P[cd["w"]]
    zero = nd is not None and nd["kind"] in (_INSTANCE, _BATCH_TRAIN)
    has_b = cd["b"] >= 0
    if split:
        # [X_hi | X_lo]^T dY_hi (hi / lo columns folded in the reduction), then += X_hi^T dY_lo
        N = w.shape[0]
        cx = x.shape[3] // 3
        dw = torch.empty_like(w, dtype=torch.float32)
        db = torch.empty(N, device=w.device, dtype=torch.float32) if has_b else None
        ops().enc_conv_wgrad(x[..., :2 * cx], dy[..., :N], dw, db, cd["stride"], cd["pad"], False, zero, cx)
        ops().enc_conv_wgrad(x[..., :cx], dy[..., N:2 * N], dw, db, cd["stride"], cd["pad"], True, zero)
    else:
        dw = torch.empty_like(w, dtype=torch.float32)
        db = torch.empty(w.shape[0], device=w.device, dtype=torch.float32) if has_b else None
        ops().enc_conv_wgrad(x, dy, dw, db, cd["stride"], cd["pad"], False, zero)
    grads[cd["w"]] = dw.to(w.dtype) if w.dtype != torch.float32 else dw
    if db is not None:
        b = P[cd["b"]]
        grads[cd["b"]] = db.to(b.dtype) if b.dtype != torch.float32 else db


def _norm_grads(nd, dg, dbt, grads):
    if nd["kind"] in (_BATCH_TRAIN, _BATCH_EVAL) and dg is not None:
        grads[nd["g"]] = dg
        grads[nd["bt"]] = dbt


def _norm_bwd(o, nd, g, a0, c0, relu0, a1, c1, split: bool = False):
    """Norm backward of one conv tail (optionally both tail branches of a block)."""
    m = nd["module"]
    if nd["kind"] == _BATCH_TRAIN and sync_bn.is_synced(m):
        return sync_bn.native_norm_bwd(o, g, a0, c0, relu0, a1, c1, nd["kind"], m.process_group, split)
    return o.enc_norm_bwd(g, a0, c0, relu0, a1, c1, nd["kind"], split)


def _backward(L, P, gy, stem_rec, recs, split: bool = False, pk=None):
    o = ops()
    sp = split
    grads = [None] * len(P)
    bp = pk.bwd if pk is not None else {}  # ordered before the backward by _forward
    last_h = recs[-1][4] if recs else stem_rec[3]
    _wgrad(last_h, gy, L.out, P, grads, split=sp)
    oc = L.out
    g = o.enc_conv_dgrad([gy], [P[oc["w"]]], [oc["stride"]], [oc["pad"]], last_h.shape[1], last_h.shape[2],
                         None, last_h, sp, bp.get(id(oc)))
    for (units, down), (ins, acts, coefs, drec, _h) in zip(reversed(L.blocks), reversed(recs)):
        dnd = down[1] if down is not None else None
        r = _norm_bwd(o, units[-1][1], g, acts[-1], coefs[-1], True, drec[0] if drec else None,
                      drec[1] if drec else None, sp)
        # both tail norms of a block share a kind (one norm_fn per encoder)
        da, dad = r[0], r[1] if drec else None
        _norm_grads(units[-1][1], r[2], r[3], grads)
        if down is not None:
            _norm_grads(dnd, r[4], r[5], grads)
        for u in range(len(units) - 1, -1, -1):
            cd, nd = units[u]
            x = ins[u]
            _wgrad(x, da, cd, P, grads, nd, split=sp)
            if u > 0:
                dh = o.enc_conv_dgrad([da], [P[cd["w"]]], [cd["stride"]], [cd["pad"]], x.shape[1], x.shape[2],
                                      None, x, sp, bp.get(id(cd)))
                pnd = units[u - 1][1]
                r = _norm_bwd(o, pnd, dh, acts[u - 1], coefs[u - 1], False, None, None, sp)
                da = r[0]
                _norm_grads(pnd, r[2], r[3], grads)
            else:
                dys, ws, ss, ps = [da], [P[cd["w"]]], [cd["stride"]], [cd["pad"]]
                if down is not None:
                    dcd = down[0]
                    dys.append(dad)
                    ws.append(P[dcd["w"]])
                    ss.append(dcd["stride"])
                    ps.append(dcd["pad"])
                    _wgrad(x, dad, dcd, P, grads, dnd, split=sp)
                g = o.enc_conv_dgrad(dys, ws, ss, ps, x.shape[1], x.shape[2], None if down is not None else g, x, sp,
                                     bp.get(id(cd)))
    x0, a0, c0, _h0 = stem_rec
    sc, sn = L.stem
    r = _norm_bwd(o, sn, g, a0, c0, False, None, None, sp)
    _norm_grads(sn, r[2], r[3], grads)
    _wgrad(x0, r[0], sc, P, grads, sn, split=sp)
    return grads


def _one_block(grads):
    """The gradients packed into views of one fp32 allocation (one multi-tensor copy).

    Gradients computed on a side stream and consumed on the main stream must be
    ``record_stream``-ed; the caching allocator then records an event on the main stream for
    every such block when it is freed (``optimizer.zero_grad``), and each event costs the main
    stream GPU time (~7 us on MI355X).  Packed, the ~45 context-encoder gradients free as one
    block: one event."""
    live = [g for g in grads if g is not None]
    if len(live) < 2 or any(g.dtype != torch.float32 for g in live):
        return grads
    flat = torch.empty(sum(g.numel() for g in live), device=live[0].device, dtype=torch.float32)
    views, off = {}, 0
    for i, g in enumerate(grads):
        if g is None:
            continue
        dims = sorted((st, n) for st, n in zip(g.stride(), g.shape) if n != 1)
        expect, dense = 1, True
        for st, n in dims:
            dense = dense and st == expect
            expect *= n
        stride = g.stride() if dense else torch.empty(g.shape).stride()
        views[i] = torch.as_strided(flat, g.shape, stride, off)
        off += g.numel()
    idx = sorted(views)
    torch._foreach_copy_([views[i] for i in idx], [grads[i] for i in idx])
    return [views.get(i) for i in range(len(grads))]


class _EncoderFn(torch.autograd.Function):
    """bf16 AMP (``split=False``: bf16 NHWC output) or fp32 training (``split=True``: the
    split-bf16 network, fp32 NHWC output = hi + lo planes)."""

    @staticmethod
    def forward(ctx, layout, x0, join, split, pk, *params):
        y, stem_rec, recs = _forward(layout, x0, params, split, pk)
        ctx.pk = pk
        ctx.layout = layout
        ctx.params = params
        ctx.join = join
        ctx.split = split
        ctx.dt16 = x0.dtype  # bf16, or fp16 under fp16 AMP
        # records hold only tensors created here (activations, statistics coefficients)
        ctx.stem_rec, ctx.recs = stem_rec, recs
        if split:
            return _unsplit(y, split)
        return y

    @staticmethod
    def backward(ctx, gy):
        gy = _split_rows(gy, ctx.split) if ctx.split else gy.contiguous().to(ctx.dt16)
        pk = ctx.pk if ctx.pk is not None and ctx.pk.need_bwd else None
        grads = _backward(ctx.layout, ctx.params, gy, ctx.stem_rec, ctx.recs, ctx.split, pk)
        ctx.stem_rec = ctx.recs = None
        if ctx.join is not None:
            # the forward ran on a side stream, so autograd ran this backward there too: make
            # the join stream (the model's main stream) wait for the parameter gradients before
            # anything else reads them -- DDP starts a bucket's all-reduce from whichever
            # gradient hook fires last and orders it only after THAT hook's stream, so a bucket
            # shared with main-stream gradients must not see these still in flight
            cur = torch.cuda.current_stream(gy.device)
            if cur != ctx.join:
                grads = _one_block(grads)
                ctx.join.wait_stream(cur)
                for g in grads:  # views of one block: ONE allocator event when it is freed
                    if g is not None:
                        g.record_stream(ctx.join)
                        break
        return (None, None, None, None, None, *grads)


def _layout(enc):
    # the parameter objects and the BatchNorm train/eval state define the layout
    # (and the norm modules themselves: convert_sync_bn swaps BatchNorm2d modules for synced ones
    # that keep the same parameter objects)
    key = tuple(id(p) for p in enc.parameters()) + tuple(
        (id(m), type(m), m.training) for m in enc.modules() if isinstance(m, nn.BatchNorm2d))
    cached = getattr(enc, "_native_layout", None)
    if cached is None or cached[0] != key:
        cached = (key, _Layout(enc))
        object.__setattr__(enc, "_native_layout", cached)
    return cached[1]


def encode(enc, image1: torch.Tensor, image2: torch.Tensor | None = None,
           join_stream: torch.cuda.Stream | None = None, split: bool = False, f16: bool = False,
           pack_stream: str = "wgrad") -> torch.Tensor:
    """Run ``enc`` natively on raw 0..255 fp32 images (``image2``: second frame of a
    paired batch).  Returns the (n, C, H/8, W/8) bf16 feature map in channels-last
    layout (``n`` = 2B when paired).  ``join_stream``: when this runs on a side stream,
    the stream that must see the parameter gradients complete (see ``_EncoderFn.backward``).
    ``split``: fp32-faithful mode (no AMP; training or inference): the fp32 feature map.
    ``f16``: fp16 activations (fp16 AMP, v_mfma_f32_32x32x16_f16) instead of bf16.
    ``pack_stream``: the auxiliary stream (ops/streams.py) that packs the weights ahead."""
    L = _layout(enc)
    # split mode: 1 = [hi | lo | hi] planes (inference: fp32-faithful to ~2^-17, EPE within 1e-5 px
    # of the fp32 reference), 2 = [hi | mid | lo] planes with a six-plane forward GEMM (training:
    # the forward activations are fp32-exact; their 16-bit rounding was the fp32 training path's
    # dominant gradient error, profiles/r5_split_precision_by_scope.txt)
    mode = 0 if not split else (2 if torch.is_grad_enabled() and SPLIT3 else 1)
    x0 = ops().enc_prep(image1.float(), image2.float() if image2 is not None else None, mode, f16 and not split)
    pk = _prepack(L, x0, mode, bool(f16 and not split), pack_stream)
    if split and not torch.is_grad_enabled():
        y = _forward_split(L, x0, L.params, pk, mode)
        return _unsplit(y, mode).permute(0, 3, 1, 2)
    y = _EncoderFn.apply(L, x0, join_stream, mode, pk, *L.params)
    return y.permute(0, 3, 1, 2)
