"""Correlation blocks: dense all-pairs pyramid and the memory-efficient local path.

``CorrPyramid`` is the MI355X replacement for the reference ``CorrBlock``
(core/corr.py:12-50) and ``LocalCorrPyramid`` for ``AlternateCorrBlock``
(core/corr.py:63-91).  Both expose ``__call__(coords) -> (B, L*(2r+1)^2, H, W)``.

Dense path on the GPU (kernels: csrc/corr_volume.hip):

* ``_BuildPyramid`` computes every level as its own MFMA GEMM,
  ``level_l = f1 . pool_l(f2)^T / sqrt(C)`` (the volume is linear in fmap2, so
  pooling fmap2 equals pooling the volume; no pass over the O(HW^2) volume).
  Without AMP the GEMMs run in split mode (fp32 operands as hi+lo bf16, three
  MFMAs per product), which keeps the volume fp32-faithful like the reference
  (core/raft.py:102-103); under AMP the operands are rounded to bf16.
  Its only differentiable output is a scalar *token*.
* every refinement iteration calls ``_Lookup(token, coords)`` (or the fused
  update step does the same lookup); its backward only records the window
  gradient.  The pyramid backward then writes every query's level-gradient row
  once (``corr_lookup_grad_rows``: the row accumulated in LDS over all the
  step's lookups, bf16 under AMP) -- instead of zeroing an fp32 buffer and
  read-modify-writing it once per lookup.
* autograd runs ``_BuildPyramid.backward`` only after every lookup's backward
  (they all feed the token): ``dF1 = sum_l dL_l . pool_l(f2)`` and
  ``dF2 = sum_l unpool_l(dL_l^T . f1)`` as GEMMs straight from the level
  gradients -- no dense HW x HW ``dC`` / ``dC^T`` is ever formed.

Each level is stored in 16-column blocks (pixel (y, x) of a level at
((x // 16) * Hl + y) * 16 + x % 16 of the query's row) by ordering the pooled-fmap2
GEMM operand that way: a (2r+2)^2 lookup window is then 1-2 contiguous runs instead
of 2r+2 rows, which is what the memory-bound lookup kernels pay for.
"""
from __future__ import annotations

import math
import os
from typing import List, Optional

import torch
import torch.nn.functional as F

from . import reference as ref
from ._ext import ops, use_native

# RAFT_CORR_BWD_BLAS=1: the bf16 pyramid-backward GEMMs on hipBLASLt (torch.baddbmm) instead of
# the hand-written corr_bwd_kernel (csrc/corr_volume.hip) -- an A/B switch only
BWD_BLAS = os.environ.get("RAFT_CORR_BWD_BLAS", "0") == "1"

# Lookup backward mode (see _PyramidState.add_grad): deferred row accumulation (default) or
# one read-modify-write pass per lookup (RAFT_DEFER_LOOKUP_GRADS=0, for A/B measurements)
DEFER_LOOKUP_GRADS = os.environ.get("RAFT_DEFER_LOOKUP_GRADS", "1") != "0"
_GRAD_ROWS_MAX_LD = 15616  # csrc/kernel_abi.h kGradRowsMaxLd


def _pad_to(n: int, m: int) -> int:
    return (n + m - 1) // m * m


class _PyramidState:
    """Forward/backward state shared by a pyramid build and its lookups.

    All levels live in ONE buffer of B*HW rows (fp32; bf16 under AMP): level l occupies columns
    [off_l, off_l + Hl*Wl) (each level's width padded to a multiple of 8), so the
    pyramid build, dF1 and dF2 are one GEMM each over the concatenated levels."""

    def __init__(self, num_levels: int, radius: int):
        self.num_levels = num_levels
        self.radius = radius
        self.buf: Optional[torch.Tensor] = None
        self.levels: List[torch.Tensor] = []   # (B*HW, Hl, Wl) views into buf
        self.dbuf: Optional[torch.Tensor] = None
        self.dlevels: Optional[List[torch.Tensor]] = None
        self.sizes = []                        # (Hl, Wl, off) per level
        self.tail = None                       # stream of fused-step lookup backwards (to join)
        self.tail_event = None                 # or the point of it to join (work queued after it is not ours)
        self.ld = 0
        self.shape = None
        self.pending: List[tuple] = []         # deferred (coords, window gradient) of each lookup

    def deferrable(self) -> bool:
        """Whether lookup gradients can be deferred to one row-accumulating pass at the pyramid
        backward (a level-gradient row fits the kernel's LDS) instead of read-modify-writing a
        zeroed fp32 buffer once per lookup."""
        return DEFER_LOOKUP_GRADS and 0 < self.ld <= _GRAD_ROWS_MAX_LD and self.radius <= 6 and self.num_levels <= 4

    def add_grad(self, coords: torch.Tensor, grad: torch.Tensor) -> None:
        """The window gradient ``grad`` (B, H, W, >= L*(2r+1)^2) of the lookup at ``coords``."""
        if self.deferrable():
            self.pending.append((coords, grad))
        else:
            ops().corr_lookup_backward_(self.grad_buffers(), coords, grad, self.radius)

    def level_grads(self, dtype: torch.dtype) -> Optional[torch.Tensor]:
        """(B*HW, ld) level-gradient rows of every lookup so far: the deferred ones written in
        one pass (``dtype``: bf16 for the AMP volume, fp32 for split mode), or the buffer the
        per-lookup backward accumulated into; None when no lookup has a gradient."""
        if self.pending:
            assert self.dbuf is None, "deferred and immediate lookup gradients cannot mix"
            # more lookups than one row-accumulating pass takes (kGradRowsMaxT): chunks add into
            # the rows, so keep them fp32 (no bf16 rounding of the partial sums between chunks)
            if len(self.pending) > 32:
                dtype = torch.float32
            rows = torch.empty(self.buf.shape, device=self.buf.device, dtype=dtype)
            for i in range(0, len(self.pending), 32):
                chunk = self.pending[i:i + 32]
                ops().corr_lookup_grad_rows(rows, [c for c, _ in chunk], [g for _, g in chunk], self.segments(),
                                            self.radius, i > 0)
            self.pending = []
            return rows
        return self.dbuf

    def views(self, buf: torch.Tensor) -> List[torch.Tensor]:
        # 16-column blocks: level pixel (y, x) at ((x // 16) * Hl + y) * 16 + x % 16, so a lookup
        # window is 1-2 contiguous runs instead of 2r+2 separate rows (cache lines touched)
        return [buf.as_strided((buf.shape[0], -(-Wl // 16), Hl, 16), (self.ld, Hl * 16, 16, 1),
                               buf.storage_offset() + off)
                for Hl, Wl, off in self.sizes]

    def grad_buffers(self) -> List[torch.Tensor]:
        if self.dlevels is None:  # fp32 even for a bf16 volume: 12 iterations accumulate here
            self.dbuf = torch.zeros(self.buf.shape, device=self.buf.device, dtype=torch.float32)
            self.dlevels = self.views(self.dbuf)
        return self.dlevels

    def segments(self) -> List[int]:
        out = []
        for Hl, Wl, off in self.sizes:
            out += [off, Hl, Wl]
        return out

    def release(self):
        self.buf = None
        self.levels = []
        self.dbuf = None
        self.dlevels = None
        self.pending = []


def _pooled(f: torch.Tensor, levels: int) -> List[torch.Tensor]:
    """fmap (B, C, H, W) fp32 and its 2x2 average pools (floor), levels in total."""
    out = [f]
    for _ in range(levels - 1):
        out.append(F.avg_pool2d(out[-1], 2, stride=2))
    return out


def _concat_levels(fs: List[torch.Tensor], ld: int, offs: List[int], nchw: bool, blocked: bool = False) -> torch.Tensor:
    """Pooled fmaps -> one zero-padded operand: (B, ld, C) (NHWC rows q) or (B, C, ld).
    ``blocked``: each level's pixels in 16-column block order (padding columns are zero rows,
    so their correlations are 0 -- the zero padding of the reference's grid_sample)."""
    B, C = fs[0].shape[:2]
    out = fs[0].new_zeros((B, C, ld) if nchw else (B, ld, C))
    for f, off in zip(fs, offs):
        if blocked:
            Hl, Wl = f.shape[2:]
            nb = -(-Wl // 16)
            f = F.pad(f, (0, nb * 16 - Wl)).reshape(B, C, Hl, nb, 16).permute(0, 1, 3, 2, 4)
        n = f.shape[2] * f.shape[3] * (f.shape[4] if f.dim() == 5 else 1)
        if nchw:
            out[:, :, off:off + n] = f.reshape(B, C, n)
        else:
            out[:, off:off + n] = f.reshape(B, C, n).permute(0, 2, 1)
    return out


class _BuildPyramid(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fmap1, fmap2, state: _PyramidState, split: bool):
        B, C, H, W = fmap1.shape
        HW = H * W
        k = ops()
        alpha = 1.0 / math.sqrt(C)
        # bf16 operands for the AMP volume (the store-bound v2 kernel); fp32 for split mode
        op_dt = torch.float32 if split else torch.bfloat16
        f1 = fmap1.detach().permute(0, 2, 3, 1).reshape(B, HW, C).to(op_dt).contiguous()
        sizes, off = [], 0
        for l in range(state.num_levels):
            Hl, Wl = H >> l, W >> l  # repeated 2x2 floor pooling
            sizes.append((Hl, Wl, off))
            off += -(-Wl // 16) * 16 * Hl  # 16-column blocks (see _PyramidState.views)
        ld = off
        state.sizes, state.ld = sizes, ld
        # pooled fmap2 levels in blocked order, (B, ld, C): one HIP launch (== _concat_levels(_pooled))
        f2cat = k.pyramid_operand(fmap2.detach(), state.segments(), ld, True, False, op_dt == torch.bfloat16)
        # AMP (not split): the volume is stored in bf16 -- its lookups feed bf16 convs, and the
        # lookup kernels are bound by the bytes they gather; split mode keeps it fp32-faithful
        buf = torch.empty(B * HW, ld, device=f1.device, dtype=torch.float32 if split else torch.bfloat16)
        # every level at once: buf[p][q] = alpha * f1[p] . f2cat[q]  (pad columns get 0)
        k.corr_gemm(f1, f2cat, buf, HW, ld, C, B, C, HW * C, C, ld * C, ld, HW * ld, alpha, False, split, 0)
        state.buf = buf
        state.levels = state.views(buf)
        state.shape = (B, C, H, W)
        ctx.state, ctx.split = state, split
        ctx.save_for_backward(fmap1, fmap2)
        ctx.set_materialize_grads(False)  # the token gradient is never used (may be None)
        return fmap1.new_empty((), dtype=torch.float32)  # ordering token: never read (no fill launch)

    @staticmethod
    def backward(ctx, gtoken):
        state: _PyramidState = ctx.state
        fmap1, fmap2 = ctx.saved_tensors
        tail = getattr(state, "tail", None)
        if tail is not None:  # lookups' backward ran on the fused step's tail stream
            torch.cuda.current_stream().wait_stream(tail)
            state.tail = None
            if state.dbuf is not None:
                state.dbuf.record_stream(tail)
        split = ctx.split
        # bf16 level gradients for the AMP volume: the two GEMMs below read them at half the
        # bytes (they round their A operand to bf16 anyway unless split)
        dbuf = state.level_grads(torch.float32 if split else torch.bfloat16)
        if dbuf is None:
            state.release()
            return None, None, None, None
        B, C, H, W = state.shape
        HW, ld = H * W, state.ld
        k = ops()
        alpha = 1.0 / math.sqrt(C)
        bf_ops = not split and dbuf.dtype == torch.bfloat16
        # (B, C, ld) / (B, C, HW + pad) K-contiguous B operands, bf16 straight from the kernel
        f2t = k.pyramid_operand(fmap2.detach(), state.segments(), ld, True, True, bf_ops)
        f1t = k.pyramid_operand(fmap1.detach(), [0, H, W], _pad_to(HW, 8), False, True, bf_ops)
        if bf_ops and not BWD_BLAS:
            # bf16 level gradients: both GEMMs in ONE launch of the hand-written DMA-ring MFMA
            # kernel (csrc/corr_volume.hip corr_bwd_pair_kernel):
            #   dF1 = alpha * dL . f2cat   (M = HW, N = C, K = every level column)
            #   G   = alpha * dL^T . f1    (M = every level column, N = C, K = HW; dL read
            #                               transposed through ds_read_b64_tr_b16, no dL^T copy)
            d1 = torch.empty(B, HW, C, device=fmap1.device, dtype=torch.bfloat16)
            G = torch.empty(B, ld, C, device=fmap1.device)
            k.corr_pyramid_bwd(dbuf.view(B, HW, ld), f2t, f1t, d1, G, alpha)
        elif bf_ops:
            # bf16 level gradients: both are plain batched GEMMs (the unpool is its own pass), on
            # hipBLASLt -- the generic MFMA GEMM ran them at ~9-12 % of peak (215 + 158 us per step
            # at config #2, profiles/r5o_bf16_kernels.txt) on the backward's critical path
            dL, bf = dbuf.view(B, HW, ld), torch.bfloat16
            d1 = torch.baddbmm(torch.empty(B, HW, C, device=fmap1.device, dtype=bf), dL,
                               f2t.transpose(1, 2), beta=0.0, alpha=alpha)
            G = torch.baddbmm(torch.empty(B, ld, C, device=fmap1.device, dtype=bf), dL.transpose(1, 2),
                              f1t[:, :, :HW].transpose(1, 2), beta=0.0, alpha=alpha).float()
        else:
            d1 = torch.empty(B, HW, C, device=fmap1.device)
            G = torch.empty(B, ld, C, device=fmap1.device)
            # dF1 = alpha * dL . f2cat            (M = HW, N = C, K = all levels)
            k.corr_gemm(dbuf, f2t, d1, HW, C, ld, B, ld, HW * ld, ld, C * ld, C, HW * C, alpha, False, split, 0)
            # G = alpha * dL^T . f1  per level row (M = all levels, N = C, K = HW; A read transposed),
            # dF2 = sum_l unpool_l(G_l)
            k.corr_gemm(dbuf, f1t, G, ld, C, HW, B, ld, HW * ld, f1t.shape[2], C * f1t.shape[2], C, ld * C, alpha,
                        True, split, 0)
        d2 = k.pyramid_unpool(G, H, W, state.segments(), True)
        state.release()
        g1 = d1.view(B, H, W, C).permute(0, 3, 1, 2)
        g2 = d2.view(B, H, W, C).permute(0, 3, 1, 2)
        return g1.to(fmap1.dtype), g2.to(fmap2.dtype), None, None


class _Lookup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, token, coords, state: _PyramidState, out_dtype, out_channels=0):
        coords = coords.detach().float().contiguous()
        out = ops().corr_lookup(state.levels, coords, state.radius, out_dtype, out_channels)
        ctx.state = state
        ctx.save_for_backward(coords)
        return out

    @staticmethod
    def backward(ctx, gout):
        (coords,) = ctx.saved_tensors
        state: _PyramidState = ctx.state
        if state.levels:
            state.add_grad(coords, gout.contiguous())
        return torch.zeros((), device=gout.device), None, None, None, None


class CorrPyramid:
    """All-pairs correlation pyramid with radius-``radius`` lookup.

    GPU: native HIP/MFMA path (see module docstring); ``split=True`` keeps the volume
    fp32-faithful (use it without AMP).  CPU: reference ops.  ``out_dtype`` selects the
    dtype of the looked-up features (bf16 under autocast feeds the motion encoder
    without an extra cast).
    """

    def __init__(self, fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4, radius: int = 4,
                 split: bool = False):
        self.num_levels = num_levels
        self.radius = radius
        self.native = use_native(fmap1)
        if self.native:
            self.state = _PyramidState(num_levels, radius)
            self.token = _BuildPyramid.apply(fmap1, fmap2, self.state, bool(split))
        else:
            corr = ref.corr_volume(fmap1.float(), fmap2.float())
            self.pyramid = ref.build_pyramid(corr, num_levels)

    def lookup_padded(self, coords: torch.Tensor, out_channels: int, out_dtype=torch.bfloat16) -> torch.Tensor:
        """Native only: (B, H, W, out_channels) NHWC features, zero beyond L*(2r+1)^2
        (the K padding the fused motion encoder's 1x1 conv expects)."""
        return _Lookup.apply(self.token, coords, self.state, out_dtype, out_channels)

    def __call__(self, coords: torch.Tensor, out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        if self.native:
            dt = out_dtype or torch.float32
            out = _Lookup.apply(self.token, coords, self.state, dt, 0)
            return out.permute(0, 3, 1, 2)  # channels-last view (B, Ch, H, W)
        out = ref.pyramid_lookup(self.pyramid, coords, self.radius)
        return out if out_dtype is None else out.to(out_dtype)


# --------------------------------------------------------------------- local path
class _LocalCorr(torch.autograd.Function):
    """fp32 scalar kernel (csrc/local_corr.hip): the exact path used without AMP."""

    @staticmethod
    def forward(ctx, f1, f2, coords, radius: int, scale: float):
        coords = coords.detach().float().contiguous()
        out = ops().local_corr(f1, f2, coords, radius, scale)
        ctx.save_for_backward(f1, f2, coords)
        ctx.radius, ctx.scale = radius, scale
        return out

    @staticmethod
    def backward(ctx, gout):
        f1, f2, coords = ctx.saved_tensors
        g1, g2 = ops().local_corr_backward(f1, f2, coords, gout, ctx.radius, ctx.scale,
                                           torch.are_deterministic_algorithms_enabled())
        return g1.to(f1.dtype), g2.to(f2.dtype), None, None, None


class _LocalCorrMFMA(torch.autograd.Function):
    """All levels in one MFMA launch (csrc/local_corr_mfma.hip); output (P, out_channels)
    rows, level l taps at channel l*(2r+1)^2 (the fused update block's layout)."""

    @staticmethod
    def forward(ctx, fmap1, fmap2, coords, st: "LocalCorrPyramid", out_channels: int, out_dtype):
        coords = coords.detach().float().contiguous()
        P = st.f1.shape[0]
        out = torch.empty(P, out_channels, device=coords.device, dtype=out_dtype)
        ops().local_corr_mfma(st.f1, st.f2cat, coords, st.segs, st.radius, st.scale, out)
        ctx.st = st
        ctx.save_for_backward(coords)
        ctx.dtypes = (fmap1.dtype, fmap2.dtype)
        return out

    @staticmethod
    def backward(ctx, gout):
        (coords,) = ctx.saved_tensors
        st: LocalCorrPyramid = ctx.st
        g1 = torch.empty(st.f1.shape, device=gout.device)
        g2 = torch.zeros(st.f2cat.shape, device=gout.device)
        gout = gout.reshape(st.f1.shape[0], -1).contiguous()
        ops().local_corr_mfma_backward(st.f1, st.f2cat, coords, st.segs, st.radius, st.scale, gout, g1, g2,
                                       torch.are_deterministic_algorithms_enabled())
        B, C, H, W = st.shape
        d2 = ops().pyramid_unpool(g2, H, W, st.segs)  # level gradients -> level 0 (adjoint pools)
        d1 = g1.view(B, H, W, C).permute(0, 3, 1, 2)
        d2 = d2.view(B, H, W, C).permute(0, 3, 1, 2)
        return d1.to(ctx.dtypes[0]), d2.to(ctx.dtypes[1]), None, None, None, None


def _split_cat(x: torch.Tensor, planes) -> torch.Tensor:
    """fp32 rows (..., C) -> bf16 (..., 3C): the hi (0) / lo (1) bf16 parts in ``planes`` order."""
    xf = x.float()
    hi = xf.to(torch.bfloat16)
    lo = (xf - hi.float()).to(torch.bfloat16)
    return torch.cat([(hi, lo)[p] for p in planes], dim=-1).contiguous()


class LocalCorrPyramid:
    """Memory-efficient correlation: no HW x HW volume is ever stored.

    Pools fmap2 (not the volume; equivalent by linearity) into ``num_levels`` levels once,
    and per lookup computes the (2r+1)^2 window correlations on the fly.  Under AMP (bf16)
    every level is done by one MFMA kernel over 8x4 query tiles (``local_corr_mfma``);
    without AMP (``split=True``) inference runs the same kernel on split-bf16 operands
    (f1 as [hi | lo | hi], the pooled f2 as [hi | hi | lo] along K: one GEMM computes
    hi.hi + lo.hi + hi.lo, fp32-faithful) and fp32 training the exact scalar fp32 kernel.
    Both train (the reference's alt_cuda_corr path is forward-only, core/corr.py:86).
    """

    def __init__(self, fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4, radius: int = 4,
                 feature_dtype: Optional[torch.dtype] = None, split: bool = True):
        self.num_levels = num_levels
        self.radius = radius
        self.native = use_native(fmap1)
        B, C, H, W = fmap1.shape
        self.C = C
        self.shape = (B, C, H, W)
        self.scale = 1.0 / math.sqrt(C)
        mfma_ok = self.native and C % 64 == 0 and C <= 256 and radius <= 4
        # split-bf16 MFMA: fp32-faithful, forward only (the backward keeps the exact kernel)
        self.split_mfma = mfma_ok and split and not torch.is_grad_enabled()
        self.mfma = mfma_ok and (not split or self.split_mfma)
        self.fmap1, self.fmap2 = fmap1, fmap2
        if self.mfma:
            f1 = fmap1.detach().permute(0, 2, 3, 1).reshape(B * H * W, C)
            segs, off = [], 0
            for l in range(num_levels):
                Hl, Wl = H >> l, W >> l  # repeated 2x2 floor pooling
                segs += [off, Hl, Wl]
                off += _pad_to(Hl * Wl, 8)
            self.segs = segs
            # pooled fmap2 levels, (B, rows, C): one HIP launch (== _concat_levels(_pooled))
            f2cat = ops().pyramid_operand(fmap2.detach(), segs, off, False, False)
            if self.split_mfma:
                self.f1 = _split_cat(f1, (0, 1, 0))
                self.f2cat = _split_cat(f2cat, (0, 0, 1))
            else:
                self.f1 = f1.to(torch.bfloat16).contiguous()
                self.f2cat = f2cat.to(torch.bfloat16)
        elif self.native:
            dt = feature_dtype or torch.float32
            self.f1 = fmap1.permute(0, 2, 3, 1).to(dt).contiguous()
            f2 = fmap2
            self.f2 = []
            for i in range(num_levels):
                if i > 0:
                    f2 = F.avg_pool2d(f2, 2, stride=2)
                self.f2.append(f2.permute(0, 2, 3, 1).to(dt).contiguous())
        else:
            self.fmap1 = fmap1.float()
            self.fmap2 = [fmap2.float()]
            for i in range(1, num_levels):
                self.fmap2.append(F.avg_pool2d(self.fmap2[-1], 2, stride=2))

    def lookup_padded(self, coords: torch.Tensor, out_channels: int, out_dtype=torch.bfloat16) -> torch.Tensor:
        """MFMA path only: (B, H, W, out_channels) features, zero beyond L*(2r+1)^2."""
        B, _, H, W = self.shape
        out = _LocalCorrMFMA.apply(self.fmap1, self.fmap2, coords, self, out_channels, out_dtype)
        return out.view(B, H, W, out_channels)

    def __call__(self, coords: torch.Tensor, out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        if self.mfma:
            win = (2 * self.radius + 1) ** 2
            dt = out_dtype or torch.float32
            kdt = dt if dt in (torch.float32, torch.bfloat16) else torch.float32  # the kernel writes fp32 / bf16
            out = self.lookup_padded(coords, self.num_levels * win, kdt)
            return (out if kdt == dt else out.to(dt)).permute(0, 3, 1, 2)
        outs = []
        for i in range(self.num_levels):
            ci = coords / (2 ** i)
            if self.native:
                o = _LocalCorr.apply(self.f1, self.f2[i], ci.detach().contiguous(), self.radius, self.scale)
                outs.append(o)  # (B, H, W, win)
            else:
                outs.append(ref.local_corr(self.fmap1, self.fmap2[i], ci, self.radius).permute(0, 2, 3, 1) * self.scale)
        out = torch.cat(outs, dim=-1).permute(0, 3, 1, 2)
        return out if out_dtype is None else out.to(out_dtype)
