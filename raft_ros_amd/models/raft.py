"""RAFT: Recurrent All-Pairs Field Transforms, MI355X-native execution.

Behaviour and API follow the reference orchestrator (core/raft.py:24-144):

* ``RAFT(args)`` with ``args.small``, ``args.mixed_precision``,
  ``args.alternate_corr``, ``args.dropout`` (the constructor sets
  ``args.corr_levels`` / ``args.corr_radius`` like the reference, :29-45);
* ``forward(image1, image2, iters=12, flow_init=None, upsample=True,
  test_mode=False)`` -> list of ``iters`` full-resolution flows, or
  ``(flow_lowres, flow_up)`` in test mode;
* identical parameter names, so ``raft-*.pth`` checkpoints load.

Execution differences (GPU):

* the correlation pyramid build / lookup / backward, the convex upsampler and
  the GRU gate math are native HIP kernels (``raft_ros_amd.ops``);
* under bf16 AMP both encoders run on native HIP kernels as one autograd node
  each (``ops/encoder.py``; ``args.native_encoder=False`` selects the module path);
* fp32 inference (no AMP, no autograd: the demo / evaluate / ROS default) runs the
  encoders and the refinement step on the same kernels in split-bf16 mode (hi / lo
  bf16 planes, 3 MFMA products per GEMM: fp32-faithful), so no MIOpen kernel runs;
* fp32 training (no AMP, autograd: the reference's default recipe) runs the encoders and
  the refinement step on the split-bf16 kernels too, forward and backward
  (``ops/update_split.py``, ``ops/encoder.py``);
* ``args.corr_fp32`` keeps the correlation volume fp32-faithful under bf16 AMP;
* the lookup emits channels-last features already in the autocast dtype;
* mixed precision uses ``args.amp_dtype`` (default bf16 on MI355X; 'fp16'
  reproduces the reference's fp16 autocast);
* ``args.channels_last`` (default True on GPU) keeps every conv in NHWC;
* ``args.query_shard`` (inference in a process group): the correlation volume is sharded
  over query pixels across the ranks (parallel/query_shard.py).
"""
from __future__ import annotations

from argparse import Namespace

import torch
import torch.nn as nn

from ..ops import CorrPyramid, LocalCorrPyramid, convex_upsample, upflow8
from ..ops import encoder as encoder_native
from ..ops import update_fused, update_fused_small, update_split, update_split_small
from ..ops._ext import use_native
from ..ops.reference import coords_grid
from .extractor import BasicEncoder, SmallEncoder
from .update import BasicUpdateBlock, SmallUpdateBlock

_AMP_DTYPES = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp16": torch.float16,
               "float16": torch.float16, "half": torch.float16}


def _arg(args, name, default):
    return getattr(args, name) if name in args else default


class RAFT(nn.Module):
    def __init__(self, args):
        super().__init__()
        if isinstance(args, dict):
            args = Namespace(**args)
        self.args = args
        if _arg(args, "small", False):
            self.hidden_dim = hdim = 96
            self.context_dim = cdim = 64
            args.corr_levels = 4
            args.corr_radius = 3
        else:
            self.hidden_dim = hdim = 128
            self.context_dim = cdim = 128
            args.corr_levels = 4
            args.corr_radius = 4
        if "dropout" not in args:
            args.dropout = 0
        if "alternate_corr" not in args:
            args.alternate_corr = False
        if "mixed_precision" not in args:
            args.mixed_precision = False
        if "small" not in args:
            args.small = False
        self.amp_dtype = _AMP_DTYPES[str(_arg(args, "amp_dtype", "bf16")).lower()]

        if args.small:
            self.fnet = SmallEncoder(output_dim=128, norm_fn="instance", dropout=args.dropout)
            self.cnet = SmallEncoder(output_dim=hdim + cdim, norm_fn="none", dropout=args.dropout)
            self.update_block = SmallUpdateBlock(args, hidden_dim=hdim)
        else:
            self.fnet = BasicEncoder(output_dim=256, norm_fn="instance", dropout=args.dropout)
            self.cnet = BasicEncoder(output_dim=hdim + cdim, norm_fn="batch", dropout=args.dropout)
            self.update_block = BasicUpdateBlock(args, hidden_dim=hdim)

    # ------------------------------------------------------------------ helpers
    def freeze_bn(self):
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eval()

    def initialize_flow(self, img):
        """flow = coords1 - coords0, both (N, 2, H/8, W/8) pixel grids."""
        N, _, H, W = img.shape
        coords0 = coords_grid(N, H // 8, W // 8, device=img.device)
        coords1 = coords_grid(N, H // 8, W // 8, device=img.device)
        return coords0, coords1

    def upsample_flow(self, flow, mask):
        """[H/8, W/8] -> [H, W] flow by convex combination (fused HIP kernel on GPU)."""
        return convex_upsample(flow, mask)

    def _autocast(self, device_type: str):
        enabled = bool(self.args.mixed_precision)
        if device_type == "cpu" and self.amp_dtype == torch.float16:
            enabled = False  # fp16 autocast is a GPU feature
        # the cast cache reuses a weight's bf16 copy across the refinement iterations; a
        # HIP-graph capture turns it off (runtime/train_graph.py) so that casts made outside
        # the capture cannot leak into it
        cache = getattr(self, "autocast_cache", True)
        return torch.autocast(device_type=device_type, dtype=self.amp_dtype, enabled=enabled, cache_enabled=cache)

    # ------------------------------------------------------------------ forward
    def forward(self, image1, image2, iters: int = 12, flow_init=None, upsample: bool = True,
                test_mode: bool = False):
        H, W = image1.shape[-2:]
        if min(H, W) < 128:
            # below 128 px the coarsest pyramid level degenerates (reference: NaN at
            # 64..127 px, a crash below 64 px -- SURVEY.md 2.6); refuse loudly instead
            raise ValueError(f"RAFT needs inputs of at least 128x128 pixels, got {H}x{W}")
        dev = image1.device.type
        cl = dev == "cuda" and _arg(self.args, "channels_last", True)
        fmt = torch.channels_last if cl else torch.contiguous_format

        hdim, cdim = self.hidden_dim, self.context_dim
        amp = bool(self.args.mixed_precision)
        # the batched weight-gradient token of the fused step is created before the encoders, so
        # its backward overlaps theirs (ops/update_fused.py WeightToken)
        wtoken = None
        if torch.is_grad_enabled() and update_fused.EARLY_WGRAD:
            if self._use_fused(image1, amp) and update_fused.supported(self.update_block):
                wtoken = update_fused.WeightToken(self.update_block)
            elif self._use_split_train(image1, amp):
                wtoken = (update_split_small.weight_token(self.update_block)
                          if update_split_small.supported(self.update_block)
                          else update_split.SplitWeightToken(self.update_block))
        native = self._use_native_encoders(image1, amp)
        raw1, raw2 = image1, image2
        if not native:
            image1 = (2 * (image1 / 255.0) - 1.0).contiguous(memory_format=fmt)
            image2 = (2 * (image2 / 255.0) - 1.0).contiguous(memory_format=fmt)

        cnet_native = None
        if native:
            # both encoders on the native HIP kernels (ops/encoder.py), input normalisation fused;
            # the context encoder runs on a side stream concurrently with the feature encoder
            # (autograd replays each node's backward on its forward stream, so the two backward
            # passes overlap as well)
            side = self._side_stream(raw1.device)
            main = torch.cuda.current_stream(raw1.device)
            side.wait_stream(main)
            split = not amp  # fp32: split-bf16 (fp32-faithful) encoder kernels
            f16 = amp and self.amp_dtype == torch.float16  # fp16 AMP: fp16 MFMA kernels
            with torch.cuda.stream(side):
                cnet_native = encoder_native.encode(self.cnet, raw1, join_stream=main, split=split, f16=f16,
                                                    pack_stream="tail")
            fmap1, fmap2 = encoder_native.encode(self.fnet, raw1, raw2, split=split,
                                                 f16=f16).split(raw1.shape[0], dim=0)
        else:
            with self._autocast(dev):
                fmap1, fmap2 = self.fnet([image1, image2])
        fmap1, fmap2 = fmap1.float(), fmap2.float()
        # the correlation keeps fp32 numerics (split-bf16 MFMA) except under bf16 AMP: the
        # reference builds it in fp32 outside autocast in every mode (core/raft.py:102-103),
        # so fp16 AMP and fp32 runs both get the fp32-faithful volume; ``args.corr_fp32`` keeps
        # it under bf16 AMP too (bf16 features are then looked up from the fp32 volume)
        split = (not (amp and dev == "cuda" and self.amp_dtype == torch.bfloat16)
                 or bool(_arg(self.args, "corr_fp32", False)))
        if self.args.alternate_corr:
            corr_fn = LocalCorrPyramid(fmap1, fmap2, radius=self.args.corr_radius, split=split)
        elif _arg(self.args, "query_shard", False) and not torch.is_grad_enabled():
            # inference over a process group: each rank holds the volume rows of its own query
            # pixels (parallel/query_shard.py)
            from ..parallel.query_shard import ShardedCorrPyramid

            corr_fn = ShardedCorrPyramid(fmap1, fmap2, num_levels=self.args.corr_levels,
                                         radius=self.args.corr_radius, split=split)
        else:
            corr_fn = CorrPyramid(fmap1, fmap2, radius=self.args.corr_radius, split=split)

        if native:  # join the context-encoder stream (the pyramid build above overlapped it)
            main.wait_stream(side)
            cnet_native.record_stream(main)
        with self._autocast(dev):
            cnet = cnet_native if native else self.cnet(image1)
            net, inp = torch.split(cnet, [hdim, cdim], dim=1)
            net = torch.tanh(net)
            inp = torch.relu(inp)

        coords0, coords1 = self.initialize_flow(raw1)
        if flow_init is not None:
            coords1 = coords1 + flow_init

        corr_dtype = self.amp_dtype if (amp and dev == "cuda") else None
        flow_predictions = []
        flow_up = None
        if self._use_fused(image1, amp):
            return self._forward_fused(corr_fn, net, inp, coords0, coords1, iters, test_mode, wtoken)
        if self._use_split(image1, amp):
            return self._forward_split(corr_fn, net, inp, coords0, coords1, iters, test_mode)
        if self._use_split_train(image1, amp):
            return self._forward_split_train(corr_fn, net, inp, coords0, coords1, iters, test_mode, wtoken)
        for it in range(iters):
            coords1 = coords1.detach()
            corr = corr_fn(coords1, out_dtype=corr_dtype)
            flow = coords1 - coords0
            if cl:
                flow = flow.contiguous(memory_format=fmt)
            with self._autocast(dev):
                net, up_mask, delta_flow = self.update_block(net, inp, corr, flow)
            coords1 = coords1 + delta_flow.float()
            if test_mode and it + 1 < iters:  # only the last upsampled flow is returned
                continue
            if up_mask is None:
                flow_up = upflow8(coords1 - coords0)
            else:
                flow_up = self.upsample_flow(coords1 - coords0, up_mask)
            flow_predictions.append(flow_up)

        if test_mode:
            return coords1 - coords0, flow_up
        return flow_predictions

    # ------------------------------------------------------------------ native encoders
    def _side_stream(self, device) -> torch.cuda.Stream:
        from ..ops.streams import aux_stream

        return aux_stream(device, "side")

    def _use_native_encoders(self, image1, amp: bool) -> bool:
        """bf16 / fp16 AMP, or fp32 (training and inference) on the split-bf16 kernels."""
        mode_ok = True
        return (mode_ok and _arg(self.args, "native_encoder", True)
                and encoder_native.supported(self.fnet, image1) and encoder_native.supported(self.cnet, image1))

    # ------------------------------------------------------------------ fused (HIP) update path
    def _use_fused(self, image1, amp: bool) -> bool:
        """bf16 or fp16 AMP on the fused HIP step (fp16: v_mfma_f32_32x32x16_f16, GradScaler)."""
        return (amp and _arg(self.args, "fused_update", True)
                and (update_fused.supported(self.update_block) or update_fused_small.supported(self.update_block))
                and use_native(image1))

    def _use_split(self, image1, amp: bool) -> bool:
        """fp32 inference (no AMP, no autograd) on the fused HIP step in split-bf16 mode."""
        return (not amp and not torch.is_grad_enabled() and _arg(self.args, "fused_update", True)
                and (update_fused.supported(self.update_block) or update_split_small.supported(self.update_block))
                and use_native(image1))

    def _use_split_train(self, image1, amp: bool) -> bool:
        """fp32 training (no AMP, autograd on: the reference's default recipe) on the fused HIP
        step in split-bf16 mode (ops/update_split.py)."""
        return (not amp and torch.is_grad_enabled() and _arg(self.args, "fused_update", True)
                and (update_split.supported(self.update_block) or update_split_small.supported(self.update_block))
                and use_native(image1))

    def _forward_split_train(self, corr_fn, net, inp, coords0, coords1, iters: int, test_mode: bool, wtoken=None):
        """fp32 refinement loop (with autograd; RAFT-small also without), every conv on the
        hand-written kernels (split-bf16: fp32-faithful products, fp32 gates / coordinates /
        accumulation): ops/update_split.py (base), ops/update_split_small.py (small)."""
        dense = isinstance(corr_fn, CorrPyramid)
        small = update_split_small.supported(self.update_block)
        cls = update_split_small.SplitSmallUpdate if small else update_split.SplitTrainBasicUpdate
        upd = cls(self.update_block, inp, coords0, iters, pyramid=corr_fn.state if dense else None, token=wtoken)
        flow_predictions = []
        flow_up = None
        for t in range(iters):
            up = not test_mode or t == iters - 1
            if dense:
                net, flow_up, coords1 = upd.step(t, net, coords1, ptoken=corr_fn.token, upsample=up)
            else:
                c = corr_fn(coords1.detach(), out_dtype=torch.float32).permute(0, 2, 3, 1)
                net, flow_up, coords1 = upd.step(t, net, coords1, corr=c, upsample=up)
            flow_predictions.append(flow_up)
        if test_mode:
            return coords1 - coords0, flow_up
        return flow_predictions

    def _forward_split(self, corr_fn, net, inp, coords0, coords1, iters: int, test_mode: bool):
        """fp32-faithful refinement loop (ops/update_fused.py SplitBasicUpdate): same math as
        the module loop above, every conv on the hand-written kernels."""
        if update_split_small.supported(self.update_block):
            return self._forward_split_train(corr_fn, net, inp, coords0, coords1, iters, test_mode)
        dense = isinstance(corr_fn, CorrPyramid)
        upd = update_fused.SplitBasicUpdate(self.update_block, inp, iters, pyramid=corr_fn.state if dense else None)
        flow_predictions = []
        flow_up = None
        for t in range(iters):
            up = not test_mode or t == iters - 1
            corr = None
            if not dense:
                c = corr_fn(coords1, out_dtype=torch.float32)
                corr = c.permute(0, 2, 3, 1).reshape(-1, c.shape[1]).float().contiguous()
            _, flow_up, coords1 = upd.step(t, net if t == 0 else None, coords1, coords0, corr=corr, upsample=up)
            if up:
                flow_predictions.append(flow_up)
        if test_mode:
            return coords1 - coords0, flow_up
        return flow_predictions

    def _forward_fused(self, corr_fn, net, inp, coords0, coords1, iters: int, test_mode: bool, wtoken=None):
        """Refinement loop on the fused HIP step (raft_ros_amd/ops/update_fused.py): lookup,
        update block, coords update and convex upsampling as one autograd node per
        iteration, weight gradients batched over all iterations; same math as the loop
        above."""
        dense = isinstance(corr_fn, CorrPyramid)
        small = update_fused_small.supported(self.update_block)
        fused = update_fused_small.FusedSmallUpdate if small else update_fused.FusedBasicUpdate
        pad = update_fused_small.CORR_PAD if small else update_fused.CORR_PAD
        kw = {"dt16": self.amp_dtype}
        if not small:
            kw["token"] = wtoken
        upd = fused(self.update_block, inp, iters, pyramid=corr_fn.state if dense else None, **kw)
        flow_predictions = []
        flow_up = None
        for t in range(iters):
            # test_mode returns only the last upsampled flow: earlier steps skip the mask head
            # and the upsampling (honoured only without autograd; results are unchanged)
            up = not test_mode or t == iters - 1
            if dense:
                net, flow_up, coords1 = upd.step(t, net, coords1, ptoken=corr_fn.token, upsample=up)
            elif getattr(corr_fn, "mfma", False) and self.amp_dtype == torch.bfloat16:
                corr = corr_fn.lookup_padded(coords1.detach(), pad)  # features already in the fused layout
                net, flow_up, coords1 = upd.step(t, net, coords1, corr=corr, upsample=up)
            else:
                c = corr_fn(coords1.detach(), out_dtype=self.amp_dtype).permute(0, 2, 3, 1)
                corr = torch.nn.functional.pad(c, (0, pad - c.shape[-1]))
                net, flow_up, coords1 = upd.step(t, net, coords1, corr=corr, upsample=up)
            flow_predictions.append(flow_up)
        if hasattr(upd, "join"):
            upd.join()  # upsampled flows computed on the fused step's tail stream
        if test_mode:
            return coords1 - coords0, flow_up
        return flow_predictions
