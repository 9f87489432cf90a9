"""Validation and benchmark-submission writers (reference evaluate.py:21-166).

* ``validate_chairs`` (24 iterations, EPE), ``validate_sintel`` (32 iterations,
  clean + final: EPE and 1/3/5 px rates, centred padding), ``validate_kitti``
  (24 iterations, bottom padding; EPE = mean of per-image means, F1 = % of
  valid pixels with epe > 3 and epe/|gt| > 0.05);
* ``create_sintel_submission`` (optional warm start with ``forward_interpolate``)
  and ``create_kitti_submission``;
* ``validate_synthetic`` -- the same EPE protocol on generated pairs with exact
  ground truth, for environments without the datasets.

Differences from the reference: the device is a parameter (not hard-coded
``.cuda()``), inference runs under ``torch.inference_mode``, and under DDP the
validation set is sharded over ranks with the per-pixel statistics reduced
exactly (sums and counts, not means of means).
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np
import torch

from ..data import datasets, frame_utils
from ..data.synthetic import synthetic_batch
from ..utils.utils import InputPadder, forward_interpolate


def _device(model) -> torch.device:
    return next(model.parameters()).device


def _shard(n: int, rank: int, world: int):
    return range(rank, n, world)


def _reduce(vals, device, world):
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    if world > 1:
        torch.distributed.all_reduce(t)
    return t.tolist()


@torch.inference_mode()
def create_sintel_submission(model, iters=32, warm_start=False, output_path="sintel_submission"):
    """Write .flo files for the Sintel test set (clean + final)."""
    model.eval()
    dev = _device(model)
    for dstype in ["clean", "final"]:
        test_dataset = datasets.MpiSintel(split="test", aug_params=None, dstype=dstype)
        flow_prev, sequence_prev = None, None
        for test_id in range(len(test_dataset)):
            image1, image2, (sequence, frame) = test_dataset[test_id]
            if sequence != sequence_prev:
                flow_prev = None
            padder = InputPadder(image1.shape)
            image1, image2 = padder.pad(image1[None].to(dev), image2[None].to(dev))
            flow_low, flow_pr = model(image1, image2, iters=iters, flow_init=flow_prev, test_mode=True)
            flow = padder.unpad(flow_pr[0]).permute(1, 2, 0).cpu().numpy()
            if warm_start:
                flow_prev = forward_interpolate(flow_low[0])[None].to(dev)
            output_dir = os.path.join(output_path, dstype, sequence)
            os.makedirs(output_dir, exist_ok=True)
            frame_utils.writeFlow(os.path.join(output_dir, "frame%04d.flo" % (frame + 1)), flow)
            sequence_prev = sequence


@torch.inference_mode()
def create_kitti_submission(model, iters=24, output_path="kitti_submission"):
    """Write 16-bit PNG flow files for the KITTI-2015 test set."""
    model.eval()
    dev = _device(model)
    test_dataset = datasets.KITTI(split="testing", aug_params=None)
    os.makedirs(output_path, exist_ok=True)
    for test_id in range(len(test_dataset)):
        image1, image2, (frame_id,) = test_dataset[test_id]
        padder = InputPadder(image1.shape, mode="kitti")
        image1, image2 = padder.pad(image1[None].to(dev), image2[None].to(dev))
        _, flow_pr = model(image1, image2, iters=iters, test_mode=True)
        flow = padder.unpad(flow_pr[0]).permute(1, 2, 0).cpu().numpy()
        frame_utils.writeFlowKITTI(os.path.join(output_path, frame_id), flow)


@torch.inference_mode()
def validate_chairs(model, iters=24, rank=0, world=1) -> Dict[str, float]:
    """EPE on the FlyingChairs validation split."""
    model.eval()
    dev = _device(model)
    val_dataset = datasets.FlyingChairs(split="validation")
    s = n = 0.0
    for val_id in _shard(len(val_dataset), rank, world):
        image1, image2, flow_gt, _ = val_dataset[val_id]
        _, flow_pr = model(image1[None].to(dev), image2[None].to(dev), iters=iters, test_mode=True)
        epe = torch.sum((flow_pr[0].float().cpu() - flow_gt) ** 2, dim=0).sqrt()
        s += epe.sum().item()
        n += epe.numel()
    s, n = _reduce([s, n], dev, world)
    epe = s / max(n, 1)
    if rank == 0:
        print("Validation Chairs EPE: %f" % epe)
    return {"chairs": epe}


@torch.inference_mode()
def validate_sintel(model, iters=32, rank=0, world=1) -> Dict[str, float]:
    """EPE and 1/3/5-px rates on the Sintel training split (clean and final)."""
    model.eval()
    dev = _device(model)
    results = {}
    for dstype in ["clean", "final"]:
        val_dataset = datasets.MpiSintel(split="training", dstype=dstype)
        acc = np.zeros(5)  # sum epe, count, <1, <3, <5
        for val_id in _shard(len(val_dataset), rank, world):
            image1, image2, flow_gt, _ = val_dataset[val_id]
            image1, image2 = image1[None].to(dev), image2[None].to(dev)
            padder = InputPadder(image1.shape)
            image1, image2 = padder.pad(image1, image2)
            _, flow_pr = model(image1, image2, iters=iters, test_mode=True)
            flow = padder.unpad(flow_pr[0]).float().cpu()
            epe = torch.sum((flow - flow_gt) ** 2, dim=0).sqrt().view(-1)
            acc += [epe.sum().item(), epe.numel(), (epe < 1).sum().item(), (epe < 3).sum().item(),
                    (epe < 5).sum().item()]
        acc = np.array(_reduce(acc.tolist(), dev, world))
        cnt = max(acc[1], 1)
        epe, px1, px3, px5 = acc[0] / cnt, acc[2] / cnt, acc[3] / cnt, acc[4] / cnt
        if rank == 0:
            print("Validation (%s) EPE: %f, 1px: %f, 3px: %f, 5px: %f" % (dstype, epe, px1, px3, px5))
        results[dstype] = epe
    return results


@torch.inference_mode()
def validate_kitti(model, iters=24, rank=0, world=1) -> Dict[str, float]:
    """KITTI-2015 training split: EPE (mean of per-image means) and F1-all (%)."""
    model.eval()
    dev = _device(model)
    val_dataset = datasets.KITTI(split="training")
    acc = np.zeros(4)  # sum of per-image epe means, images, outliers, valid pixels
    for val_id in _shard(len(val_dataset), rank, world):
        image1, image2, flow_gt, valid_gt = val_dataset[val_id]
        image1, image2 = image1[None].to(dev), image2[None].to(dev)
        padder = InputPadder(image1.shape, mode="kitti")
        image1, image2 = padder.pad(image1, image2)
        _, flow_pr = model(image1, image2, iters=iters, test_mode=True)
        flow = padder.unpad(flow_pr[0]).float().cpu()
        epe = torch.sum((flow - flow_gt) ** 2, dim=0).sqrt().view(-1)
        mag = torch.sum(flow_gt ** 2, dim=0).sqrt().view(-1)
        val = valid_gt.view(-1) >= 0.5
        out = ((epe > 3.0) & ((epe / mag) > 0.05)).float()
        acc += [epe[val].mean().item(), 1, out[val].sum().item(), val.sum().item()]
    acc = _reduce(acc.tolist(), dev, world)
    epe = acc[0] / max(acc[1], 1)
    f1 = 100 * acc[2] / max(acc[3], 1)
    if rank == 0:
        print("Validation KITTI: %f, %f" % (epe, f1))
    return {"kitti-epe": epe, "kitti-f1": f1}


@torch.inference_mode()
def validate_synthetic(model, iters=24, n_pairs=16, size=(368, 496), seed=12345, rank=0, world=1,
                       max_disp=20.0) -> Dict[str, float]:
    """EPE / 1/3/5 px on generated pairs with exact ground truth (no dataset needed)."""
    model.eval()
    dev = _device(model)
    acc = np.zeros(5)
    for i in _shard(n_pairs, rank, world):
        i1, i2, flow, valid = synthetic_batch(1, size[0], size[1], max_disp=max_disp, seed=seed + i, device=dev)
        _, flow_pr = model(i1, i2, iters=iters, test_mode=True)
        epe = torch.sum((flow_pr.float() - flow) ** 2, dim=1).sqrt()[valid >= 0.5]
        acc += [epe.sum().item(), epe.numel(), (epe < 1).sum().item(), (epe < 3).sum().item(), (epe < 5).sum().item()]
    acc = np.array(_reduce(acc.tolist(), dev, world))
    cnt = max(acc[1], 1)
    res = {"synthetic-epe": acc[0] / cnt, "synthetic-1px": acc[2] / cnt, "synthetic-3px": acc[3] / cnt,
           "synthetic-5px": acc[4] / cnt}
    if rank == 0:
        print("Validation (synthetic) EPE: %f, 1px: %f, 3px: %f, 5px: %f" % tuple(
            res[k] for k in ("synthetic-epe", "synthetic-1px", "synthetic-3px", "synthetic-5px")))
    return res


VALIDATORS = {"chairs": validate_chairs, "sintel": validate_sintel, "kitti": validate_kitti,
              "synthetic": validate_synthetic}


def run_validation(model, names, rank=0, world=1) -> Dict[str, float]:
    results: Dict[str, float] = {}
    for name in names or []:
        results.update(VALIDATORS[name](model, rank=rank, world=world))
    return results
