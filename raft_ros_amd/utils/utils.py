"""Geometry helpers (reference core/utils/utils.py:7-82).

``InputPadder`` (replicate-pad to a multiple of 8, 'sintel' = centred,
'kitti' = bottom only), ``forward_interpolate`` (warm start: forward-splat the
low-res flow and fill holes by nearest neighbour), ``bilinear_sampler``,
``coords_grid`` and ``upflow8``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from ..ops.reference import bilinear_sampler, coords_grid, upflow8  # noqa: F401


class InputPadder:
    """Pads images such that dimensions are divisible by 8."""

    def __init__(self, dims, mode: str = "sintel"):
        self.ht, self.wd = dims[-2:]
        pad_ht = (-self.ht) % 8
        pad_wd = (-self.wd) % 8
        if mode == "sintel":
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, pad_ht // 2, pad_ht - pad_ht // 2]
        else:
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, 0, pad_ht]

    def pad(self, *inputs):
        return [F.pad(x, self._pad, mode="replicate") for x in inputs]

    def unpad(self, x):
        ht, wd = x.shape[-2:]
        t, b, l, r = self._pad[2], ht - self._pad[3], self._pad[0], wd - self._pad[1]
        return x[..., t:b, l:r]


def forward_interpolate(flow: torch.Tensor) -> torch.Tensor:
    """Forward-warp a (2, H, W) flow onto the next frame's grid (warm start).

    Each source pixel is splatted to ``p + flow(p)``; target pixels take the
    flow of the nearest splatted point (scipy griddata 'nearest', as the
    reference does), 0 when nothing lands inside the image.
    """
    from scipy import interpolate

    f = flow.detach().cpu().numpy()
    dx, dy = f[0], f[1]
    ht, wd = dx.shape
    x0, y0 = np.meshgrid(np.arange(wd), np.arange(ht))
    x1 = (x0 + dx).reshape(-1)
    y1 = (y0 + dy).reshape(-1)
    dx = dx.reshape(-1)
    dy = dy.reshape(-1)
    keep = (x1 > 0) & (x1 < wd) & (y1 > 0) & (y1 < ht)
    x1, y1, dx, dy = x1[keep], y1[keep], dx[keep], dy[keep]
    if x1.size == 0:
        return torch.zeros(2, ht, wd, dtype=torch.float32)
    fx = interpolate.griddata((x1, y1), dx, (x0, y0), method="nearest", fill_value=0)
    fy = interpolate.griddata((x1, y1), dy, (x0, y0), method="nearest", fill_value=0)
    return torch.from_numpy(np.stack([fx, fy], axis=0)).float()
