"""Pure-PyTorch implementations of the RAFT hot ops.

These are (1) the CPU execution path (plumbing config #1 of BASELINE.json:
RAFT-small on CPU) and (2) the numerical oracle every HIP kernel is tested
against.  They reproduce the reference semantics:

* all-pairs correlation ``fmap1^T fmap2 / sqrt(C)`` -- core/corr.py:53-60
* 4-level 2x2 average-pool pyramid over the image-2 dims -- core/corr.py:25-27
* radius-r bilinear lookup (``grid_sample``, align_corners=True, zero padding,
  x-offset-major taps) -- core/corr.py:29-50, core/utils/utils.py:57-71
* convex 8x upsampling -- core/raft.py:72-83
* 8x bilinear upsampling -- core/utils/utils.py:80-82
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def coords_grid(batch: int, ht: int, wd: int, device=None, dtype=torch.float32) -> torch.Tensor:
    """(batch, 2, ht, wd) pixel-coordinate grid, channel 0 = x, channel 1 = y."""
    ys = torch.arange(ht, device=device, dtype=dtype)
    xs = torch.arange(wd, device=device, dtype=dtype)
    gy, gx = torch.meshgrid(ys, xs, indexing="ij")
    return torch.stack([gx, gy], dim=0)[None].expand(batch, 2, ht, wd).contiguous()


def bilinear_sampler(img: torch.Tensor, coords: torch.Tensor, mode: str = "bilinear", mask: bool = False):
    """``grid_sample`` with pixel coordinates (last dim of ``coords`` = (x, y))."""
    H, W = img.shape[-2:]
    x, y = coords[..., 0:1], coords[..., 1:2]
    gx = 2.0 * x / (W - 1) - 1.0
    gy = 2.0 * y / (H - 1) - 1.0
    grid = torch.cat([gx, gy], dim=-1)
    out = F.grid_sample(img, grid, mode=mode, align_corners=True)
    if mask:
        valid = (gx > -1) & (gy > -1) & (gx < 1) & (gy < 1)
        return out, valid.float()
    return out


def corr_volume(fmap1: torch.Tensor, fmap2: torch.Tensor) -> torch.Tensor:
    """(B, C, H, W) x2 -> (B*H*W, 1, H, W) all-pairs correlation scaled by 1/sqrt(C)."""
    B, C, H, W = fmap1.shape
    a = fmap1.reshape(B, C, H * W).transpose(1, 2)
    b = fmap2.reshape(B, C, H * W)
    corr = torch.matmul(a, b) / math.sqrt(C)
    return corr.reshape(B * H * W, 1, H, W)


def build_pyramid(corr: torch.Tensor, num_levels: int):
    pyr = [corr]
    for _ in range(num_levels - 1):
        corr = F.avg_pool2d(corr, 2, stride=2)
        pyr.append(corr)
    return pyr


def window_offsets(radius: int, device=None, dtype=torch.float32) -> torch.Tensor:
    """(2r+1, 2r+1, 2) offsets; [i, j] = (dx_i, dy_j): the first axis moves x."""
    d = torch.arange(-radius, radius + 1, device=device, dtype=dtype)
    dx, dy = torch.meshgrid(d, d, indexing="ij")
    return torch.stack([dx, dy], dim=-1)


def pyramid_lookup(pyramid, coords: torch.Tensor, radius: int) -> torch.Tensor:
    """Sample every pyramid level around ``coords`` (B, 2, H, W).

    Returns (B, L*(2r+1)^2, H, W) fp32, level-major / x-offset-major channels.
    """
    B, _, H, W = coords.shape
    c = coords.permute(0, 2, 3, 1).reshape(B * H * W, 1, 1, 2)
    delta = window_offsets(radius, coords.device, coords.dtype)[None]
    outs = []
    for lvl, corr in enumerate(pyramid):
        pts = c / (2 ** lvl) + delta
        sampled = bilinear_sampler(corr, pts)
        outs.append(sampled.reshape(B, H, W, -1))
    return torch.cat(outs, dim=-1).permute(0, 3, 1, 2).contiguous().float()


def convex_upsample(flow: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """Upsample (B, 2, H, W) flow 8x as a softmax-weighted 3x3 convex combination."""
    B, _, H, W = flow.shape
    m = torch.softmax(mask.reshape(B, 1, 9, 8, 8, H, W).float(), dim=2)
    nb = F.unfold(8.0 * flow, [3, 3], padding=1).reshape(B, 2, 9, 1, 1, H, W)
    up = (m * nb).sum(dim=2)  # (B, 2, 8, 8, H, W)
    return up.permute(0, 1, 4, 2, 5, 3).reshape(B, 2, 8 * H, 8 * W)


def upflow8(flow: torch.Tensor, mode: str = "bilinear") -> torch.Tensor:
    size = (8 * flow.shape[2], 8 * flow.shape[3])
    return 8.0 * F.interpolate(flow, size=size, mode=mode, align_corners=True)


def local_corr(fmap1: torch.Tensor, fmap2: torch.Tensor, coords: torch.Tensor, radius: int) -> torch.Tensor:
    """Reference for the on-the-fly local correlation of one pyramid level.

    fmap1 (B, C, H1, W1), fmap2 (B, C, H2, W2), coords (B, 2, H1, W1) already in
    level-``fmap2`` pixel units.  Returns (B, (2r+1)^2, H1, W1), *unscaled* (the
    caller divides by sqrt(C), as AlternateCorrBlock does after stacking).
    Equivalent, by linearity of bilinear sampling, to sampling the dense
    volume fmap1^T fmap2.
    """
    B, C, H1, W1 = fmap1.shape
    H2, W2 = fmap2.shape[-2:]
    vol = torch.matmul(fmap1.reshape(B, C, H1 * W1).transpose(1, 2), fmap2.reshape(B, C, H2 * W2))
    vol = vol.reshape(B * H1 * W1, 1, H2, W2)
    c = coords.permute(0, 2, 3, 1).reshape(B * H1 * W1, 1, 1, 2)
    pts = c + window_offsets(radius, coords.device, coords.dtype)[None]
    out = bilinear_sampler(vol, pts)
    return out.reshape(B, H1, W1, -1).permute(0, 3, 1, 2)
