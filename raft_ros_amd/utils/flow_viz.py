"""Middlebury colour-wheel flow visualisation (reference core/utils/flow_viz.py).

Baker et al., "A Database and Evaluation Methodology for Optical Flow"
(ICCV 2007).  The wheel has 55 hues: RY 15, YG 6, GC 4, CB 11, BM 13, MR 6.
Flow is normalised by its maximum radius, the angle picks (and linearly
blends) a hue, and the magnitude desaturates toward white; radii > 1 are
dimmed by 0.75.
"""
from __future__ import annotations

import numpy as np

_SEGMENTS = (("RY", 15), ("YG", 6), ("GC", 4), ("CB", 11), ("BM", 13), ("MR", 6))


def make_colorwheel() -> np.ndarray:
    """(55, 3) float array of RGB hues in [0, 255]."""
    rows = []
    for name, n in _SEGMENTS:
        ramp = np.floor(255 * np.arange(n) / n)
        full = np.full(n, 255.0)
        zero = np.zeros(n)
        # (R, G, B) per segment: one channel ramps up or down between two saturated ones
        seg = {
            "RY": (full, ramp, zero),
            "YG": (255 - ramp, full, zero),
            "GC": (zero, full, ramp),
            "CB": (zero, 255 - ramp, full),
            "BM": (ramp, zero, full),
            "MR": (full, zero, 255 - ramp),
        }[name]
        rows.append(np.stack(seg, axis=1))
    return np.concatenate(rows, axis=0)


def flow_uv_to_colors(u: np.ndarray, v: np.ndarray, convert_to_bgr: bool = False) -> np.ndarray:
    """Map normalised flow components (H, W) to a uint8 (H, W, 3) image."""
    wheel = make_colorwheel()
    ncols = wheel.shape[0]
    rad = np.sqrt(u * u + v * v)
    ang = np.arctan2(-v, -u) / np.pi
    fk = (ang + 1) / 2 * (ncols - 1)
    k0 = np.floor(fk).astype(np.int32)
    k1 = k0 + 1
    k1[k1 == ncols] = 0
    frac = fk - k0
    img = np.zeros(u.shape + (3,), np.uint8)
    inside = rad <= 1
    for ch in range(3):
        c0 = wheel[k0, ch] / 255.0
        c1 = wheel[k1, ch] / 255.0
        col = (1 - frac) * c0 + frac * c1
        col = np.where(inside, 1 - rad * (1 - col), col * 0.75)
        img[:, :, 2 - ch if convert_to_bgr else ch] = np.floor(255 * col)
    return img


def flow_to_image(flow_uv: np.ndarray, clip_flow=None, convert_to_bgr: bool = False) -> np.ndarray:
    """(H, W, 2) flow -> (H, W, 3) uint8 colour image."""
    assert flow_uv.ndim == 3, "input flow must have three dimensions"
    assert flow_uv.shape[2] == 2, "input flow must have shape [H,W,2]"
    if clip_flow is not None:
        flow_uv = np.clip(flow_uv, 0, clip_flow)
    u, v = flow_uv[:, :, 0], flow_uv[:, :, 1]
    rad_max = np.max(np.sqrt(u * u + v * v))
    eps = 1e-5
    return flow_uv_to_colors(u / (rad_max + eps), v / (rad_max + eps), convert_to_bgr)
