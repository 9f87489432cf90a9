"""Synthetic optical-flow pairs with exact ground truth.

There is no network access for FlyingChairs/Sintel, so benchmarks and smoke
training use procedurally generated pairs of the same shape: a multi-octave
random texture ``img2`` and a smooth random flow ``f`` (a sum of a global
affine motion and low-frequency noise); ``img1(x) = img2(x + f(x))`` is
obtained by backward warping, so ``f`` is the exact img1 -> img2 flow (the
RAFT convention) wherever ``x + f(x)`` stays inside the frame (``valid``).
Works on CPU and GPU; deterministic for a given ``torch.Generator`` seed.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _smooth_noise(n, c, h, w, scale, gen, device):
    gh, gw = max(2, h // scale), max(2, w // scale)
    base = torch.rand(n, c, gh, gw, generator=gen, device=device) * 2 - 1
    return F.interpolate(base, size=(h, w), mode="bicubic", align_corners=False)


def random_texture(n, h, w, gen=None, device="cpu"):
    img = torch.zeros(n, 3, h, w, device=device)
    amp = 1.0
    for scale in (64, 32, 16, 8, 4, 2):
        img += amp * _smooth_noise(n, 3, h, w, scale, gen, device)
        amp *= 0.6
    img = img - img.amin(dim=(1, 2, 3), keepdim=True)
    img = img / img.amax(dim=(1, 2, 3), keepdim=True).clamp_min(1e-6)
    return img * 255.0


def random_flow(n, h, w, max_disp=20.0, gen=None, device="cpu"):
    ys = torch.linspace(-1, 1, h, device=device)
    xs = torch.linspace(-1, 1, w, device=device)
    gy, gx = torch.meshgrid(ys, xs, indexing="ij")
    coef = (torch.rand(n, 2, 3, generator=gen, device=device) * 2 - 1) * max_disp * 0.5
    affine = coef[:, :, 0, None, None] + coef[:, :, 1, None, None] * gx + coef[:, :, 2, None, None] * gy
    local = _smooth_noise(n, 2, h, w, 32, gen, device) * max_disp * 0.5
    return affine + local


def warp_backward(img, flow):
    """out(x) = img(x + flow(x)), bilinear, border padding."""
    n, _, h, w = img.shape
    ys = torch.arange(h, device=img.device, dtype=img.dtype)
    xs = torch.arange(w, device=img.device, dtype=img.dtype)
    gy, gx = torch.meshgrid(ys, xs, indexing="ij")
    px = gx[None] + flow[:, 0]
    py = gy[None] + flow[:, 1]
    grid = torch.stack([2 * px / (w - 1) - 1, 2 * py / (h - 1) - 1], dim=-1)
    return F.grid_sample(img, grid, mode="bilinear", padding_mode="border", align_corners=True)


def synthetic_batch(n, h, w, max_disp=20.0, seed=0, device="cpu"):
    """Return (image1, image2, flow, valid) with shapes (n,3,h,w) x2, (n,2,h,w), (n,h,w)."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    img2 = random_texture(n, h, w, gen, device)
    flow = random_flow(n, h, w, max_disp, gen, device)
    img1 = warp_backward(img2, flow)
    ys = torch.arange(h, device=device).view(1, h, 1)
    xs = torch.arange(w, device=device).view(1, 1, w)
    tx = xs + flow[:, 0]
    ty = ys + flow[:, 1]
    valid = ((tx >= 0) & (tx <= w - 1) & (ty >= 0) & (ty <= h - 1)).float()
    return img1.clamp(0, 255), img2.clamp(0, 255), flow, valid


class SyntheticFlowDataset(torch.utils.data.Dataset):
    """Map-style dataset of synthetic pairs (CPU tensors, as FlowDataset returns)."""

    def __init__(self, size=(368, 496), length=1000, max_disp=20.0, seed=0):
        self.h, self.w = size
        self.length = length
        self.max_disp = max_disp
        self.seed = seed

    def __len__(self):
        return self.length

    def __getitem__(self, index):
        i1, i2, f, v = synthetic_batch(1, self.h, self.w, self.max_disp, seed=self.seed * 1000003 + index)
        return i1[0], i2[0], f[0], v[0]


def demo_sequence(n_frames: int = 6, h: int = 436, w: int = 1024, seed: int = 16, device="cpu"):
    """A short synthetic video (list of (3, h, w) uint8 frames) for ``demo.py``: a textured
    background under a slow global drift plus a textured disc moving on its own path, so
    consecutive frames have a piecewise-smooth flow with a motion boundary.  Default size is
    the Sintel frame size used by the reference demo."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    bg = random_texture(1, h + 64, w + 64, gen, device)
    fg = random_texture(1, h, w, gen, device) * 0.6 + 60.0
    ys = torch.arange(h, device=device, dtype=torch.float32).view(h, 1)
    xs = torch.arange(w, device=device, dtype=torch.float32).view(1, w)
    frames = []
    for t in range(n_frames):
        ox, oy = 32 + 3.0 * t, 32 + 1.5 * t  # background drift (crop window moves)
        flow_bg = torch.zeros(1, 2, h, w, device=device)
        flow_bg[:, 0], flow_bg[:, 1] = ox - 32, oy - 32
        frame = warp_backward(bg[:, :, 32:32 + h, 32:32 + w], flow_bg)
        cx, cy, r = 0.3 * w + 14.0 * t, 0.55 * h - 6.0 * t, 0.18 * h
        mask = (((xs - cx) ** 2 + (ys - cy) ** 2) <= r * r).float()[None, None]
        flow_fg = torch.zeros(1, 2, h, w, device=device)
        flow_fg[:, 0], flow_fg[:, 1] = -14.0 * t, 6.0 * t
        frame = mask * warp_backward(fg, flow_fg) + (1 - mask) * frame
        frames.append(frame[0].clamp(0, 255).round().to(torch.uint8))
    return frames


_demo_full = demo_sequence  # (tests substitute smaller frames through demo_sequence)


class DeviceSyntheticLoader:
    """``--stage synthetic`` batches generated ON the training device: ``pool`` batches of
    ``batch`` pairs are made once (``synthetic_batch``, seeded by ``seed``) and replayed in a
    per-epoch shuffled order, ``steps`` batches per epoch.  Generating on the CPU in DataLoader
    workers costs ~20 ms per 368x496 pair and capped train.py at ~200 pairs/s on an MI355X
    (profiles/r5a_train_synth.log) -- the synthetic stage is a pipeline / throughput check, so
    its batches come from device memory, as bench.py's do (pairs are what a real stage's
    decode + device augmentation would hand the model)."""

    def __init__(self, batch: int, size, device, pool: int = 8, seed: int = 0, steps: int = 12500):
        h, w = int(size[0]), int(size[1])
        self.pool = [synthetic_batch(batch, h, w, seed=seed * 7919 + i, device=device) for i in range(pool)]
        self.steps = int(steps)
        self.seed = int(seed)
        self.epoch = 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def __len__(self) -> int:
        return self.steps

    def __iter__(self):
        g = torch.Generator()
        g.manual_seed(self.seed + 104729 * self.epoch)
        n = len(self.pool)
        order = torch.randint(0, n, (self.steps,), generator=g).tolist()
        for i in order:
            yield self.pool[i]
