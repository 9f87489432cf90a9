"""Batched, device-side training augmentation for optical flow.

The reference augments one sample at a time on the CPU, inside DataLoader
workers, with OpenCV and torchvision (core/utils/augmentor.py:15-246).  Here
the workers only decode files; a whole padded batch is augmented on the GPU
(or on the CPU for tests / single samples) with a handful of tensor ops:

* photometric: ColorJitter with the PIL semantics of torchvision (random order
  of brightness / contrast / saturation / hue, each result rounded to uint8),
  symmetric on the stacked pair or (dense, p=0.2) asymmetric per image;
* occlusion eraser: p=0.5, 1-2 boxes of [50, 100) px in image 2 filled with its
  mean colour;
* spatial: ONE bilinear ``grid_sample`` per batch performs cv2.INTER_LINEAR
  resize (log-uniform scale, stretch), horizontal/vertical flips and the random
  crop at once -- every output pixel is mapped straight back to the source;
  sparse (KITTI / HD1K) flow is resized by scattering each valid sample to its
  rounded new position, with the reference's margin crop.

Per-dataset parameters (``AugSpec``) are per sample, so one batch may mix the
dense and sparse datasets of a stage mixture.  All constants are the
reference's (core/utils/augmentor.py): see ``AugSpec`` and ``DENSE`` / ``SPARSE``.
Randomness comes from one ``torch.Generator`` per augmentor (seeded per rank).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F


@dataclass(frozen=True)
class AugSpec:
    """Augmentation parameters of one dataset in a stage mixture."""

    crop_size: Tuple[int, int]
    min_scale: float = -0.2
    max_scale: float = 0.5
    do_flip: bool = True
    sparse: bool = False


# constants of the reference augmentors (dense: FlowAugmentor, sparse: SparseFlowAugmentor)
DENSE = dict(jitter=(0.4, 0.4, 0.4, 0.5 / 3.14), asym_prob=0.2, eraser_prob=0.5, eraser_box=(50, 100),
             spatial_prob=0.8, stretch_prob=0.8, max_stretch=0.2, hflip_prob=0.5, vflip_prob=0.1, crop_pad=8)
SPARSE = dict(jitter=(0.3, 0.3, 0.3, 0.3 / 3.14), asym_prob=0.0, eraser_prob=0.5, eraser_box=(50, 100),
              spatial_prob=0.8, stretch_prob=0.0, max_stretch=0.0, hflip_prob=0.5, vflip_prob=0.0, crop_pad=1,
              margin=(20, 50))


def _u(gen, n, lo, hi, device):
    return torch.rand(n, generator=gen, device=device) * (hi - lo) + lo


def _randint(gen, lo, hi, device):
    """Per-element integer in [lo, hi) for tensors lo, hi (hi > lo)."""
    r = torch.rand(lo.shape, generator=gen, device=device, dtype=torch.float64)
    return (lo + torch.floor(r * (hi - lo).double()).long()).clamp(max=hi - 1)


# ----------------------------------------------------------------------------- photometric
def _q8(x):
    """PIL keeps uint8 images between enhancements."""
    return x.round().clamp_(0, 255)


def _gray(img):
    # PIL "L" conversion: ITU-R 601-2 luma, L = R*299/1000 + G*587/1000 + B*114/1000
    return (img[:, 0] * 0.299 + img[:, 1] * 0.587 + img[:, 2] * 0.114)[:, None]


def _rgb_to_hsv(img):
    r, g, b = img[:, 0], img[:, 1], img[:, 2]
    mx, _ = img.max(1)
    mn, _ = img.min(1)
    d = mx - mn
    s = torch.where(mx > 0, d / mx.clamp_min(1e-8), torch.zeros_like(mx))
    dd = d.clamp_min(1e-8)
    h = torch.where(mx == r, (g - b) / dd, torch.where(mx == g, 2.0 + (b - r) / dd, 4.0 + (r - g) / dd))
    h = torch.where(d > 0, (h / 6.0) % 1.0, torch.zeros_like(h))
    return h, s, mx


def _hsv_to_rgb(h, s, v):
    i = torch.floor(h * 6.0)
    f = h * 6.0 - i
    p, q, t = v * (1 - s), v * (1 - s * f), v * (1 - s * (1 - f))
    i = i.long() % 6
    r = torch.stack([v, q, p, p, t, v], 0).gather(0, i[None])[0]
    g = torch.stack([t, v, v, q, p, p], 0).gather(0, i[None])[0]
    b = torch.stack([p, p, t, v, v, q], 0).gather(0, i[None])[0]
    return torch.stack([r, g, b], 1)


def _masked_mean(x, mask):
    """Mean of (B, C, H, W) over the valid region mask (B, 1, H, W)."""
    return (x * mask).sum((2, 3), keepdim=True) / mask.sum((2, 3), keepdim=True).clamp_min(1)


def color_jitter(img: torch.Tensor, mask: torch.Tensor, factors: torch.Tensor, order: torch.Tensor) -> torch.Tensor:
    """torchvision ColorJitter (PIL backend) on a batch.

    img (B, 3, H, W) float in [0, 255]; mask (B, 1, H, W) valid region (means are over
    it); factors (B, 4) = (brightness, contrast, saturation, hue shift); order (B, 4) a
    permutation of 0..3 per sample.
    """
    B = img.shape[0]
    for k in range(4):
        op = order[:, k]
        out = img
        f = factors.gather(1, op[:, None])[:, 0].view(B, 1, 1, 1)
        # all four candidates, selected per sample (a batch applies different ops per round)
        bright = _q8(img * f)
        m = torch.floor(_masked_mean(_gray(img), mask) + 0.5)  # PIL: int(mean(L) + 0.5)
        contrast = _q8(m + f * (img - m))
        gray = _q8(_gray(img))
        sat = _q8(gray + f * (img - gray))
        h, s, v = _rgb_to_hsv(img / 255.0)
        h = (h + f.view(B, 1, 1)) % 1.0
        hue = _q8(_hsv_to_rgb(h, s, v) * 255.0)
        sel = op.view(B, 1, 1, 1)
        out = torch.where(sel == 0, bright, torch.where(sel == 1, contrast, torch.where(sel == 2, sat, hue)))
        img = out
    return img


# ----------------------------------------------------------------------------- augmentor
class BatchAugmentor:
    """Augment a padded batch of decoded samples (see ``collate_padded``) to fixed crops.

    ``specs``: the mixture's AugSpecs (indexed by each sample's ``spec`` id); every spec
    shares ``crop_size``.  ``__call__(batch) -> (img1, img2, flow, valid)`` float32 on the
    batch's device: images (B, 3, ch, cw) in [0, 255], flow (B, 2, ch, cw), valid (B, ch, cw).
    """

    def __init__(self, specs: Sequence[AugSpec], seed: int = 0, device="cpu"):
        self.specs = list(specs)
        crops = {tuple(s.crop_size) for s in self.specs}
        assert len(crops) == 1, f"one crop size per mixture, got {crops}"
        self.crop = crops.pop()
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed))

    def _params(self, spec_ids: torch.Tensor) -> Dict[str, torch.Tensor]:
        dev = spec_ids.device
        cols = {}
        for key in ("min_scale", "max_scale"):
            cols[key] = torch.tensor([getattr(s, key) for s in self.specs], device=dev)[spec_ids]
        for key in ("do_flip", "sparse"):
            cols[key] = torch.tensor([getattr(s, key) for s in self.specs], device=dev)[spec_ids]
        for key in ("asym_prob", "eraser_prob", "spatial_prob", "stretch_prob", "max_stretch", "hflip_prob",
                    "vflip_prob", "crop_pad"):
            vals = [(SPARSE if s.sparse else DENSE)[key] for s in self.specs]
            cols[key] = torch.tensor(vals, device=dev, dtype=torch.float32)[spec_ids]
        jit = torch.tensor([(SPARSE if s.sparse else DENSE)["jitter"] for s in self.specs], device=dev)
        cols["jitter"] = jit[spec_ids]
        return cols

    def _factors(self, jitter: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        B, dev = jitter.shape[0], jitter.device
        lo = torch.cat([(1 - jitter[:, :3]).clamp_min(0), -jitter[:, 3:]], 1)
        hi = torch.cat([1 + jitter[:, :3], jitter[:, 3:]], 1)
        f = lo + torch.rand(B, 4, generator=self.gen, device=dev) * (hi - lo)
        order = torch.argsort(torch.rand(B, 4, generator=self.gen, device=dev), dim=1)
        return f, order

    @torch.no_grad()
    def __call__(self, batch: Dict[str, torch.Tensor]):
        img1 = batch["img1"].to(self.device, non_blocking=True).permute(0, 3, 1, 2).float()
        img2 = batch["img2"].to(self.device, non_blocking=True).permute(0, 3, 1, 2).float()
        flow = batch["flow"].to(self.device, non_blocking=True).permute(0, 3, 1, 2).float()
        valid = batch["valid"].to(self.device, non_blocking=True).float()
        sizes = batch["size"].to(self.device)
        spec = batch["spec"].to(self.device)
        B, _, Hm, Wm = img1.shape
        dev = img1.device
        gen = self.gen
        p = self._params(spec)
        hs, ws = sizes[:, 0], sizes[:, 1]
        yy = torch.arange(Hm, device=dev).view(1, 1, Hm, 1)
        xx = torch.arange(Wm, device=dev).view(1, 1, 1, Wm)
        region = ((yy < hs.view(B, 1, 1, 1)) & (xx < ws.view(B, 1, 1, 1))).float()

        # ---- photometric: asymmetric per image (p) or symmetric on the stacked pair
        asym = torch.rand(B, generator=gen, device=dev) < p["asym_prob"]
        f1, o1 = self._factors(p["jitter"])
        f2, o2 = self._factors(p["jitter"])
        f2 = torch.where(asym[:, None], f2, f1)
        o2 = torch.where(asym[:, None], o2, o1)
        # symmetric: PIL sees img1 stacked over img2, so the contrast mean spans both images
        pair = torch.cat([img1, img2], 2)
        pmask = torch.cat([region, region], 2)
        sym = color_jitter(pair, pmask, f1, o1)
        a1 = color_jitter(img1, region, f1, o1)
        a2 = color_jitter(img2, region, f2, o2)
        am = asym.view(B, 1, 1, 1)
        img1 = torch.where(am, a1, sym[:, :, :Hm])
        img2 = torch.where(am, a2, sym[:, :, Hm:])

        # ---- eraser: 1-2 boxes in image 2 filled with its mean colour (uint8 truncation)
        erase = torch.rand(B, generator=gen, device=dev) < p["eraser_prob"]
        nbox = 1 + (torch.rand(B, generator=gen, device=dev) < 0.5).long()
        mean = torch.floor(_masked_mean(img2, region))
        emask = torch.zeros(B, 1, Hm, Wm, device=dev, dtype=torch.bool)
        for k in range(2):
            x0 = _randint(gen, torch.zeros_like(ws), ws, dev)
            y0 = _randint(gen, torch.zeros_like(hs), hs, dev)
            dx = _randint(gen, torch.full_like(ws, 50), torch.full_like(ws, 100), dev)
            dy = _randint(gen, torch.full_like(hs, 50), torch.full_like(hs, 100), dev)
            box = ((xx >= x0.view(B, 1, 1, 1)) & (xx < (x0 + dx).view(B, 1, 1, 1)) &
                   (yy >= y0.view(B, 1, 1, 1)) & (yy < (y0 + dy).view(B, 1, 1, 1)))
            on = (erase & (nbox > k)).view(B, 1, 1, 1)
            emask |= box & on
        img2 = torch.where(emask & (region > 0), mean, img2)

        # ---- spatial parameters
        ch, cw = self.crop
        hf, wf = hs.float(), ws.float()
        floor = torch.maximum((ch + p["crop_pad"]) / hf, (cw + p["crop_pad"]) / wf)
        scale = torch.pow(2.0, _u(gen, B, 0, 1, dev) * (p["max_scale"] - p["min_scale"]) + p["min_scale"])
        stretch = torch.rand(B, generator=gen, device=dev) < p["stretch_prob"]
        ms = p["max_stretch"]
        sx = scale * torch.where(stretch, torch.pow(2.0, _u(gen, B, 0, 1, dev) * 2 * ms - ms), torch.ones_like(scale))
        sy = scale * torch.where(stretch, torch.pow(2.0, _u(gen, B, 0, 1, dev) * 2 * ms - ms), torch.ones_like(scale))
        sx, sy = torch.maximum(sx, floor), torch.maximum(sy, floor)
        resize = torch.rand(B, generator=gen, device=dev) < p["spatial_prob"]
        sx = torch.where(resize, sx, torch.ones_like(sx))
        sy = torch.where(resize, sy, torch.ones_like(sy))
        rh = torch.where(resize, torch.round(hf * sy), hf).long()  # cv2: round(size * f)
        rw = torch.where(resize, torch.round(wf * sx), wf).long()
        hflip = p["do_flip"] & (torch.rand(B, generator=gen, device=dev) < p["hflip_prob"])
        vflip = p["do_flip"] & (torch.rand(B, generator=gen, device=dev) < p["vflip_prob"])
        sparse = p["sparse"]
        # crops: dense y0 ~ U[0, rh - ch), sparse with margins (20, 50) then clipped
        my = torch.where(sparse, torch.full_like(rh, 20), torch.zeros_like(rh))
        mx = torch.where(sparse, torch.full_like(rw, 50), torch.zeros_like(rw))
        y0 = _randint(gen, torch.zeros_like(rh), (rh - ch + my).clamp_min(1), dev)
        x0 = _randint(gen, -mx, (rw - cw + mx).clamp_min(1 - mx), dev)
        y0 = torch.minimum(y0.clamp_min(0), (rh - ch).clamp_min(0))
        x0 = torch.minimum(x0.clamp_min(0), (rw - cw).clamp_min(0))

        # ---- one warp: crop pixel -> resized (flipped) pixel -> source (cv2 half-pixel centres)
        v = torch.arange(ch, device=dev).view(1, ch, 1).float()
        u = torch.arange(cw, device=dev).view(1, 1, cw).float()
        xr = (x0.view(B, 1, 1).float() + u).expand(B, ch, cw)
        yr = (y0.view(B, 1, 1).float() + v).expand(B, ch, cw)
        xr = torch.where(hflip.view(B, 1, 1), rw.view(B, 1, 1).float() - 1 - xr, xr)
        yr = torch.where(vflip.view(B, 1, 1), rh.view(B, 1, 1).float() - 1 - yr, yr)
        xs = ((xr + 0.5) / sx.view(B, 1, 1) - 0.5).clamp(min=0).minimum(wf.view(B, 1, 1) - 1)
        ys = ((yr + 0.5) / sy.view(B, 1, 1) - 0.5).clamp(min=0).minimum(hf.view(B, 1, 1) - 1)
        grid = torch.stack([(2 * xs + 1) / Wm - 1, (2 * ys + 1) / Hm - 1], -1)
        src = torch.cat([img1, img2, flow], 1)
        out = F.grid_sample(src, grid, mode="bilinear", padding_mode="border", align_corners=False)
        o1, o2, of = _q8(out[:, :3]), _q8(out[:, 3:6]), out[:, 6:8]
        of = of * torch.stack([sx, sy], 1).view(B, 2, 1, 1)
        of = of * torch.stack([torch.where(hflip, -1.0, 1.0), torch.where(vflip, -1.0, 1.0)], 1).view(B, 2, 1, 1)
        dvalid = ((of[:, 0].abs() < 1000) & (of[:, 1].abs() < 1000)).float()

        if bool(sparse.any()):
            sf, sv = self._sparse_flow(flow, valid, sx, sy, resize, hflip, x0, y0, rh, rw, Hm, Wm)
            sm = sparse.view(B, 1, 1, 1)
            of = torch.where(sm, sf, of)
            dvalid = torch.where(sparse.view(B, 1, 1), sv, dvalid)
        return o1, o2, of, dvalid

    def _sparse_flow(self, flow, valid, sx, sy, resize, hflip, x0, y0, rh, rw, Hm, Wm):
        """Reference ``resize_sparse_flow_map`` + flip + crop: every valid source sample is
        scattered to its rounded position in the resized map (strictly inside, as the
        reference keeps ``0 < x < w1``), then flipped and cropped."""
        B, dev = flow.shape[0], flow.device
        ch, cw = self.crop
        ys, xs = torch.meshgrid(torch.arange(Hm, device=dev), torch.arange(Wm, device=dev), indexing="ij")
        xs = xs[None].float().expand(B, -1, -1)
        ys = ys[None].float().expand(B, -1, -1)
        rs = resize.view(B, 1, 1)
        xn = torch.where(rs, torch.round(xs * sx.view(B, 1, 1)), xs).long()
        yn = torch.where(rs, torch.round(ys * sy.view(B, 1, 1)), ys).long()
        inside = torch.where(rs, (xn > 0) & (yn > 0) & (xn < rw.view(B, 1, 1)) & (yn < rh.view(B, 1, 1)),
                             torch.ones_like(xn, dtype=torch.bool))
        fv = flow * torch.where(resize.view(B, 1, 1, 1), torch.stack([sx, sy], 1).view(B, 2, 1, 1),
                                torch.ones(B, 2, 1, 1, device=dev))
        xn = torch.where(hflip.view(B, 1, 1), rw.view(B, 1, 1) - 1 - xn, xn)
        fv = fv * torch.stack([torch.where(hflip, -1.0, 1.0), torch.ones_like(sx)], 1).view(B, 2, 1, 1)
        cx, cy = xn - x0.view(B, 1, 1), yn - y0.view(B, 1, 1)
        keep = (valid >= 1) & inside & (cx >= 0) & (cx < cw) & (cy >= 0) & (cy < ch)
        b = torch.arange(B, device=dev).view(B, 1, 1).expand_as(cx)
        idx = ((b * ch + cy) * cw + cx)[keep]
        # below scale 1 several samples round onto one target pixel; the reference's numpy
        # assignment keeps the LAST one in row-major source order, so keep the largest source
        # index per target explicitly (a plain indexed write leaves the winner unspecified on
        # the GPU)
        src = (ys * Wm + xs).long()[keep]
        win = torch.full((B * ch * cw,), -1, device=dev, dtype=torch.long).scatter_reduce(0, idx, src, "amax")
        last = win[idx] == src
        out_f = torch.zeros(B * ch * cw, 2, device=dev)
        out_v = torch.zeros(B * ch * cw, device=dev)
        out_f[idx[last]] = fv.permute(0, 2, 3, 1)[keep][last]
        out_v[idx] = 1.0
        return out_f.view(B, ch, cw, 2).permute(0, 3, 1, 2), out_v.view(B, ch, cw)


def collate_padded(samples: List[Dict[str, torch.Tensor]]) -> Dict[str, torch.Tensor]:
    """Stack decoded samples of different sizes into one zero-padded batch (uint8 images)."""
    Hm = max(s["img1"].shape[0] for s in samples)
    Wm = max(s["img1"].shape[1] for s in samples)
    B = len(samples)
    out = {
        "img1": torch.zeros(B, Hm, Wm, 3, dtype=torch.uint8),
        "img2": torch.zeros(B, Hm, Wm, 3, dtype=torch.uint8),
        "flow": torch.zeros(B, Hm, Wm, 2, dtype=torch.float32),
        "valid": torch.zeros(B, Hm, Wm, dtype=torch.float32),
        "size": torch.zeros(B, 2, dtype=torch.long),
        "spec": torch.zeros(B, dtype=torch.long),
    }
    for i, s in enumerate(samples):
        h, w = s["img1"].shape[:2]
        for k in ("img1", "img2", "flow", "valid"):
            out[k][i, :h, :w] = s[k]
        out["size"][i, 0], out["size"][i, 1] = h, w
        out["spec"][i] = int(s["spec"])
    return out


def augment_one(sample: Dict[str, torch.Tensor], spec: AugSpec, gen_seed: Optional[int] = None):
    """Augment a single decoded sample on the CPU (the reference's per-item API)."""
    seed = int(torch.randint(0, 2**31 - 1, (1,)).item()) if gen_seed is None else gen_seed
    aug = BatchAugmentor([spec], seed=seed)
    s = dict(sample)
    s["spec"] = 0
    i1, i2, f, v = aug(collate_padded([s]))
    return i1[0], i2[0], f[0], v[0]


# ----------------------------------------------------------------------------- per-item API
class FlowAugmentor:
    """Reference-style per-sample augmentor (numpy HWC in/out) on top of ``BatchAugmentor``."""

    sparse = False

    def __init__(self, crop_size, min_scale=-0.2, max_scale=0.5, do_flip=True, seed: Optional[int] = None):
        self.spec = AugSpec(tuple(crop_size), min_scale, max_scale, do_flip, self.sparse)
        seed = int(torch.randint(0, 2**31 - 1, (1,)).item()) if seed is None else seed
        self.aug = BatchAugmentor([self.spec], seed=seed)

    def _run(self, img1, img2, flow, valid):
        h, w = img1.shape[:2]
        s = {"img1": torch.as_tensor(np.ascontiguousarray(img1)), "img2": torch.as_tensor(np.ascontiguousarray(img2)),
             "flow": torch.as_tensor(np.ascontiguousarray(flow, dtype=np.float32)),
             "valid": torch.as_tensor(np.ascontiguousarray(valid, dtype=np.float32)), "spec": 0}
        i1, i2, f, v = self.aug(collate_padded([s]))
        hwc = lambda t: t[0].permute(1, 2, 0).numpy()  # noqa: E731
        return hwc(i1).astype(np.uint8), hwc(i2).astype(np.uint8), hwc(f).astype(np.float32), v[0].numpy()

    def __call__(self, img1, img2, flow):
        valid = (np.abs(flow[..., 0]) < 1000) & (np.abs(flow[..., 1]) < 1000)
        return self._run(img1, img2, flow, valid)[:3]


class SparseFlowAugmentor(FlowAugmentor):
    sparse = True

    def __init__(self, crop_size, min_scale=-0.2, max_scale=0.5, do_flip=False, seed: Optional[int] = None):
        super().__init__(crop_size, min_scale, max_scale, do_flip, seed)

    def __call__(self, img1, img2, flow, valid):
        return self._run(img1, img2, flow, valid)
