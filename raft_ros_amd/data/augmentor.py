"""Training-time data augmentation (reference core/utils/augmentor.py:15-246).

The reference depends on OpenCV (resize) and torchvision (ColorJitter), neither
of which exists in this environment; both are re-implemented here with the same
semantics:

* ``ColorJitter`` follows torchvision's PIL path: a random order of brightness
  (ImageEnhance.Brightness), contrast (ImageEnhance.Contrast), saturation
  (ImageEnhance.Color) and hue (shift of the H channel in HSV) with factors drawn
  uniformly from [max(0, 1-x), 1+x] (hue: [-h, h]).
* ``resize_linear`` is cv2.INTER_LINEAR (half-pixel centres, no antialiasing),
  implemented with ``F.interpolate(mode='bilinear', align_corners=False)``; the
  output size is ``round(size * scale)`` like cv2.resize with fx/fy.

Probabilities and constants are those of the reference: asymmetric colour jitter
p=0.2, eraser p=0.5 (1-2 boxes of 50-100 px filled with the mean colour),
spatial scale 2**U(min_scale, max_scale), stretch p=0.8 (2**U(-0.2, 0.2)),
resize p=0.8, h-flip 0.5, v-flip 0.1 (dense only), crops, and the sparse
(KITTI/HD1K) flow-map resize that scatters valid samples.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F
from PIL import Image, ImageEnhance


def resize_linear(img: np.ndarray, fx: float, fy: float) -> np.ndarray:
    """cv2.resize(img, None, fx=fx, fy=fy, interpolation=cv2.INTER_LINEAR) for HxW[xC]."""
    h, w = img.shape[:2]
    nh, nw = int(round(h * fy)), int(round(w * fx))
    squeeze = img.ndim == 2
    arr = img[..., None] if squeeze else img
    t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float32)).permute(2, 0, 1)[None]
    out = F.interpolate(t, size=(nh, nw), mode="bilinear", align_corners=False)[0].permute(1, 2, 0).numpy()
    if img.dtype == np.uint8:
        out = np.clip(np.rint(out), 0, 255).astype(np.uint8)
    else:
        out = out.astype(img.dtype)
    return out[..., 0] if squeeze else out


def _adjust_hue(img: Image.Image, hue_factor: float) -> Image.Image:
    if img.mode in ("L", "1", "I", "F"):
        return img
    h, s, v = img.convert("HSV").split()
    np_h = np.array(h, dtype=np.uint8)
    with np.errstate(over="ignore"):
        np_h = (np_h.astype(np.int16) + int(round(hue_factor * 255))) % 256
    h = Image.fromarray(np_h.astype(np.uint8), "L")
    return Image.merge("HSV", (h, s, v)).convert(img.mode)


class ColorJitter:
    """torchvision.transforms.ColorJitter (PIL backend) without torchvision."""

    def __init__(self, brightness=0.0, contrast=0.0, saturation=0.0, hue=0.0, rng=None):
        self.brightness = (max(0.0, 1 - brightness), 1 + brightness) if brightness else None
        self.contrast = (max(0.0, 1 - contrast), 1 + contrast) if contrast else None
        self.saturation = (max(0.0, 1 - saturation), 1 + saturation) if saturation else None
        self.hue = (-hue, hue) if hue else None

    def __call__(self, img: Image.Image) -> Image.Image:
        order = torch.randperm(4).tolist()
        b = None if self.brightness is None else float(torch.empty(1).uniform_(*self.brightness))
        c = None if self.contrast is None else float(torch.empty(1).uniform_(*self.contrast))
        s = None if self.saturation is None else float(torch.empty(1).uniform_(*self.saturation))
        h = None if self.hue is None else float(torch.empty(1).uniform_(*self.hue))
        for fn in order:
            if fn == 0 and b is not None:
                img = ImageEnhance.Brightness(img).enhance(b)
            elif fn == 1 and c is not None:
                img = ImageEnhance.Contrast(img).enhance(c)
            elif fn == 2 and s is not None:
                img = ImageEnhance.Color(img).enhance(s)
            elif fn == 3 and h is not None:
                img = _adjust_hue(img, h)
        return img


class FlowAugmentor:
    def __init__(self, crop_size, min_scale=-0.2, max_scale=0.5, do_flip=True):
        self.crop_size = crop_size
        self.min_scale = min_scale
        self.max_scale = max_scale
        self.spatial_aug_prob = 0.8
        self.stretch_prob = 0.8
        self.max_stretch = 0.2
        self.do_flip = do_flip
        self.h_flip_prob = 0.5
        self.v_flip_prob = 0.1
        self.photo_aug = ColorJitter(brightness=0.4, contrast=0.4, saturation=0.4, hue=0.5 / 3.14)
        self.asymmetric_color_aug_prob = 0.2
        self.eraser_aug_prob = 0.5

    def color_transform(self, img1, img2):
        if np.random.rand() < self.asymmetric_color_aug_prob:
            img1 = np.array(self.photo_aug(Image.fromarray(img1)), dtype=np.uint8)
            img2 = np.array(self.photo_aug(Image.fromarray(img2)), dtype=np.uint8)
        else:
            stack = np.concatenate([img1, img2], axis=0)
            stack = np.array(self.photo_aug(Image.fromarray(stack)), dtype=np.uint8)
            img1, img2 = np.split(stack, 2, axis=0)
        return img1, img2

    def eraser_transform(self, img1, img2, bounds=(50, 100)):
        ht, wd = img1.shape[:2]
        if np.random.rand() < self.eraser_aug_prob:
            img2 = img2.copy()
            mean_color = np.mean(img2.reshape(-1, 3), axis=0)
            for _ in range(np.random.randint(1, 3)):
                x0 = np.random.randint(0, wd)
                y0 = np.random.randint(0, ht)
                dx = np.random.randint(bounds[0], bounds[1])
                dy = np.random.randint(bounds[0], bounds[1])
                img2[y0:y0 + dy, x0:x0 + dx, :] = mean_color
        return img1, img2

    def spatial_transform(self, img1, img2, flow):
        ht, wd = img1.shape[:2]
        min_scale = np.maximum((self.crop_size[0] + 8) / float(ht), (self.crop_size[1] + 8) / float(wd))
        scale = 2 ** np.random.uniform(self.min_scale, self.max_scale)
        scale_x = scale_y = scale
        if np.random.rand() < self.stretch_prob:
            scale_x *= 2 ** np.random.uniform(-self.max_stretch, self.max_stretch)
            scale_y *= 2 ** np.random.uniform(-self.max_stretch, self.max_stretch)
        scale_x = np.clip(scale_x, min_scale, None)
        scale_y = np.clip(scale_y, min_scale, None)
        if np.random.rand() < self.spatial_aug_prob:
            img1 = resize_linear(img1, scale_x, scale_y)
            img2 = resize_linear(img2, scale_x, scale_y)
            flow = resize_linear(flow, scale_x, scale_y) * np.array([scale_x, scale_y], dtype=np.float32)
        if self.do_flip:
            if np.random.rand() < self.h_flip_prob:
                img1, img2 = img1[:, ::-1], img2[:, ::-1]
                flow = flow[:, ::-1] * np.array([-1.0, 1.0], dtype=np.float32)
            if np.random.rand() < self.v_flip_prob:
                img1, img2 = img1[::-1, :], img2[::-1, :]
                flow = flow[::-1, :] * np.array([1.0, -1.0], dtype=np.float32)
        y0 = np.random.randint(0, img1.shape[0] - self.crop_size[0])
        x0 = np.random.randint(0, img1.shape[1] - self.crop_size[1])
        sl = (slice(y0, y0 + self.crop_size[0]), slice(x0, x0 + self.crop_size[1]))
        return img1[sl], img2[sl], flow[sl]

    def __call__(self, img1, img2, flow):
        img1, img2 = self.color_transform(img1, img2)
        img1, img2 = self.eraser_transform(img1, img2)
        img1, img2, flow = self.spatial_transform(img1, img2, flow)
        return np.ascontiguousarray(img1), np.ascontiguousarray(img2), np.ascontiguousarray(flow, dtype=np.float32)


class SparseFlowAugmentor:
    def __init__(self, crop_size, min_scale=-0.2, max_scale=0.5, do_flip=False):
        self.crop_size = crop_size
        self.min_scale = min_scale
        self.max_scale = max_scale
        self.spatial_aug_prob = 0.8
        self.stretch_prob = 0.8
        self.max_stretch = 0.2
        self.do_flip = do_flip
        self.h_flip_prob = 0.5
        self.v_flip_prob = 0.1
        self.photo_aug = ColorJitter(brightness=0.3, contrast=0.3, saturation=0.3, hue=0.3 / 3.14)
        self.asymmetric_color_aug_prob = 0.2
        self.eraser_aug_prob = 0.5

    def color_transform(self, img1, img2):
        stack = np.concatenate([img1, img2], axis=0)
        stack = np.array(self.photo_aug(Image.fromarray(stack)), dtype=np.uint8)
        return tuple(np.split(stack, 2, axis=0))

    def eraser_transform(self, img1, img2):
        ht, wd = img1.shape[:2]
        if np.random.rand() < self.eraser_aug_prob:
            img2 = img2.copy()
            mean_color = np.mean(img2.reshape(-1, 3), axis=0)
            for _ in range(np.random.randint(1, 3)):
                x0 = np.random.randint(0, wd)
                y0 = np.random.randint(0, ht)
                dx = np.random.randint(50, 100)
                dy = np.random.randint(50, 100)
                img2[y0:y0 + dy, x0:x0 + dx, :] = mean_color
        return img1, img2

    @staticmethod
    def resize_sparse_flow_map(flow, valid, fx=1.0, fy=1.0):
        """Scale a sparse flow map by scattering each valid sample to its rounded new position."""
        ht, wd = flow.shape[:2]
        xs, ys = np.meshgrid(np.arange(wd), np.arange(ht))
        coords = np.stack([xs, ys], axis=-1).reshape(-1, 2).astype(np.float32)
        flow = flow.reshape(-1, 2).astype(np.float32)
        valid = valid.reshape(-1).astype(np.float32)
        coords0, flow0 = coords[valid >= 1], flow[valid >= 1]
        ht1, wd1 = int(round(ht * fy)), int(round(wd * fx))
        coords1 = coords0 * [fx, fy]
        flow1 = flow0 * [fx, fy]
        xx = np.round(coords1[:, 0]).astype(np.int32)
        yy = np.round(coords1[:, 1]).astype(np.int32)
        keep = (xx > 0) & (xx < wd1) & (yy > 0) & (yy < ht1)
        xx, yy, flow1 = xx[keep], yy[keep], flow1[keep]
        flow_img = np.zeros([ht1, wd1, 2], dtype=np.float32)
        valid_img = np.zeros([ht1, wd1], dtype=np.int32)
        flow_img[yy, xx] = flow1
        valid_img[yy, xx] = 1
        return flow_img, valid_img

    def spatial_transform(self, img1, img2, flow, valid):
        ht, wd = img1.shape[:2]
        min_scale = np.maximum((self.crop_size[0] + 1) / float(ht), (self.crop_size[1] + 1) / float(wd))
        scale = 2 ** np.random.uniform(self.min_scale, self.max_scale)
        scale_x = np.clip(scale, min_scale, None)
        scale_y = np.clip(scale, min_scale, None)
        if np.random.rand() < self.spatial_aug_prob:
            img1 = resize_linear(img1, scale_x, scale_y)
            img2 = resize_linear(img2, scale_x, scale_y)
            flow, valid = self.resize_sparse_flow_map(flow, valid, fx=scale_x, fy=scale_y)
        if self.do_flip and np.random.rand() < 0.5:
            img1, img2 = img1[:, ::-1], img2[:, ::-1]
            flow = flow[:, ::-1] * np.array([-1.0, 1.0], dtype=np.float32)
            valid = valid[:, ::-1]
        margin_y, margin_x = 20, 50
        y0 = np.random.randint(0, img1.shape[0] - self.crop_size[0] + margin_y)
        x0 = np.random.randint(-margin_x, img1.shape[1] - self.crop_size[1] + margin_x)
        y0 = np.clip(y0, 0, img1.shape[0] - self.crop_size[0])
        x0 = np.clip(x0, 0, img1.shape[1] - self.crop_size[1])
        sl = (slice(y0, y0 + self.crop_size[0]), slice(x0, x0 + self.crop_size[1]))
        return img1[sl], img2[sl], flow[sl], valid[sl]

    def __call__(self, img1, img2, flow, valid):
        img1, img2 = self.color_transform(img1, img2)
        img1, img2 = self.eraser_transform(img1, img2)
        img1, img2, flow, valid = self.spatial_transform(img1, img2, flow, valid)
        return (np.ascontiguousarray(img1), np.ascontiguousarray(img2), np.ascontiguousarray(flow, dtype=np.float32),
                np.ascontiguousarray(valid))
