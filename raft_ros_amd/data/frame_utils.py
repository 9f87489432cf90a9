"""Flow / image file I/O (reference core/utils/frame_utils.py).

* Middlebury ``.flo``: float32 magic 202021.25, int32 width, int32 height, then
  interleaved (u, v) float32 rows.  ``readFlow`` raises on a bad magic number
  (the reference prints and returns None, which crashes later).
* ``.pfm`` (FlyingThings3D): header 'PF'/'Pf', scale sign = endianness, rows
  stored bottom-up; 3-channel flow files drop the third channel in ``read_gen``.
* KITTI 16-bit PNG flow: (u, v) = (value - 2^15) / 64, valid flag in channel 3;
  KITTI disparity: value / 256.
* ``read_gen`` dispatches on the extension like the reference.
"""
from __future__ import annotations

import re
from os.path import splitext

import numpy as np
from PIL import Image

from .png16 import read_png, write_png

TAG_FLOAT = 202021.25
TAG_CHAR = np.array([TAG_FLOAT], np.float32)


def readFlow(fn: str) -> np.ndarray:
    """Read a Middlebury .flo file -> (H, W, 2) float32."""
    with open(fn, "rb") as f:
        magic = np.fromfile(f, np.float32, count=1)
        if magic.size != 1 or magic[0] != TAG_FLOAT:
            raise ValueError(f"{fn}: invalid .flo magic number")
        w = int(np.fromfile(f, np.int32, count=1)[0])
        h = int(np.fromfile(f, np.int32, count=1)[0])
        data = np.fromfile(f, np.float32, count=2 * w * h)
    if data.size != 2 * w * h:
        raise ValueError(f"{fn}: truncated .flo file")
    return data.reshape(h, w, 2)


def writeFlow(filename: str, uv: np.ndarray, v: np.ndarray | None = None) -> None:
    """Write (H, W, 2) flow (or separate u, v) as a Middlebury .flo file."""
    if v is None:
        assert uv.ndim == 3 and uv.shape[2] == 2
        u, v = uv[:, :, 0], uv[:, :, 1]
    else:
        u = uv
    assert u.shape == v.shape
    h, w = u.shape
    with open(filename, "wb") as f:
        f.write(TAG_CHAR.tobytes())
        np.array([w, h], dtype=np.int32).tofile(f)
        np.stack([u, v], axis=-1).astype(np.float32).tofile(f)


def readPFM(file: str) -> np.ndarray:
    with open(file, "rb") as f:
        header = f.readline().rstrip()
        if header == b"PF":
            color = True
        elif header == b"Pf":
            color = False
        else:
            raise ValueError("Not a PFM file.")
        m = re.match(rb"^(\d+)\s(\d+)\s$", f.readline())
        if not m:
            raise ValueError("Malformed PFM header.")
        width, height = map(int, m.groups())
        scale = float(f.readline().rstrip())
        endian = "<" if scale < 0 else ">"
        data = np.fromfile(f, endian + "f")
    shape = (height, width, 3) if color else (height, width)
    return np.flipud(data.reshape(shape))


def writePFM(file: str, image: np.ndarray, scale: float = 1.0) -> None:
    image = np.asarray(image, dtype=np.float32)
    color = image.ndim == 3 and image.shape[2] == 3
    if not (color or image.ndim == 2 or (image.ndim == 3 and image.shape[2] == 1)):
        raise ValueError("PFM images are HxW or HxWx3")
    with open(file, "wb") as f:
        f.write(b"PF\n" if color else b"Pf\n")
        f.write(f"{image.shape[1]} {image.shape[0]}\n".encode())
        f.write(f"{-abs(scale)}\n".encode())  # little endian
        np.flipud(image).astype("<f4").tofile(f)


def readFlowKITTI(filename: str):
    """-> (flow (H, W, 2) float32, valid (H, W) float32)."""
    img = read_png(filename).astype(np.float32)
    flow, valid = img[:, :, :2], img[:, :, 2]
    return (flow - 2 ** 15) / 64.0, valid


def readDispKITTI(filename: str):
    disp = read_png(filename).astype(np.float32) / 256.0
    valid = disp > 0.0
    flow = np.stack([-disp, np.zeros_like(disp)], -1)
    return flow, valid


def writeFlowKITTI(filename: str, uv: np.ndarray) -> None:
    uv = 64.0 * uv + 2 ** 15
    valid = np.ones([uv.shape[0], uv.shape[1], 1])
    img = np.concatenate([uv, valid], axis=-1)
    # truncation like the reference's astype(np.uint16); file channel order (u, v, valid) as RGB
    write_png(filename, np.clip(img, 0, 65535).astype(np.uint16))


def read_gen(file_name: str, pil: bool = False):
    ext = splitext(file_name)[-1].lower()
    if ext in (".png", ".jpeg", ".ppm", ".jpg"):
        return Image.open(file_name)
    if ext in (".bin", ".raw"):
        return np.load(file_name)
    if ext == ".flo":
        return readFlow(file_name).astype(np.float32)
    if ext == ".pfm":
        flow = readPFM(file_name).astype(np.float32)
        return flow if flow.ndim == 2 else flow[:, :, :-1]
    return []
