"""Minimal PNG codec for 16-bit (and 8-bit) grayscale / RGB / RGBA images.

KITTI and HD1K store flow as 16-bit RGB PNGs (u, v, valid), which PIL cannot
read or write and OpenCV (what the reference uses, core/utils/frame_utils.py:
102-120) is not available here.  This implements the subset of the PNG spec
those files use: colour types 0/2/4/6, bit depth 8/16, no interlacing, all five
scanline filters on decode, filter 0 on encode.  Pure numpy + zlib.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

_SIG = b"\x89PNG\r\n\x1a\n"
_CHANNELS = {0: 1, 2: 3, 4: 2, 6: 4}


def _chunks(data: bytes):
    pos = len(_SIG)
    while pos < len(data):
        (length,) = struct.unpack(">I", data[pos:pos + 4])
        ctype = data[pos + 4:pos + 8]
        yield ctype, data[pos + 8:pos + 8 + length]
        pos += 12 + length


def _unfilter(raw: np.ndarray, h: int, stride: int, bpp: int) -> np.ndarray:
    out = np.zeros((h, stride), dtype=np.uint8)
    prev = np.zeros(stride, dtype=np.int32)
    rows = raw.reshape(h, stride + 1)
    for y in range(h):
        ftype = rows[y, 0]
        line = rows[y, 1:].astype(np.int32)
        if ftype == 0:
            cur = line
        elif ftype == 2:
            cur = (line + prev) & 0xFF
        elif ftype in (1, 3, 4):
            cur = np.zeros(stride, dtype=np.int32)
            # left neighbours depend on already-decoded bytes: process one bpp-group column at a time
            for x in range(0, stride, bpp):
                sl = slice(x, x + bpp)
                left = cur[x - bpp:x] if x >= bpp else np.zeros(bpp, dtype=np.int32)
                if ftype == 1:
                    cur[sl] = (line[sl] + left) & 0xFF
                elif ftype == 3:
                    cur[sl] = (line[sl] + ((left + prev[sl]) >> 1)) & 0xFF
                else:
                    up = prev[sl]
                    ul = prev[x - bpp:x] if x >= bpp else np.zeros(bpp, dtype=np.int32)
                    p = left + up - ul
                    pa, pb, pc = np.abs(p - left), np.abs(p - up), np.abs(p - ul)
                    pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, up, ul))
                    cur[sl] = (line[sl] + pred) & 0xFF
        else:
            raise ValueError(f"bad PNG filter type {ftype}")
        out[y] = cur
        prev = cur
    return out


def read_png(path: str) -> np.ndarray:
    """Decode a PNG to (H, W) or (H, W, C) uint8 / uint16."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:8] != _SIG:
        raise ValueError(f"{path}: not a PNG file")
    idat = []
    w = h = depth = ctype = None
    for kind, body in _chunks(data):
        if kind == b"IHDR":
            w, h, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", body)
            if interlace:
                raise NotImplementedError("interlaced PNG")
            if ctype not in _CHANNELS or depth not in (8, 16):
                raise NotImplementedError(f"PNG colour type {ctype} depth {depth}")
        elif kind == b"IDAT":
            idat.append(body)
        elif kind == b"IEND":
            break
    ch = _CHANNELS[ctype]
    bpp = ch * depth // 8
    stride = w * bpp
    raw = np.frombuffer(zlib.decompress(b"".join(idat)), dtype=np.uint8)
    img = _unfilter(raw, h, stride, bpp)
    if depth == 16:
        img = img.reshape(h, w * ch, 2)
        img = (img[..., 0].astype(np.uint16) << 8) | img[..., 1].astype(np.uint16)
    img = img.reshape(h, w, ch)
    return img[..., 0] if ch == 1 else img


def write_png(path: str, img: np.ndarray) -> None:
    """Encode uint8 / uint16 (H, W) or (H, W, 1|2|3|4) to PNG (filter 0)."""
    img = np.asarray(img)
    if img.ndim == 2:
        img = img[..., None]
    h, w, ch = img.shape
    ctype = {1: 0, 2: 4, 3: 2, 4: 6}[ch]
    if img.dtype == np.uint16:
        depth = 16
        body = img.astype(">u2").tobytes()
    elif img.dtype == np.uint8:
        depth = 8
        body = img.tobytes()
    else:
        raise TypeError(f"unsupported dtype {img.dtype}")
    stride = len(body) // h
    rows = np.frombuffer(body, dtype=np.uint8).reshape(h, stride)
    raw = np.concatenate([np.zeros((h, 1), dtype=np.uint8), rows], axis=1).tobytes()

    def chunk(kind: bytes, payload: bytes) -> bytes:
        return struct.pack(">I", len(payload)) + kind + payload + struct.pack(">I", zlib.crc32(kind + payload) & 0xFFFFFFFF)

    out = _SIG + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0))
    out += chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(out)
