"""Minimal PNG -> RGBA8 decoder for the raytracer's texture assets.

The reference loads its textures with ``sf::Image::loadFromFile`` (SFML 2.4.2,
which decodes through stb_image), e.g. ``textures[0].loadFromFile("Floor.png")``
at /root/reference/Raytracing/SphereWorld.cpp:52.  stb_image expands 8-bit
palette images (+ tRNS alpha) and RGB images to RGBA8 and ignores gAMA/sRGB;
this decoder does the same for the formats the reference's assets use
(colour types 0, 2, 3, 4, 6 at bit depth 8, non-interlaced).  Host-side
asset pipeline only: the kernels consume the decoded RGBA8 bytes.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

_SIG = b"\x89PNG\r\n\x1a\n"
_CHANNELS = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}


def _unfilter(raw: bytes, width: int, height: int, bpp: int) -> np.ndarray:
    stride = width * bpp
    out = np.zeros((height, stride), dtype=np.uint8)
    prev = np.zeros(stride, dtype=np.int32)
    pos = 0
    for y in range(height):
        ftype = raw[pos]
        line = np.frombuffer(raw, dtype=np.uint8, count=stride, offset=pos + 1).astype(np.int32)
        pos += 1 + stride
        cur = np.zeros(stride, dtype=np.int32)
        if ftype == 0:
            cur = line
        elif ftype == 2:
            cur = (line + prev) & 0xFF
        elif ftype in (1, 3, 4):
            # left-dependent filters: sequential over pixels
            for x in range(stride):
                a = cur[x - bpp] if x >= bpp else 0
                b = prev[x]
                c = prev[x - bpp] if x >= bpp else 0
                if ftype == 1:
                    pred = a
                elif ftype == 3:
                    pred = (a + b) >> 1
                else:
                    p = a + b - c
                    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                    pred = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                cur[x] = (line[x] + pred) & 0xFF
        else:
            raise ValueError(f"bad PNG filter type {ftype}")
        out[y] = cur
        prev = cur
    return out


def decode_png_rgba(data: bytes) -> tuple[np.ndarray, int, int]:
    """Decode PNG bytes to (rgba uint8 array [h, w, 4], width, height)."""
    if data[:8] != _SIG:
        raise ValueError("not a PNG file")
    pos = 8
    idat = []
    palette = None
    trns = None
    width = height = depth = ctype = interlace = None
    while pos < len(data):
        (length,) = struct.unpack(">I", data[pos:pos + 4])
        tag = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + length]
        pos += 12 + length
        if tag == b"IHDR":
            width, height, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", body)
        elif tag == b"PLTE":
            palette = np.frombuffer(body, dtype=np.uint8).reshape(-1, 3)
        elif tag == b"tRNS":
            trns = body
        elif tag == b"IDAT":
            idat.append(body)
        elif tag == b"IEND":
            break
    if depth != 8 or interlace != 0 or ctype not in _CHANNELS:
        raise ValueError(f"unsupported PNG (depth={depth}, type={ctype}, interlace={interlace})")
    bpp = _CHANNELS[ctype]
    px = _unfilter(zlib.decompress(b"".join(idat)), width, height, bpp).reshape(height, width, bpp)
    rgba = np.empty((height, width, 4), dtype=np.uint8)
    if ctype == 3:
        if palette is None:
            raise ValueError("palette PNG without PLTE")
        idx = px[..., 0]
        rgba[..., :3] = palette[idx]
        alpha = np.full(256, 255, dtype=np.uint8)
        if trns is not None:
            t = np.frombuffer(trns, dtype=np.uint8)
            alpha[: len(t)] = t
        rgba[..., 3] = alpha[idx]
    elif ctype == 2:
        rgba[..., :3] = px
        rgba[..., 3] = 255
        if trns is not None and len(trns) == 6:
            key = np.array(struct.unpack(">HHH", trns), dtype=np.uint16).astype(np.uint8)
            rgba[..., 3][np.all(px == key, axis=-1)] = 0
    elif ctype == 6:
        rgba[...] = px
    elif ctype == 0:
        rgba[..., :3] = px[..., :1]
        rgba[..., 3] = 255
    elif ctype == 4:
        rgba[..., :3] = px[..., :1]
        rgba[..., 3] = px[..., 1]
    return rgba, width, height


def load_png_rgba(path: str) -> tuple[np.ndarray, int, int]:
    with open(path, "rb") as f:
        return decode_png_rgba(f.read())
