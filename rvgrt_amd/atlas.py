"""Texture-atlas loading (reference: src/Texturepack.cu:20-120).

The reference decodes the embedded 256x256 RGBA8 PNG with stb_image
(`stbi_load_from_memory(..., 4)`) and uploads it as float4 = byte/255.  PNG is
lossless, so any conforming decoder yields identical bytes; this is a minimal
decoder for 8-bit, non-interlaced truecolour(+alpha) PNGs, plus a PNG writer
for the offscreen framebuffer dump that replaces the D3D12 present path.
"""
from __future__ import annotations

import hashlib
import os
import struct
import zlib

import numpy as np

ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")
ATLAS_PNG = os.path.join(ASSET_DIR, "texturepack.png")
# sha256 of resources/texturepack.png in the reference snapshot
ATLAS_SHA256 = "bd5ad2a3cac34b73b4ddd3407afa27a003e60624f86c8073b50a78079f3ac807"


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def decode_png(data: bytes) -> np.ndarray:
    """Decode an 8-bit non-interlaced RGB/RGBA PNG to an (H, W, 4) uint8 array."""
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError("not a PNG")
    pos, idat, hdr = 8, [], None
    while pos < len(data):
        (length,) = struct.unpack(">I", data[pos:pos + 4])
        ctype = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + length]
        if ctype == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif ctype == b"IDAT":
            idat.append(body)
        elif ctype == b"IEND":
            break
        pos += 12 + length
    if hdr is None:
        raise ValueError("PNG without IHDR")
    w, h, depth, color, _, _, interlace = hdr
    if depth != 8 or color not in (2, 6) or interlace != 0:
        raise ValueError(f"unsupported PNG format depth={depth} color={color} il={interlace}")
    bpp = 4 if color == 6 else 3
    raw = zlib.decompress(b"".join(idat))
    stride = w * bpp
    out = np.zeros((h, stride), np.uint8)
    prev = np.zeros(stride, np.int32)
    for y in range(h):
        ft = raw[y * (stride + 1)]
        line = np.frombuffer(raw, np.uint8, stride, y * (stride + 1) + 1).astype(np.int32)
        cur = np.zeros(stride, np.int32)
        if ft == 0:
            cur[:] = line
        elif ft == 2:
            cur[:] = (line + prev) & 255
        elif ft in (1, 3, 4):
            for i in range(stride):
                a = cur[i - bpp] if i >= bpp else 0
                b = prev[i]
                c = prev[i - bpp] if i >= bpp else 0
                if ft == 1:
                    p = a
                elif ft == 3:
                    p = (a + b) >> 1
                else:
                    p = _paeth(a, b, c)
                cur[i] = (line[i] + p) & 255
        else:
            raise ValueError(f"bad PNG filter {ft}")
        out[y] = cur
        prev = cur
    img = out.reshape(h, w, bpp)
    if bpp == 3:
        img = np.concatenate([img, np.full((h, w, 1), 255, np.uint8)], axis=2)
    return np.ascontiguousarray(img)


_ATLAS_CACHE = None


def load_atlas() -> np.ndarray:
    """The reference texture atlas as a (256, 256, 4) uint8 array (row 0 = top).
    The asset must be the reference's resources/texturepack.png byte for byte
    (ATLAS_SHA256); a different file raises instead of rendering other pixels."""
    global _ATLAS_CACHE
    if _ATLAS_CACHE is None:
        with open(ATLAS_PNG, "rb") as f:
            data = f.read()
        digest = hashlib.sha256(data).hexdigest()
        if digest != ATLAS_SHA256:
            raise ValueError(f"{ATLAS_PNG}: sha256 {digest} is not the reference atlas {ATLAS_SHA256}")
        _ATLAS_CACHE = decode_png(data)
    return _ATLAS_CACHE


def write_png(path: str, rgba: np.ndarray) -> None:
    """Write an (H, W, 4) uint8 image as a PNG (filter 0, zlib level 6)."""
    rgba = np.ascontiguousarray(rgba, np.uint8)
    h, w, c = rgba.shape
    color = 6 if c == 4 else 2
    raw = b"".join(b"\x00" + rgba[y].tobytes() for y in range(h))

    def chunk(t, body):
        return (struct.pack(">I", len(body)) + t + body +
                struct.pack(">I", zlib.crc32(t + body) & 0xFFFFFFFF))

    png = (b"\x89PNG\r\n\x1a\n" +
           chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, color, 0, 0, 0)) +
           chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))
    with open(path, "wb") as f:
        f.write(png)
