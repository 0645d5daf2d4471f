"""Framebuffer output: the reference's 8-bit encode, PNG and PFM files.

encode_8bit reproduces CVMCTracer/main.cpp:19-29 (and the per-launch PNGs of
CUTracer.cu:383-396): ``cvSet2D(img, y, x, CvScalar(c.z*255, c.y*255,
c.x*255))`` on an IPL_DEPTH_8U image -- the channel is multiplied by 255 in
float (PWVector3f * int), widened to double, and saturate_cast<uchar> rounds
it to nearest, ties to even (cvRound), then clamps to [0, 255].  cvRound on
x86 (cvtsd2si) turns NaN and anything outside int32 -- including +inf --
into INT_MIN, which saturates to 0.
No gamma.  The QuinEngine viewer stores gamma-encoded colour in a UNORM8
render target (rtx.hlsl:402-404): the same rounding applies to its output.

write_png is dependency-free (zlib from the standard library); write_pfm
stores the linear float image (Portable Float Map, bottom-up rows) so
progressive renders can be resumed or compared without 8-bit loss.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np


def encode_8bit(hostcolor: np.ndarray) -> np.ndarray:
    """(H, W, 3) float RGB -> (H, W, 3) uint8 RGB exactly as main.cpp:19-29 writes it."""
    c = np.asarray(hostcolor, np.float32)[..., :3]
    v = (c * np.float32(255)).astype(np.float64)
    with np.errstate(invalid="ignore"):
        ok = np.abs(v) < 2147483648.0           # cvtsd2si range; NaN/inf/huge -> INT_MIN -> 0
        r = np.where(ok, np.rint(np.where(ok, v, 0.0)), 0.0)   # cvRound: nearest, ties to even
    return np.clip(r, 0, 255).astype(np.uint8)


def write_png(path: str, image: np.ndarray) -> None:
    """Write (H, W, 3) uint8 RGB, or float RGB (encoded with encode_8bit), as PNG."""
    img = np.asarray(image)
    if img.dtype != np.uint8:
        img = encode_8bit(img)
    if img.ndim != 3 or img.shape[2] != 3:
        raise ValueError("expected an (H, W, 3) image")
    h, w, _ = img.shape
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))     # filter 0 per row

    def chunk(tag: bytes, data: bytes) -> bytes:
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        f.write(chunk(b"IEND", b""))


def read_png(path: str) -> np.ndarray:
    """Read an 8-bit RGB or RGBA, non-interlaced PNG (as write_png, OpenCV and
    D3DX11SaveTextureToFile write them): (H, W, 3) or (H, W, 4) uint8."""
    data = open(path, "rb").read()
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError("not a PNG file")
    pos, idat = 8, b""
    w = h = 0
    nc = 3
    while pos < len(data):
        n, tag = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            w, h, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", body)
            if depth != 8 or ctype not in (2, 6) or interlace:
                raise ValueError("only 8-bit RGB / RGBA non-interlaced PNGs are supported")
            nc = 3 if ctype == 2 else 4
        elif tag == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + nc * w)
    out = np.zeros((h, nc * w), np.int32)
    prev = np.zeros(nc * w, np.int32)
    for y in range(h):
        ft, line = raw[y, 0], raw[y, 1:].astype(np.int32)
        if ft in (0, 2):                     # none / up: whole row at once
            cur = (line + (prev if ft == 2 else 0)) & 0xFF
            out[y] = cur
            prev = cur
            continue
        cur = np.zeros(nc * w, np.int32)
        if ft == 1:                          # sub: a running sum per channel
            cur = (np.cumsum(line.reshape(w, nc), axis=0) & 0xFF).reshape(-1)
            out[y] = cur
            prev = cur
            continue
        for x in range(nc * w):
            a = cur[x - nc] if x >= nc else 0
            b = prev[x]
            c = prev[x - nc] if x >= nc else 0
            if ft == 3:
                p = (a + b) // 2
            else:
                pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
            cur[x] = (line[x] + p) & 0xFF
        out[y] = cur
        prev = cur
    return out.reshape(h, w, nc).astype(np.uint8)


def write_pfm(path: str, hostcolor: np.ndarray) -> None:
    """Linear float RGB (H, W, 3) as little-endian PFM (rows stored bottom-up)."""
    c = np.ascontiguousarray(np.asarray(hostcolor, np.float32)[..., :3])
    h, w, _ = c.shape
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode())
        f.write(c[::-1].astype("<f4").tobytes())


def read_pfm(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        if f.readline().strip() != b"PF":
            raise ValueError("not an RGB PFM file")
        w, h = (int(x) for x in f.readline().split())
        scale = float(f.readline())
        dt = "<f4" if scale < 0 else ">f4"
        img = np.frombuffer(f.read(w * h * 12), dt).reshape(h, w, 3)
    return np.ascontiguousarray(img[::-1]).astype(np.float32)
