"""TEST INFRASTRUCTURE ONLY (the checker, never the product): a pure-Python restatement of
Image::saveHDR (path_tracer/src/image.cpp:44-49) through the reference's vendored
stb_image_write.h Radiance writer (external/include/stb_image_write.h:246-387) and of the pixels
saveImage hands it (main.cpp:88-112: x-mirrored, accumulated / samples).  Small images only.
Parity note: no reference-written .hdr file exists to pin these bytes; the restatement follows the
vendored source line by line (stbiw__linear_to_rgbe, stbiw__write_hdr_scanline)."""
from __future__ import annotations

import math

import numpy as np


def _rgbe(r: np.float32, g: np.float32, b: np.float32) -> bytes:
    # stbiw__max(a, b) = a > b ? a : b; maxcomp = max(r, max(g, b))
    m = g if g > b else b
    maxcomp = r if r > m else m
    if float(maxcomp) < 1e-32:
        return bytes(4)
    mant, e = math.frexp(float(maxcomp))
    scale = np.float32(np.float32(mant) * np.float32(256.0)) / maxcomp
    return bytes([int(np.float32(r * scale)), int(np.float32(g * scale)), int(np.float32(b * scale)), e + 128])


def _scanline(c: bytes) -> bytes:
    out = bytearray()
    w = len(c)
    x = 0
    while x < w:
        r = x
        while r + 2 < w:
            if c[r] == c[r + 1] and c[r] == c[r + 2]:
                break
            r += 1
        if r + 2 >= w:
            r = w
        while x < r:
            n = min(r - x, 128)
            out += bytes([n]) + c[x:x + n]
            x += n
        if r + 2 < w:
            while r < w and c[r] == c[x]:
                r += 1
            while x < r:
                n = min(r - x, 127)
                out += bytes([n + 128, c[x]])
                x += n
    return bytes(out)


def encode_hdr(image: np.ndarray, samples: float) -> bytes:
    img = np.asarray(image, np.float32)
    H, W = img.shape[0], img.shape[1]
    pix = np.empty_like(img)
    for y in range(H):
        for x in range(W):
            pix[y, W - 1 - x] = img[y, x] / np.float32(samples)
    out = bytearray(b"#?RADIANCE\n# Written by stb_image_write.h\nFORMAT=32-bit_rle_rgbe\n")
    out += f"EXPOSURE=          1.0000000000000\n\n-Y {H} +X {W}\n".encode()
    for y in range(H):
        px = [_rgbe(*pix[y, x]) for x in range(W)]
        if W < 8 or W >= 32768:
            out += b"".join(px)
        else:
            out += bytes([2, 2, (W & 0xff00) >> 8, W & 0xff])
            for k in range(4):
                out += _scanline(bytes(p[k] for p in px))
    return bytes(out)


def decode_hdr(data: bytes) -> np.ndarray:
    """Standard Radiance RLE decoder (new-style scanlines, or flat RGBE when W < 8): (H, W, 3)."""
    head, _, rest = data.partition(b"\n\n")
    dims, _, body = rest.partition(b"\n")
    _, H, _, W = dims.split()
    H, W = int(H), int(W)
    out = np.zeros((H, W, 3), np.float32)
    pos = 0
    for y in range(H):
        if W < 8 or W >= 32768:
            line = np.frombuffer(body[pos:pos + 4 * W], np.uint8).reshape(W, 4)
            pos += 4 * W
        else:
            assert body[pos:pos + 2] == b"\x02\x02"
            pos += 4
            chans = []
            for _k in range(4):
                ch = bytearray()
                while len(ch) < W:
                    n = body[pos]
                    pos += 1
                    if n > 128:
                        ch += bytes([body[pos]]) * (n - 128)
                        pos += 1
                    else:
                        ch += body[pos:pos + n]
                        pos += n
                chans.append(np.frombuffer(bytes(ch), np.uint8))
            line = np.stack(chans, 1)
        e = line[:, 3].astype(np.int32)
        f = np.where(e > 0, np.ldexp(1.0, e - 136), 0.0)
        out[y] = line[:, :3] * f[:, None]
    return out
