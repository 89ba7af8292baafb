"""Minimal PNG writer for the dataset-reader tests: every colour type and bit
depth, every scanline filter (cycled per row), Adam7 interlacing and IDAT
split into several chunks — the cases an encoder like PIL does not produce."""
import struct
import zlib

import numpy as np

ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]
SPP = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}


def _chunk(t: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + t + data + struct.pack(">I", zlib.crc32(t + data) & 0xFFFFFFFF)


def _pack_row(samples: np.ndarray, bit: int) -> bytes:
    s = samples.astype(np.int64).ravel()
    if bit == 16:
        return b"".join(struct.pack(">H", int(v)) for v in s)
    if bit == 8:
        return bytes(s.astype(np.uint8).tolist())
    per = 8 // bit
    out = bytearray((len(s) + per - 1) // per)
    for k, v in enumerate(s):
        out[k // per] |= int(v) << (8 - bit - (k % per) * bit)
    return bytes(out)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def _filter(row: bytes, prev: bytes, ft: int, bpp: int) -> bytes:
    out = bytearray([ft])
    for i, x in enumerate(row):
        a = row[i - bpp] if i >= bpp else 0
        b = prev[i]
        c = prev[i - bpp] if i >= bpp else 0
        pred = [0, a, b, (a + b) >> 1, _paeth(a, b, c)][ft]
        out.append((x - pred) & 0xFF)
    return bytes(out)


def write_png(path, img: np.ndarray, bit: int, ctype: int, interlace=False, palette=None, idat_parts=3):
    """img: (H, W) or (H, W, spp) samples (palette: indices)."""
    img = np.asarray(img)
    if img.ndim == 2:
        img = img[:, :, None]
    h, w, spp = img.shape
    assert spp == SPP[ctype]
    bpp = max(1, spp * bit // 8)
    raw = bytearray()
    passes = ADAM7 if interlace else [(0, 0, 1, 1)]
    ft = 0
    for x0, y0, dx, dy in passes:
        sub = img[y0::dy, x0::dx]
        if sub.shape[0] == 0 or sub.shape[1] == 0:
            continue
        prev = bytes(len(_pack_row(sub[0], bit)))
        for r in range(sub.shape[0]):
            row = _pack_row(sub[r], bit)
            raw += _filter(row, prev, ft % 5, bpp)
            ft += 1
            prev = row
    comp = zlib.compress(bytes(raw), 6)
    parts = [comp[i * len(comp) // idat_parts:(i + 1) * len(comp) // idat_parts] for i in range(idat_parts)]
    out = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, bit, ctype, 0, 0, int(interlace)))
    out += _chunk(b"tEXt", b"Comment\x00kfx test")  # ancillary chunk: skipped
    if palette is not None:
        out += _chunk(b"PLTE", bytes(np.asarray(palette, np.uint8).ravel().tolist()))
    for p in parts:
        out += _chunk(b"IDAT", p)
    out += _chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(out)


def opencv_color(img: np.ndarray, bit: int, ctype: int, palette=None) -> np.ndarray:
    """What imread(IMREAD_COLOR) returns for this PNG: (H, W, 3) uint8 BGR."""
    img = np.asarray(img)
    if img.ndim == 2:
        img = img[:, :, None]
    if ctype == 3:
        rgb = np.asarray(palette, np.uint8)[img[:, :, 0]]
    else:
        v = img.astype(np.int64)
        if bit == 16:
            v = v >> 8
        elif bit < 8:
            v = v * 255 // ((1 << bit) - 1)
        rgb = np.repeat(v[:, :, :1], 3, axis=2) if ctype in (0, 4) else v[:, :, :3]
    return np.ascontiguousarray(rgb[:, :, ::-1]).astype(np.uint8)
