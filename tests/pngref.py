"""Test infrastructure: a tiny independent PNG encoder/decoder (zlib + numpy) used to pin
rt_image_load (Surface::LoadImage, template/template.cpp:1579-1601, reading PNGs the way
stb_image's stbi_load(.., req_comp 0) does).  Never imported by the product."""
import struct
import zlib

import numpy as np


def _chunk(t, data):
    return struct.pack(">I", len(data)) + t + data + struct.pack(">I", zlib.crc32(t + data) & 0xffffffff)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)


def encode(samples, ctype, depth, palette=None, trns=None):
    """samples: uint array [h, w, ch] (ch per colour type; palette indices for ctype 3).
    Rows cycle through filter types 0..4 so every filter is exercised."""
    h, w, ch = samples.shape
    rows = []
    prev = None
    for y in range(h):
        if depth >= 8:
            dt = ">u2" if depth == 16 else "u1"
            raw = np.asarray(samples[y], dtype=np.uint32).astype(dt).tobytes()
        else:   # pack sub-byte samples big-endian within the byte
            bits = []
            for v in samples[y, :, 0]:
                bits += [(int(v) >> (depth - 1 - k)) & 1 for k in range(depth)]
            bits += [0] * (-len(bits) % 8)
            raw = np.packbits(np.array(bits, np.uint8)).tobytes()
        bpp = max(1, ch * depth // 8)
        ft = y % 5
        out = bytearray(len(raw))
        for x in range(len(raw)):
            a = raw[x - bpp] if x >= bpp else 0
            b = prev[x] if prev is not None else 0
            c = prev[x - bpp] if (prev is not None and x >= bpp) else 0
            pred = [0, a, b, (a + b) >> 1, _paeth(a, b, c)][ft]
            out[x] = (raw[x] - pred) & 255
        rows.append(bytes([ft]) + bytes(out))
        prev = raw
    ihdr = struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0)
    png = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr)
    if palette is not None:
        png += _chunk(b"PLTE", bytes(np.asarray(palette, np.uint8).reshape(-1)))
    if trns is not None:
        png += _chunk(b"tRNS", bytes(trns))
    png += _chunk(b"IDAT", zlib.compress(b"".join(rows), 6)) + _chunk(b"IEND", b"")
    return png


def expected_pixels(samples, ctype, depth, palette=None):
    """0x00RRGGBB as Surface::LoadImage builds it from stb's 8-bit channels"""
    s = np.asarray(samples, np.int64)
    if depth == 16:
        s = s >> 8
    elif depth < 8 and ctype == 0:
        s = s * {1: 0xff, 2: 0x55, 4: 0x11}[depth]
    if ctype == 3:
        rgb = np.asarray(palette, np.int64)[s[..., 0]]
        return ((rgb[..., 0] << 16) + (rgb[..., 1] << 8) + rgb[..., 2]).astype(np.uint32)
    if s.shape[2] == 1:
        g = s[..., 0]
        return (g + (g << 8) + (g << 16)).astype(np.uint32)
    flat = s.reshape(-1, s.shape[2]).reshape(-1)             # bytes i*n .. i*n+2, past the end = 0
    n = s.shape[2]
    flat = np.concatenate([flat, np.zeros(3, np.int64)])
    i = np.arange(s.shape[0] * s.shape[1]) * n
    return ((flat[i] << 16) + (flat[i + 1] << 8) + flat[i + 2]).astype(np.uint32).reshape(s.shape[:2])


def decode_rgb8_rows(path, nrows):
    """independent decode of the first nrows of an 8-bit RGB PNG -> 0x00RRGGBB"""
    d = open(path, "rb").read()
    i, idat, w = 8, b"", None
    while i < len(d):
        n, t = struct.unpack(">I", d[i:i + 4])[0], d[i + 4:i + 8]
        if t == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", d[i + 8:i + 18])
            assert depth == 8 and ctype == 2
        elif t == b"IDAT":
            idat += d[i + 8:i + 8 + n]
        i += 12 + n
    raw = zlib.decompressobj().decompress(idat, (3 * w + 1) * nrows)
    stride, prev, out = 3 * w, bytearray(3 * w), []
    for y in range(nrows):
        ft, row = raw[y * (stride + 1)], bytearray(raw[y * (stride + 1) + 1:(y + 1) * (stride + 1)])
        for x in range(stride):
            a = row[x - 3] if x >= 3 else 0
            b, c = prev[x], (prev[x - 3] if x >= 3 else 0)
            row[x] = (row[x] + [0, a, b, (a + b) >> 1, _paeth(a, b, c)][ft]) & 255
        px = np.frombuffer(bytes(row), np.uint8).reshape(w, 3).astype(np.uint32)
        out.append((px[:, 0] << 16) + (px[:, 1] << 8) + px[:, 2])
        prev = row
    return np.array(out, np.uint32)
