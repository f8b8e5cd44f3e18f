"""PSD (composited image) decoding for LoadTexture (stbi_loadf,
scene.cpp:294-313; DecodePSD in csrc/scene/image.cpp).

stb_image itself is not built here, so parity with it is
unpinned; files are written by the encoder below and the expected pixels
restate stb_image 2.29's stbi__psd_load (the reference's vendored copy, read
as text): RGB mode, 8/16-bit, raw or PackBits planes, the first four
channels, missing ones 0 (alpha 255), and with >= 4 channels the white matte
removed from partly transparent pixels in float32 as v * (1/a) + 255 * (1 - 1/a),
truncated and kept modulo 256.
"""
from __future__ import annotations

import struct

import numpy as np
import pytest

from test_gif_pnm import check_both


def packbits(row: bytes) -> bytes:
    """PackBits: runs of >= 3 equal bytes as repeats, the rest as literals."""
    out = bytearray()
    i, n = 0, len(row)
    lit = bytearray()

    def flush():
        nonlocal lit
        while lit:
            chunk, lit = lit[:128], lit[128:]
            out.append(len(chunk) - 1)
            out.extend(chunk)

    while i < n:
        j = i
        while j < n and j - i < 128 and row[j] == row[i]:
            j += 1
        if j - i >= 3:
            flush()
            out.append(257 - (j - i))
            out.append(row[i])
            i = j
        else:
            lit.append(row[i])
            i += 1
    flush()
    return bytes(out)


def psd_bytes(planes, depth, rle, mode=3, extra_sections=True, noop=False):
    c, h, w = planes.shape
    out = bytearray(b"8BPS")
    out += struct.pack(">H", 1) + bytes(6)
    out += struct.pack(">HIIHH", c, h, w, depth, mode)
    if extra_sections:
        out += struct.pack(">I", 5) + b"mode!"
        out += struct.pack(">I", 3) + b"res"
        out += struct.pack(">I", 7) + b"layers!"
    else:
        out += bytes(12)
    out += struct.pack(">H", 1 if rle else 0)
    if rle:
        rows = [packbits(bytes(planes[k, y].astype(np.uint8).tolist())) for k in range(c) for y in range(h)]
        if noop:
            rows = [b"\x80" + r for r in rows]
        out += b"".join(struct.pack(">H", len(r)) for r in rows)
        out += b"".join(rows)
    elif depth == 16:
        out += planes.astype(">u2").tobytes()
    else:
        out += planes.astype(np.uint8).tobytes()
    return bytes(out)


def psd_expected(planes, depth):
    c, h, w = planes.shape
    v = planes >> 8 if depth == 16 else planes
    out = np.zeros((h, w, 4), np.int64)
    out[..., 3] = 255
    for k in range(min(c, 4)):
        out[..., k] = v[k]
    if c >= 4:
        a = out[..., 3]
        m = (a != 0) & (a != 255)
        af = a.astype(np.float32) / np.float32(255.0)
        with np.errstate(divide="ignore", invalid="ignore"):
            ra = np.float32(1.0) / af
        inv = np.float32(255.0) * (np.float32(1.0) - ra)
        for k in range(3):
            with np.errstate(invalid="ignore"):
                f = out[..., k].astype(np.float32) * ra + inv
            t = np.trunc(np.where(m, f, 0)).astype(np.int64) & 0xFF
            out[..., k] = np.where(m, t, out[..., k])
    return out.astype(np.uint8)


CASES = [
    # (channels, depth, rle)
    (3, 8, False), (3, 8, True), (4, 8, False), (4, 8, True),
    (5, 8, True), (1, 8, False), (2, 8, True), (3, 16, False), (4, 16, False),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_psd(pt, tmp_path, case):
    c, depth, rle = CASES[case]
    rng = np.random.default_rng(300 + case)
    h, w = 11, 37
    hi = 65536 if depth == 16 else 256
    planes = rng.integers(0, hi, size=(c, h, w))
    planes[:, : h // 2, : w // 2] = planes[:, :1, :1]           # runs for PackBits
    if c >= 4:
        a = planes[3] >> 8 if depth == 16 else planes[3]
        a[0, :3] = [0, 255, 1]                                    # both edges and a tiny alpha
    p = tmp_path / "t.psd"
    p.write_bytes(psd_bytes(planes, depth, rle, noop=(case == 3)))
    check_both(pt, p, psd_expected(planes, depth))


def test_psd_long_rows(pt, tmp_path):
    """Runs and literals longer than 128 bytes, split over several packets."""
    rng = np.random.default_rng(9)
    planes = rng.integers(0, 256, size=(3, 4, 300))
    planes[:, 1, :] = 77
    planes[:, 2, 50:250] = planes[:, 2, 50:51]
    p = tmp_path / "l.psd"
    p.write_bytes(psd_bytes(planes, 8, True, extra_sections=False))
    check_both(pt, p, psd_expected(planes, 8))


def test_psd_errors(pt, tmp_path):
    p = tmp_path / "e.psd"
    planes = np.zeros((3, 2, 2), np.int64)
    p.write_bytes(psd_bytes(planes, 8, False, mode=4))
    with pytest.raises(ValueError, match="RGB"):
        pt.load_image_rgba8(p)
    p.write_bytes(psd_bytes(planes, 32, False))
    with pytest.raises(ValueError, match="bit depth"):
        pt.load_image_rgba8(p)
    hdr = psd_bytes(planes, 8, False)[:-12 - 2]     # up to the compression field
    # row counts, then a 6-byte literal where the plane holds 4 pixels
    p.write_bytes(hdr + b"\x00\x01" + bytes(2 * 2 * 3) + b"\x05" + bytes(6) + bytes(32))
    with pytest.raises(ValueError, match="RLE"):
        pt.load_image_rgba8(p)
    bad = bytearray(psd_bytes(planes, 8, False))
    bad[4:6] = b"\x00\x02"
    p.write_bytes(bytes(bad))
    with pytest.raises(ValueError, match="version"):
        pt.load_image_rgba8(p)
