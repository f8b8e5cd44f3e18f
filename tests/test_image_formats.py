"""BMP and TGA texture decoding (LoadTexture via stbi_loadf, scene.cpp:294-313).

stb_image is not vendored-runnable here; the files are
made by the encoders below, written from the BMP (Microsoft
BITMAPINFOHEADER / V4 / V5) and Truevision TGA 2.0 layouts, and the expected
8-bit samples follow stb_image's documented conversions: TGA RGB555 channels
as (v * 255) / 31, BMP bit fields widened by bit replication, BGR(A) byte
order, bottom-up rows unless flagged, a 32-bit BMP with all-zero alpha read
as opaque.  The loader then linearises exactly as for PNG (stbi__ldr_to_hdr).
"""
from __future__ import annotations

import struct

import numpy as np
import pytest

from test_ingestion import stbi_float, texture_pixels, ulps

RNG = np.random.default_rng(31)
H, W = 7, 11   # odd width: BMP row padding, TGA packets crossing rows


def check(pt, path, exp):
    s = pt.Scene.empty()
    got, _ = texture_pixels(pt, s, path)
    want = stbi_float(exp.astype(np.uint8))
    assert got.shape == want.shape
    assert np.max(ulps(got, want)) <= 1
    s.close()


def replicate(x, n):
    """n-bit field -> 8 bits by repeating its bit pattern."""
    s, bits = x.astype(np.int64), n
    while bits < 8:
        s = (s << n) | x
        bits += n
    return s >> (bits - 8)


# --- TGA ----------------------------------------------------------------------

def tga_rle(pixels, pb):
    """Run-length packets over the flattened pixel byte strings."""
    out, i, n = b"", 0, len(pixels)
    while i < n:
        j = i
        while j + 1 < n and pixels[j + 1] == pixels[i] and j - i < 127:
            j += 1
        if j > i:
            out += bytes([0x80 | (j - i)]) + pixels[i]
            i = j + 1
            continue
        j = i
        while j + 1 < n and pixels[j + 1] != pixels[j] and j - i < 127:
            j += 1
        out += bytes([j - i]) + b"".join(pixels[i:j + 1])
        i = j + 1
    return out


def tga_bytes(pix, itype, bits, top_down=False, palette=b"", cmbits=0, cmlen=0, ident=b"ab"):
    """pix: H x W list of per-pixel byte strings, top row first."""
    rows = pix if top_down else pix[::-1]
    flat = [p for r in rows for p in r]
    data = tga_rle(flat, bits // 8) if itype >= 9 else b"".join(flat)
    hdr = struct.pack("<BBBHHBHHHHBB", len(ident), 1 if palette else 0, itype, 0, cmlen, cmbits, 0, 0,
                      len(pix[0]), len(pix), bits, 0x20 if top_down else 0)
    return hdr + ident + palette + data


def rand8(shape, runs=True):
    a = RNG.integers(0, 256, size=shape)
    if runs:
        a[:, 2:6] = a[:, 2:3]           # repeated pixels for RLE runs
    return a


@pytest.mark.parametrize("itype,top_down", [(2, False), (10, True), (10, False)])
def test_tga_truecolor(pt, tmp_path, itype, top_down):
    for bits in (24, 32):
        c = rand8((H, W, 4))
        if bits == 24:
            c[..., 3] = 255
        pix = [[bytes([c[y, x, 2], c[y, x, 1], c[y, x, 0]] + ([c[y, x, 3]] if bits == 32 else [])) for x in range(W)]
               for y in range(H)]
        (tmp_path / "t.tga").write_bytes(tga_bytes(pix, itype, bits, top_down))
        check(pt, tmp_path / "t.tga", c)


def test_tga_rgb555(pt, tmp_path):
    v = RNG.integers(0, 1 << 16, size=(H, W))
    pix = [[struct.pack("<H", int(v[y, x])) for x in range(W)] for y in range(H)]
    (tmp_path / "t.tga").write_bytes(tga_bytes(pix, 2, 16))
    exp = np.zeros((H, W, 4), np.int64)
    for c, sh in enumerate((10, 5, 0)):
        exp[..., c] = ((v >> sh) & 31) * 255 // 31
    exp[..., 3] = 255                    # the attribute bit is not alpha
    check(pt, tmp_path / "t.tga", exp)


@pytest.mark.parametrize("itype", [3, 11])
def test_tga_grey(pt, tmp_path, itype):
    g = rand8((H, W))
    (tmp_path / "g.tga").write_bytes(tga_bytes([[bytes([g[y, x]]) for x in range(W)] for y in range(H)], itype, 8))
    check(pt, tmp_path / "g.tga", np.stack([g, g, g, np.full_like(g, 255)], -1))
    a = rand8((H, W))
    pix = [[bytes([g[y, x], a[y, x]]) for x in range(W)] for y in range(H)]
    (tmp_path / "ga.tga").write_bytes(tga_bytes(pix, itype, 16))
    check(pt, tmp_path / "ga.tga", np.stack([g, g, g, a], -1))


@pytest.mark.parametrize("itype,cmbits", [(1, 24), (9, 32)])
def test_tga_colormapped(pt, tmp_path, itype, cmbits):
    n = 20
    pal = RNG.integers(0, 256, size=(n, 4))
    if cmbits == 24:
        pal[:, 3] = 255
    palette = b"".join(bytes([p[2], p[1], p[0]] + ([p[3]] if cmbits == 32 else [])) for p in pal)
    idx = RNG.integers(0, n, size=(H, W))
    idx[0, 0] = 200                       # past the map: entry 0 (stb)
    pix = [[bytes([idx[y, x]]) for x in range(W)] for y in range(H)]
    (tmp_path / "p.tga").write_bytes(tga_bytes(pix, itype, 8, palette=palette, cmbits=cmbits, cmlen=n))
    exp = pal[np.where(idx < n, idx, 0)]
    check(pt, tmp_path / "p.tga", exp)


# --- BMP ----------------------------------------------------------------------

def bmp_bytes(rows_bytes, w, h, bpp, hsz=40, comp=0, masks=None, palette=b"", top_down=False):
    """rows_bytes: unpadded rows, top row first."""
    stride = ((w * bpp + 31) // 32) * 4
    rows = rows_bytes if top_down else rows_bytes[::-1]
    data = b"".join(r + b"\0" * (stride - len(r)) for r in rows)
    if hsz == 12:
        info = struct.pack("<IhhHH", 12, w, h, 1, bpp)
        extra = b""
    else:
        info = struct.pack("<IiiHHIIiiII", hsz, w, -h if top_down else h, 1, bpp, comp, len(data), 2835, 2835, 0, 0)
        extra = b""
        if comp == 3 and hsz == 40:
            extra = struct.pack("<III", *masks[:3])
        elif hsz > 40:
            m = list(masks or (0, 0, 0, 0)) + [0] * 4
            info += struct.pack("<IIII", *m[:4])
            info += b"\0" * (hsz - len(info))
    off = 14 + len(info) + len(extra) + len(palette)
    return b"BM" + struct.pack("<IHHI", off + len(data), 0, 0, off) + info + extra + palette + data


def test_bmp_24bit(pt, tmp_path):
    for hsz in (40, 12):
        c = rand8((H, W, 3), runs=False)
        rows = [b"".join(bytes([c[y, x, 2], c[y, x, 1], c[y, x, 0]]) for x in range(W)) for y in range(H)]
        (tmp_path / "c.bmp").write_bytes(bmp_bytes(rows, W, H, 24, hsz=hsz))
        check(pt, tmp_path / "c.bmp", np.concatenate([c, np.full((H, W, 1), 255)], -1))


@pytest.mark.parametrize("zero_alpha,top_down", [(False, False), (True, True)])
def test_bmp_32bit_default_masks(pt, tmp_path, zero_alpha, top_down):
    c = rand8((H, W, 4), runs=False)
    if zero_alpha:
        c[..., 3] = 0
    rows = [b"".join(bytes([c[y, x, 2], c[y, x, 1], c[y, x, 0], c[y, x, 3]]) for x in range(W)) for y in range(H)]
    (tmp_path / "a.bmp").write_bytes(bmp_bytes(rows, W, H, 32, top_down=top_down))
    exp = c.copy()
    if zero_alpha:
        exp[..., 3] = 255                 # all-zero alpha reads as opaque
    check(pt, tmp_path / "a.bmp", exp)


@pytest.mark.parametrize("comp,masks", [(0, None), (3, (0xF800, 0x07E0, 0x001F))])
def test_bmp_16bit(pt, tmp_path, comp, masks):
    v = RNG.integers(0, 1 << 16, size=(H, W))
    rows = [b"".join(struct.pack("<H", int(v[y, x])) for x in range(W)) for y in range(H)]
    (tmp_path / "s.bmp").write_bytes(bmp_bytes(rows, W, H, 16, comp=comp, masks=masks))
    fields = [(10, 5), (5, 5), (0, 5)] if comp == 0 else [(11, 5), (5, 6), (0, 5)]
    exp = np.zeros((H, W, 4), np.int64)
    for c, (sh, n) in enumerate(fields):
        exp[..., c] = replicate((v >> sh) & ((1 << n) - 1), n)
    exp[..., 3] = 255
    check(pt, tmp_path / "s.bmp", exp)


def test_bmp_v5_bitfields(pt, tmp_path):
    """BITMAPV5HEADER (124) with its masks: 10-10-10 colour (top 8 bits kept),
    2-bit alpha (replicated)."""
    v = RNG.integers(0, 1 << 32, size=(H, W), dtype=np.uint64)
    masks = (0x3FF00000, 0x000FFC00, 0x000003FF, 0xC0000000)
    rows = [b"".join(struct.pack("<I", int(v[y, x])) for x in range(W)) for y in range(H)]
    (tmp_path / "v5.bmp").write_bytes(bmp_bytes(rows, W, H, 32, hsz=124, comp=3, masks=masks))
    v = v.astype(np.int64)
    exp = np.stack([(v >> 22) & 255, (v >> 12) & 255, (v >> 2) & 255, replicate((v >> 30) & 3, 2)], -1)
    check(pt, tmp_path / "v5.bmp", exp)


@pytest.mark.parametrize("bpp,hsz", [(8, 40), (4, 40), (1, 40), (8, 12)])
def test_bmp_palette(pt, tmp_path, bpp, hsz):
    n = 1 << bpp
    pal = RNG.integers(0, 256, size=(n, 3))
    es = 3 if hsz == 12 else 4
    palette = b"".join(bytes([p[2], p[1], p[0]] + [0] * (es - 3)) for p in pal)
    idx = RNG.integers(0, n, size=(H, W))
    rows = []
    for y in range(H):
        bits = "".join(format(int(i), f"0{bpp}b") for i in idx[y])
        bits += "0" * (-len(bits) % 8)
        rows.append(bytes(int(bits[i:i + 8], 2) for i in range(0, len(bits), 8)))
    (tmp_path / "p.bmp").write_bytes(bmp_bytes(rows, W, H, bpp, hsz=hsz, palette=palette))
    exp = np.concatenate([pal[idx], np.full((H, W, 1), 255)], -1)
    check(pt, tmp_path / "p.bmp", exp)


def test_unknown_format_rejected(pt, tmp_path):
    pic = b"\x53\x80\xf6\x34" + b"\0" * 84 + b"PICT" + b"\0" * 16
    (tmp_path / "x.pic").write_bytes(pic)      # Softimage PIC: a stb format this build does not read
    (tmp_path / "x.jpg").write_bytes(b"\xff\xd8\xff\xe0" + b"\0" * 64)   # SOI, then an APP0 of length 0
    s = pt.Scene.empty()
    with pytest.raises(OSError, match="unsupported image format"):
        s.load_texture(tmp_path / "x.pic", 0)
    with pytest.raises(OSError, match="JPEG"):
        s.load_texture(tmp_path / "x.jpg", 0)
    s.close()
