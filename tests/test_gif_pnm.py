"""GIF (first frame) and binary PNM decoding for LoadTexture (stbi_loadf,
scene.cpp:294-313; decoders in csrc/scene/image.cpp).

stb_image itself is not built here, so parity with it is
unpinned; the decoders are checked against these restatements of stb_image
2.29's documented behaviour (the reference's vendored copy, read as text):

* PNM: P5 / P6 only, header integers separated by whitespace and '#'
  comments, maxval only selects 8- or 16-bit samples; a 16-bit sample keeps
  its second (low-order) byte, since stb reads the big-endian samples in host
  order and reduces with >> 8.
* GIF: the LZW data of each test image comes from Pillow's encoder (a
  reference implementation of the format) and is re-wrapped in a container
  written here, so that the logical screen, frame rectangle, interlacing,
  global / local palettes, graphic-control transparency and background index
  vary independently.  Expected pixels: Pillow's decoded palette indices
  mapped the way stb maps them (transparent entries not drawn, so 0,0,0,0;
  when the background index is not 0, pixels outside the frame take the
  global background entry in B,G,R order with alpha 255).
"""
from __future__ import annotations

import io
import struct

import numpy as np
import pytest

from test_ingestion import stbi_float, texture_pixels, ulps

PIL = pytest.importorskip("PIL.Image")
RNG = np.random.default_rng(77)


def check_both(pt, path, exp):
    got = pt.load_image_rgba8(path)
    assert got.shape == exp.shape
    bad = np.argwhere(got != exp)
    assert bad.size == 0, f"{len(bad)} samples differ, first {bad[:3].tolist()}"
    s = pt.Scene.empty()
    f, _ = texture_pixels(pt, s, path)
    assert np.max(ulps(f, stbi_float(exp.astype(np.uint8)))) <= 1
    s.close()


# --- PNM ------------------------------------------------------------------------

def pnm_bytes(magic, w, h, maxval, samples, header_style=0):
    if header_style == 0:
        hdr = f"{magic}\n{w} {h}\n{maxval}\n".encode()
    else:   # comments, tabs, CR and several spaces between the fields
        hdr = f"{magic}# made by a test\n \t{w}\r\n# second comment\n {h}   {maxval}\n".encode()
    if maxval > 255:
        data = b"".join(struct.pack(">H", int(v)) for v in samples.reshape(-1))
    else:
        data = bytes(samples.astype(np.uint8).reshape(-1).tolist())
    return hdr + data


@pytest.mark.parametrize("magic,maxval,style", [("P6", 255, 0), ("P6", 100, 1), ("P5", 255, 1), ("P6", 65535, 0),
                                                ("P5", 1000, 1), ("P6", 256, 0)])
def test_pnm(pt, tmp_path, magic, maxval, style):
    W, H = 13, 7
    comp = 3 if magic == "P6" else 1
    v = RNG.integers(0, maxval + 1, size=(H, W, comp))
    p = tmp_path / "t.pnm"
    p.write_bytes(pnm_bytes(magic, W, H, maxval, v, style))
    s8 = (v & 0xFF) if maxval > 255 else v            # 16-bit: the sample's low-order byte
    exp = np.full((H, W, 4), 255, np.int64)
    exp[..., :3] = s8 if comp == 3 else np.repeat(s8, 3, axis=-1)
    check_both(pt, p, exp.astype(np.uint8))


def test_pnm_errors(pt, tmp_path):
    p = tmp_path / "t.ppm"
    v = RNG.integers(0, 256, size=(4, 5, 3))
    full = pnm_bytes("P6", 5, 4, 255, v)
    p.write_bytes(full[:-7])
    with pytest.raises(ValueError, match="truncated"):
        pt.load_image_rgba8(p)
    p.write_bytes(b"P6\n0 4\n255\n" + bytes(60))
    with pytest.raises(ValueError, match="width"):
        pt.load_image_rgba8(p)
    p.write_bytes(b"P6\n5 4\n70000\n" + bytes(120))
    with pytest.raises(ValueError, match="65535"):
        pt.load_image_rgba8(p)
    p.write_bytes(b"P3\n2 1\n255\n1 2 3 4 5 6\n")      # ASCII PNM: not a stb format
    with pytest.raises(ValueError, match="unsupported image format"):
        pt.load_image_rgba8(p)


# --- GIF ------------------------------------------------------------------------

def pillow_lzw(indices, palette_rgb, interlace):
    """Pillow's encoding of a P image: (LZW minimum code size, raw data
    sub-blocks incl. terminator, interlaced flag as written, decoded indices)."""
    h, w = indices.shape
    im = PIL.fromarray(indices.astype(np.uint8), mode="P")
    pal = np.zeros((256, 3), np.uint8)
    pal[: len(palette_rgb)] = palette_rgb
    im.putpalette(pal.reshape(-1).tolist())
    buf = io.BytesIO()
    im.save(buf, format="GIF", optimize=False, interlace=interlace)
    data = buf.getvalue()
    # skip the header, the global table and any extensions up to the image descriptor
    flags = data[10]
    pos = 13 + (3 * (2 << (flags & 7)) if flags & 0x80 else 0)
    while data[pos] == 0x21:
        pos += 2
        while data[pos]:
            pos += 1 + data[pos]
        pos += 1
    assert data[pos] == 0x2C
    lflags = data[pos + 9]
    pos += 10
    if lflags & 0x80:
        pos += 3 * (2 << (lflags & 7))
    start = pos
    pos += 1
    while data[pos]:
        pos += 1 + data[pos]
    raster = data[start: pos + 1]
    decoded = np.asarray(PIL.open(io.BytesIO(data)).convert("P"), dtype=np.int64)
    # Pillow may write with a smaller code size or reorder nothing: the indices it
    # decodes from its own file are the ground truth for the raster bytes.
    return raster, bool(lflags & 0x40), decoded


def gif_bytes(W, H, raster, rect, interlaced, gpal=None, bgindex=0, lpal=None, transparent=None, pre_ext=True):
    out = bytearray(b"GIF89a")
    gbits = 7
    flags = (0x80 | gbits) if gpal is not None else 0
    out += struct.pack("<HHBBB", W, H, flags, bgindex, 0)
    if gpal is not None:
        t = np.zeros((2 << gbits, 3), np.uint8)
        t[: len(gpal)] = gpal
        out += t.tobytes()
    if pre_ext:   # an application / comment extension stb must skip
        out += b"\x21\xFE\x05hello\x00"
    if transparent is not None:
        out += struct.pack("<BBBBHBB", 0x21, 0xF9, 4, 0x01, 0, transparent, 0)
    x, y, w, h = rect
    lflags = (0x40 if interlaced else 0) | ((0x80 | 7) if lpal is not None else 0)
    out += struct.pack("<BHHHHB", 0x2C, x, y, w, h, lflags)
    if lpal is not None:
        t = np.zeros((256, 3), np.uint8)
        t[: len(lpal)] = lpal
        out += t.tobytes()
    out += raster
    out += b"\x21\xF9\x04\x00\x00\x00\x00\x00"   # a second frame's control block, never read
    out += b"\x3B"
    return bytes(out)


def gif_expected(W, H, indices, rect, gpal, bgindex, lpal, transparent):
    table = lpal if lpal is not None else gpal
    out = np.zeros((H, W, 4), np.int64)
    drawn = np.zeros((H, W), bool)
    x, y, w, h = rect
    drawn[y:y + h, x:x + w] = True
    rgb = np.asarray(table, np.int64)[indices]
    opaque = indices != transparent if transparent is not None else np.ones_like(indices, bool)
    sub = out[y:y + h, x:x + w]
    sub[opaque, :3] = rgb[opaque]
    sub[opaque, 3] = 255
    if bgindex > 0:
        b = np.zeros(3, np.int64) if gpal is None or bgindex >= len(gpal) else np.asarray(gpal[bgindex], np.int64)
        out[~drawn] = [b[2], b[1], b[0], 255]          # stb copies the stored B,G,R entry
    return out.astype(np.uint8)


GIF_CASES = [
    # (W, H, rect, interlace, local palette, transparent, bgindex, colours)
    (24, 18, (0, 0, 24, 18), False, False, None, 0, 16),
    (40, 33, (0, 0, 40, 33), True, False, None, 0, 200),
    (31, 27, (3, 5, 20, 17), True, True, 7, 9, 60),
    (50, 40, (10, 2, 30, 33), False, False, 3, 2, 256),
    (17, 9, (1, 1, 15, 7), False, True, None, 0, 3),
    (64, 64, (0, 0, 64, 64), True, False, 0, 5, 256),     # large tables: codes past 4096 entries
]


@pytest.mark.parametrize("case", range(len(GIF_CASES)))
def test_gif(pt, tmp_path, case):
    W, H, rect, interlace, local, transparent, bgindex, ncol = GIF_CASES[case]
    rng = np.random.default_rng(500 + case)
    x, y, w, h = rect
    pal = rng.integers(0, 256, size=(ncol, 3))
    idx = rng.integers(0, ncol, size=(h, w))
    idx[: h // 2, : w // 2] = idx[0, 0]                    # runs for the LZW dictionary
    raster, inter_written, decoded = pillow_lzw(idx, pal, interlace)
    gpal = rng.integers(0, 256, size=(256, 3))
    if not local:
        gpal = np.concatenate([pal, gpal[ncol:]])[:256]
    lpal = pal if local else None
    data = gif_bytes(W, H, raster, rect, inter_written, gpal=gpal, bgindex=bgindex, lpal=lpal, transparent=transparent)
    p = tmp_path / "t.gif"
    p.write_bytes(data)
    exp = gif_expected(W, H, decoded, rect, gpal, bgindex, lpal, transparent)
    check_both(pt, p, exp)


def test_gif_pillow_files(pt, tmp_path):
    """Whole files as Pillow writes them (global palette, optional GCE
    transparency), decoded like Pillow decodes them."""
    for k, (w, h, transp) in enumerate([(37, 23, None), (64, 48, 5), (8, 200, 1)]):
        rng = np.random.default_rng(900 + k)
        n = 32
        idx = rng.integers(0, n, size=(h, w))
        im = PIL.fromarray(idx.astype(np.uint8), mode="P")
        pal = rng.integers(0, 256, size=(256, 3)).astype(np.uint8)
        im.putpalette(pal.reshape(-1).tolist())
        p = tmp_path / f"p{k}.gif"
        kw = {"transparency": transp} if transp is not None else {}
        im.save(p, optimize=False, **kw)
        back = PIL.open(p)
        bi = np.asarray(back, dtype=np.int64)
        bp = np.asarray(back.getpalette(), np.int64).reshape(-1, 3)
        exp = np.zeros((h, w, 4), np.int64)
        exp[..., :3] = bp[bi]
        exp[..., 3] = 255
        if transp is not None:
            exp[bi == transp] = 0
        check_both(pt, p, exp.astype(np.uint8))


def test_gif_errors(pt, tmp_path):
    p = tmp_path / "t.gif"
    p.write_bytes(b"GIF89a" + struct.pack("<HHBBB", 4, 4, 0, 0, 0) + b"\x2C" + struct.pack("<HHHHB", 0, 0, 4, 4, 0)
                  + b"\x02\x00\x3B")
    with pytest.raises(ValueError, match="color table"):
        pt.load_image_rgba8(p)
    # a raster that does not start with a clear code
    pal = bytes(3 * 4)
    p.write_bytes(b"GIF89a" + struct.pack("<HHBBB", 2, 1, 0x81, 0, 0) + pal + b"\x2C"
                  + struct.pack("<HHHHB", 0, 0, 2, 1, 0) + b"\x02\x01\x01\x00\x3B")
    with pytest.raises(ValueError, match="clear code"):
        pt.load_image_rgba8(p)
