"""Decoder corpus for the sanitizer runs (tools/sanitize/run.sh): valid files
of every format LoadTexture / LoadModelAsPrefab / LoadScene read, then for
each one its truncations and random bit flips, plus headers claiming huge
images (the allocation guards).  Deterministic (fixed seeds).

usage: python tools/sanitize/make_corpus.py OUT_DIR
"""
from __future__ import annotations

import io
import struct
import sys
import zlib
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))


def pil_files(rng):
    from PIL import Image
    out = {}
    W, H = 37, 23
    rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    rgba = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    grey = rng.integers(0, 256, (H, W), dtype=np.uint8)
    im_rgb, im_rgba, im_l = Image.fromarray(rgb), Image.fromarray(rgba), Image.fromarray(grey)
    im_p = im_rgb.convert("P", palette=Image.ADAPTIVE, colors=64)

    def save(name, im, fmt, **kw):
        b = io.BytesIO()
        im.save(b, fmt, **kw)
        out[name] = b.getvalue()

    save("rgb.png", im_rgb, "PNG")
    save("rgba.png", im_rgba, "PNG")
    save("grey.png", im_l, "PNG")
    save("pal.png", im_p, "PNG")
    save("rgb24.bmp", im_rgb, "BMP")
    save("pal8.bmp", im_p, "BMP")
    save("mono.bmp", im_l.convert("1"), "BMP")
    save("rgb.tga", im_rgb, "TGA")
    save("rgba_rle.tga", im_rgba, "TGA", compression="tga_rle")
    save("grey.tga", im_l, "TGA")
    save("pal.gif", im_p, "GIF")
    save("interlaced.gif", im_p, "GIF", interlace=True)
    save("rgb.ppm", im_rgb, "PPM")
    save("grey.pgm", im_l, "PPM")
    save("base.jpg", im_rgb, "JPEG", quality=80)
    save("prog.jpg", im_rgb, "JPEG", quality=70, progressive=True)
    save("sub420.jpg", im_rgb, "JPEG", quality=60, subsampling=2)
    save("grey.jpg", im_l, "JPEG", quality=90)
    save("cmyk.jpg", im_rgb.convert("CMYK"), "JPEG", quality=85)
    return out


def png_interlaced(rng):
    import test_ingestion as ti
    s = rng.integers(0, 256, (13, 17, 4)).astype(np.uint16)
    return ti.png_bytes(s, 6, 8, interlace=True)


def hdr_bytes(rng, W=19, H=7, rle=False):
    head = b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n" + f"-Y {H} +X {W}\n".encode()
    px = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    px[..., 3] = rng.integers(120, 140, (H, W))
    if not rle:
        return head + px.tobytes()
    body = b""
    for y in range(H):   # new-style RLE scanline: 2,2,W>>8,W&255 then 4 channel runs (literals)
        body += bytes([2, 2, W >> 8, W & 255])
        for c in range(4):
            ch = px[y, :, c].tobytes()
            for i in range(0, W, 128):
                seg = ch[i:i + 128]
                body += bytes([len(seg)]) + seg
    return head + body


def psd_files(rng):
    import test_psd as tp
    planes = rng.integers(0, 256, (4, 9, 11), dtype=np.uint8)
    return {"raw8.psd": tp.psd_bytes(planes, 8, False), "rle8.psd": tp.psd_bytes(planes, 8, True),
            "raw16.psd": tp.psd_bytes(planes.astype(np.uint16) * 257, 16, False)}


def huge_headers():
    """Headers claiming images past stb's size guards (must be rejected
    before allocating)."""
    out = {}
    # GIF: 65535 x 65535, global palette, one empty frame
    g = b"GIF89a" + struct.pack("<HH", 65535, 65535) + bytes([0x80, 0, 0]) + bytes(6)
    g += b"\x2c" + struct.pack("<HHHH", 0, 0, 65535, 65535) + b"\x00\x02\x00\x3b"
    out["huge.gif"] = g
    out["huge13.gif"] = b"GIF89a" + struct.pack("<HH", 65535, 65535) + bytes([0, 0, 0])
    # PSD: 2^24 x 2^24 RGB, raw
    p = b"8BPS" + struct.pack(">H", 1) + bytes(6) + struct.pack(">HIIHH", 3, 1 << 24, 1 << 24, 8, 3)
    p += struct.pack(">III", 0, 0, 0) + struct.pack(">H", 0)
    out["huge.psd"] = p
    # PSD: legal size, raw planes missing (truncated before the pixels)
    p2 = b"8BPS" + struct.pack(">H", 1) + bytes(6) + struct.pack(">HIIHH", 3, 4000, 4000, 8, 3)
    p2 += struct.pack(">III", 0, 0, 0) + struct.pack(">H", 0) + bytes(100)
    out["short_raw.psd"] = p2
    # JPEG: SOF0 65535 x 65535, 3 components
    j = b"\xff\xd8" + b"\xff\xc0" + struct.pack(">HBHHB", 17, 8, 65535, 65535, 3)
    j += bytes([1, 0x11, 0, 2, 0x11, 0, 3, 0x11, 0]) + b"\xff\xd9"
    out["huge.jpg"] = j
    # PNG: IHDR 2^24 x 2^24 RGBA8, empty IDAT
    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", 1 << 24, 1 << 24, 8, 6, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(b"")) + chunk(b"IEND", b"")
    out["huge.png"] = png
    # BMP 24-bit 2^24 x 2^24 (pixels absent)
    out["huge.bmp"] = b"BM" + struct.pack("<IHHI", 0, 0, 0, 54) + struct.pack("<IiiHHIIiiII", 40, 1 << 24, 1 << 24, 1, 24, 0, 0, 0, 0, 0, 0)
    # TGA 65535 x 65535 true-colour 32-bit
    out["huge.tga"] = bytes([0, 0, 2]) + bytes(9) + struct.pack("<HH", 65535, 65535) + bytes([32, 8])
    # PNM 65535 x 65535 P6
    out["huge.ppm"] = b"P6\n65535 65535\n255\n" + bytes(16)
    # HDR 2^24 x 2^24
    out["huge.hdr"] = b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y 16777216 +X 16777216\n" + bytes(16)
    return out


def obj_files(tmp: Path):
    import test_ingestion as ti
    d = tmp / "obj_src"
    d.mkdir(parents=True, exist_ok=True)
    path = Path(ti.write_model(d))
    return {p.name: p.read_bytes() for p in path.parent.iterdir() if p.is_file()}, path.name


def mutations(name, data, rng, n_trunc=12, n_flip=24):
    out = {}
    L = len(data)
    cuts = sorted(set([0, 1, 2, 4, 8, 12, 16, 24, 32, L // 4, L // 2, L - 1] +
                      list(rng.integers(0, max(L, 1), n_trunc))))
    for c in cuts:
        if 0 <= c < L:
            out[f"trunc{c}_{name}"] = data[:c]
    arr = np.frombuffer(data, np.uint8)
    for k in range(n_flip):
        a = arr.copy()
        nb = int(rng.integers(1, 9))
        head = min(L, 64)
        for _ in range(nb):
            # half the flips land in the first 64 bytes (headers), half anywhere
            i = int(rng.integers(0, head if k % 2 == 0 else L))
            a[i] ^= np.uint8(1 << int(rng.integers(0, 8)))
        out[f"flip{k}_{name}"] = a.tobytes()
    return out


def main():
    out = Path(sys.argv[1])
    (out / "images").mkdir(parents=True, exist_ok=True)
    (out / "models").mkdir(parents=True, exist_ok=True)
    rng = np.random.default_rng(1234)
    import conftest  # noqa: F401  (package import)
    base = pil_files(rng)
    base["interlaced.png"] = png_interlaced(rng)
    base["flat.hdr"] = hdr_bytes(rng)
    base["rle.hdr"] = hdr_bytes(rng, W=40, H=5, rle=True)
    base.update(psd_files(rng))
    files = dict(base)
    for k, v in base.items():
        files.update(mutations(k, v, rng))
    files.update(huge_headers())
    for k, v in files.items():
        (out / "images" / k).write_bytes(v)
    # OBJ + MTL + PNG texture, and corrupted OBJ / MTL texts
    objs, main_name = obj_files(out)
    mdir = out / "models"
    for k, v in objs.items():
        (mdir / k).write_bytes(v)
    obj = objs[main_name]
    count = 0
    for k, v in mutations(main_name, obj, rng, n_trunc=16, n_flip=48).items():
        sub = mdir / f"m{count}"
        sub.mkdir(exist_ok=True)
        for kk, vv in objs.items():
            (sub / kk).write_bytes(vv)
        (sub / main_name).write_bytes(v)
        count += 1
    # scene file (LoadScene): a saved scene + corrupted JSON / zlib blobs
    sdir = out / "scenes"
    sdir.mkdir(exist_ok=True)
    pt = conftest.load_package()
    sc = pt.Scene.create()
    sc.create_entity(pt.ENTITY_SPHERE, position=(0, 0, 1))
    sc.instantiate_prefab(sc.load_model_as_prefab(str(mdir / main_name)))
    src = sdir / "src"
    src.mkdir(exist_ok=True)
    sc.save(str(src / "scene.json"))
    sc.close()
    parts = {p.name: p.read_bytes() for p in src.iterdir() if p.is_file()}
    nscene = 0
    for target, data in sorted(parts.items()):
        for k, v in mutations(target, data, rng, n_trunc=6, n_flip=10).items():
            d = sdir / f"s{nscene}"
            d.mkdir(exist_ok=True)
            for kk, vv in parts.items():
                (d / kk).write_bytes(vv)
            (d / target).write_bytes(v)
            nscene += 1
    print(f"{len(files)} image files, {count + 1} model variants, {nscene + 1} scene variants in {out}")


if __name__ == "__main__":
    main()
