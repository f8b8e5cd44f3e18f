"""Scene ingestion: Wavefront OBJ/MTL (restating the reference's vendored
tinyobjloader), LoadModelAsPrefab (scene.cpp:601-903) and LoadTexture
(scene.cpp:294-313; PNG / Radiance HDR with stbi_loadf semantics).

The reference's vendored parsers could not be run here, so
the expected values come from the OBJ / PNG / RGBE specifications, encoded by
the helpers below: parity with tinyobjloader / stb_image is unpinned.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np
import pytest

import oracle_lib

# --- PNG encoder (ISO/IEC 15948) used to make test vectors --------------------


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)


def _filter_rows(rows, bpp, filters):
    out = bytearray()
    prev = bytes(len(rows[0])) if rows else b""
    for y, row in enumerate(rows):
        ft = filters[y % len(filters)]
        out.append(ft)
        for i, x in enumerate(row):
            a = row[i - bpp] if i >= bpp else 0
            b = prev[i]
            c = prev[i - bpp] if i >= bpp else 0
            pred = [0, a, b, (a + b) >> 1, _paeth(a, b, c)][ft]
            out.append((x - pred) & 0xFF)
        prev = row
    return bytes(out)


def _pack_row(samples, depth):
    if depth == 8:
        return bytes(int(s) for s in samples)
    if depth == 16:
        return b"".join(struct.pack(">H", int(s)) for s in samples)
    out, acc, n = bytearray(), 0, 0
    for s in samples:
        acc = (acc << depth) | int(s)
        n += depth
        if n == 8:
            out.append(acc); acc = 0; n = 0
    if n:
        out.append(acc << (8 - n))
    return bytes(out)


def png_bytes(samples, ctype, depth, filters=(0, 1, 2, 3, 4), palette=None, trns=None, interlace=False):
    """samples: (H, W, C) integer array of raw samples (palette indices for type 3)."""
    h, w, c = samples.shape
    bpp = max(1, c * depth // 8)

    def encode(img):
        rows = [_pack_row(img[y].reshape(-1), depth) for y in range(img.shape[0])]
        return _filter_rows(rows, bpp, filters)

    if interlace:
        raw = b""
        for x0, y0, dx, dy in ((0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2),
                               (0, 1, 1, 2)):
            sub = samples[y0::dy, x0::dx]
            if sub.shape[0] and sub.shape[1]:
                raw += encode(sub)
    else:
        raw = encode(samples)

    def chunk(k, d):
        return struct.pack(">I", len(d)) + k + d + struct.pack(">I", zlib.crc32(k + d) & 0xFFFFFFFF)
    data = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, int(interlace)))
    if palette is not None:
        data += chunk(b"PLTE", bytes(np.asarray(palette, np.uint8).reshape(-1)))
    if trns is not None:
        data += chunk(b"tRNS", bytes(trns))
    return data + chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b"")


def stbi_float(rgba8):
    """stbi__ldr_to_hdr: colour pow(v/255, 2.2), alpha v/255 (float32)."""
    f = rgba8.astype(np.float32) / np.float32(255.0)
    out = np.empty(rgba8.shape, np.float32)
    out[..., :3] = np.power(f[..., :3], np.float32(2.2))
    out[..., 3] = (rgba8[..., 3].astype(np.float32) / np.float32(255.0))
    return out


def texture_pixels(pt, scene, path, ttype=0):
    t = scene.load_texture(path, ttype)
    # read back through the packed atlas: the texture's placement in layer 0
    scene.pack()
    a = scene.arrays()
    tex = a["textures"][-1]
    p = scene.packs()
    import ctypes as C
    W, H = p.atlas_width, p.atlas_height
    atlas = np.frombuffer((C.c_float * (W * H * 4 * p.atlas_layer_count)).from_address(p.atlas),
                          dtype=np.float32).reshape(-1, H, W, 4)
    x0 = int(round(tex["AtlasPlacementMinimum"][0] * W - 0.5))
    y1 = int(round(tex["AtlasPlacementMinimum"][1] * H + 0.5))
    x1 = int(round(tex["AtlasPlacementMaximum"][0] * W + 0.5))
    y0 = int(round(tex["AtlasPlacementMaximum"][1] * H - 0.5))
    return atlas[tex["AtlasImageIndex"], y0:y1, x0:x1].copy(), t


def ulps(a, b):
    ia = a.view(np.int32).astype(np.int64)
    ib = b.view(np.int32).astype(np.int64)
    return np.abs(ia - ib)


RNG = np.random.default_rng(12)


@pytest.mark.parametrize("ctype,depth,interlace", [
    (0, 8, False), (0, 1, False), (0, 4, False), (0, 16, False), (2, 8, False), (2, 16, True),
    (4, 8, False), (6, 8, False), (6, 16, False), (6, 8, True), (3, 8, False), (3, 2, True),
])
def test_png_decoding(pt, tmp_path, ctype, depth, interlace):
    H, W = 13, 11
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    hi = (1 << depth) - 1
    palette = trns = None
    if ctype == 3:
        n = 1 << depth
        palette = RNG.integers(0, 256, size=(n, 3))
        trns = list(RNG.integers(0, 256, size=n // 2))
    samples = RNG.integers(0, hi + 1, size=(H, W, ch))
    (tmp_path / "t.png").write_bytes(png_bytes(samples, ctype, depth, palette=palette, trns=trns, interlace=interlace))
    # expected 8-bit RGBA (stb: 16 -> top byte, low depths scaled)
    to8 = (lambda s: s >> 8) if depth == 16 else (lambda s: s * (255 // hi))
    exp = np.zeros((H, W, 4), np.int64)
    if ctype == 3:
        exp[..., :3] = palette[samples[..., 0]]
        t = np.array(list(trns) + [255] * ((1 << depth) - len(trns)))
        exp[..., 3] = t[samples[..., 0]]
    elif ctype in (0, 4):
        exp[..., :3] = to8(samples[..., :1])
        exp[..., 3] = to8(samples[..., 1]) if ctype == 4 else 255
    else:
        exp[..., :3] = to8(samples[..., :3])
        exp[..., 3] = to8(samples[..., 3]) if ctype == 6 else 255
    s = pt.Scene.empty()
    got, _ = texture_pixels(pt, s, tmp_path / "t.png")
    want = stbi_float(exp.astype(np.uint8))
    assert got.shape == want.shape
    assert np.max(ulps(got, want)) <= 1
    s.close()


def test_png_color_key_transparency(pt, tmp_path):
    samples = np.array([[[10, 20, 30], [1, 2, 3]]])
    trns = struct.pack(">HHH", 1, 2, 3)
    (tmp_path / "k.png").write_bytes(png_bytes(samples, 2, 8, trns=trns))
    s = pt.Scene.empty()
    got, _ = texture_pixels(pt, s, tmp_path / "k.png")
    assert got[0, 0, 3] == 1.0 and got[0, 1, 3] == 0.0
    s.close()


def _rgbe(rgb):
    m = max(rgb)
    if m < 1e-32:
        return bytes([0, 0, 0, 0])
    mant, e = np.frexp(m)
    scale = mant * 256.0 / m
    return bytes([int(rgb[0] * scale), int(rgb[1] * scale), int(rgb[2] * scale), int(e + 128)])


@pytest.mark.parametrize("rle", [False, True])
def test_hdr_decoding(pt, tmp_path, rle):
    H, W = 5, 12
    px = RNG.uniform(0, 40, size=(H, W, 3))
    px[0, 0] = 0
    enc = np.array([[list(_rgbe(px[y, x])) for x in range(W)] for y in range(H)], np.uint8)
    body = bytearray()
    for y in range(H):
        if rle:
            body += bytes([2, 2, W >> 8, W & 0xFF])
            for c in range(4):
                row = enc[y, :, c]
                x = 0
                while x < W:                    # a run of 3, then literal dumps
                    if x + 3 <= W and row[x] == row[x + 1] == row[x + 2]:
                        body += bytes([128 + 3, row[x]]); x += 3
                    else:
                        n = min(W - x, 4)
                        body += bytes([n]) + bytes(row[x:x + n]); x += n
        else:
            body += bytes(enc[y].reshape(-1))
    data = b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n" + f"-Y {H} +X {W}\n".encode() + bytes(body)
    (tmp_path / "s.hdr").write_bytes(data)
    s = pt.Scene.empty()
    got, _ = texture_pixels(pt, s, tmp_path / "s.hdr")            # RAW: atlas holds the decoded floats
    e = enc.astype(np.float32)
    f1 = np.where(enc[..., 3] > 0, np.ldexp(np.float32(1), enc[..., 3].astype(np.int32) - 136), 0).astype(np.float32)
    want = np.concatenate([e[..., :3] * f1[..., None], np.ones((H, W, 1), np.float32)], -1)
    assert np.array_equal(got, want)
    s.close()


# --- OBJ -------------------------------------------------------------------------

CUBE_OBJ = """# a cube: quads, shared corners, two objects / materials
mtllib box.mtl
v -1 -1 -1
v 1 -1 -1
v 1 1 -1
v -1 1 -1
v -1 -1 1
v 1 -1 1
v 1 1 1
v -1 1 1
vt 0 0
vt 1 0
vt 1 1
vt 0 1
vn 0 0 -1
vn 0 0 1
o Bottom
usemtl Red
f 1/1/1 4/4/1 3/3/1 2/2/1
o Top
usemtl Blue
f -4/1/2 -3/2/2 -2/3/2 -1/4/2
usemtl Red
f 1/1/1 2/2/1 6/2/1
"""

BOX_MTL = """newmtl Red
Kd 0.8 0.1 0.1
Ke 0 0 0
newmtl Blue
Kd 0.1 0.2 0.9
map_Kd -s 1 1 1 -bm 0.5 checker.png
"""


def write_model(tmp_path, obj=CUBE_OBJ, mtl=BOX_MTL, tex=True):
    (tmp_path / "box.obj").write_text(obj)
    (tmp_path / "box.mtl").write_text(mtl)
    if tex:
        img = np.array([[[255, 255, 255, 255], [0, 0, 0, 255]], [[0, 0, 0, 255], [255, 255, 255, 255]]])
        (tmp_path / "checker.png").write_bytes(png_bytes(img, 6, 8))
    return tmp_path / "box.obj"


def test_model_import_structure(pt, tmp_path):
    path = write_model(tmp_path)
    s = pt.Scene.empty()
    prefab = s.load_model_as_prefab(path)
    meshes = s.prefab_meshes(prefab)
    # shapes: Bottom (Red), Top (Blue + Red) -> 3 (shape, material) meshes
    assert len(meshes) == 3
    faces = sorted(len(f) for _, f, _, _ in meshes)
    assert faces == [1, 2, 2]                  # the quads split into two triangles each
    for v, f, mtype, pos in meshes:
        assert mtype == 3                      # OpenPBR, as the reference imports
        assert np.all(f < len(v))
        n = v[:, 3:6]
        assert np.allclose(np.linalg.norm(n, axis=1), 1, atol=1e-6)
    # bottom quad: vertices re-centred on the shape's bounds centre
    v0 = meshes[0][0]
    assert np.allclose(v0[:, :3].mean(axis=0)[:2], 0, atol=1e-6)
    s.close()


def test_quad_split_uses_shorter_diagonal(pt, tmp_path):
    # quad whose 1-3 diagonal is shorter than 0-2: split [0,1,3], [1,2,3]
    obj = "v 0 0 0\nv 4 0 0\nv 5 1 0\nv 1 1 0\nf 1 2 3 4\n"
    (tmp_path / "q.obj").write_text(obj)
    s = pt.Scene.empty()
    (v, f, _, _), = s.prefab_meshes(s.load_model_as_prefab(tmp_path / "q.obj"))
    P = v[:, :3][f]                             # (2, 3, 3)
    tris = {tuple(sorted(map(tuple, np.round(t, 5)))) for t in P}
    c = np.array([2.5, 0.5, 0])                 # shape centre subtracted
    want = {tuple(sorted(map(tuple, np.round(np.array(t) - c, 5)))) for t in
            ([(0, 0, 0), (4, 0, 0), (1, 1, 0)], [(4, 0, 0), (5, 1, 0), (1, 1, 0)])}
    assert tris == want
    s.close()


def test_polygon_ear_clipping_covers_area(pt, tmp_path):
    # convex hexagon: 4 triangles whose areas sum to the polygon's
    ang = np.linspace(0, 2 * np.pi, 7)[:-1]
    pts = np.stack([np.cos(ang), np.sin(ang), np.zeros(6)], 1)
    obj = "".join(f"v {x:.6f} {y:.6f} {z:.6f}\n" for x, y, z in pts) + "f 1 2 3 4 5 6\n"
    (tmp_path / "h.obj").write_text(obj)
    s = pt.Scene.empty()
    (v, f, _, _), = s.prefab_meshes(s.load_model_as_prefab(tmp_path / "h.obj"))
    assert len(f) == 4
    P = v[:, :3][f].astype(np.float64)
    area = 0.5 * np.linalg.norm(np.cross(P[:, 1] - P[:, 0], P[:, 2] - P[:, 0]), axis=1).sum()
    assert abs(area - 1.5 * np.sqrt(3)) < 1e-5
    s.close()


def test_negative_indices_and_number_formats(pt, tmp_path):
    obj = ("v 1.5e0 -2.25 .5\nv +3 0.125E+1 -0.0\nv 1e-3 2 3\n"
           "vt 0.25 0.75\nf -3/-1 -2/-1 -1/-1\n")
    (tmp_path / "n.obj").write_text(obj)
    s = pt.Scene.empty()
    (v, f, _, _), = s.prefab_meshes(s.load_model_as_prefab(tmp_path / "n.obj"))
    P = np.array([[1.5, -2.25, 0.5], [3, 1.25, 0], [0.001, 2, 3]], np.float32)
    c = 0.5 * (P.min(0) + P.max(0))
    assert np.allclose(v[:, :3][f[0]], P - c, atol=1e-6)
    assert np.allclose(v[:, 6:8], [0.25, 0.75])
    s.close()


def test_import_errors(pt, tmp_path):
    s = pt.Scene.empty()
    with pytest.raises(OSError):
        s.load_model_as_prefab(tmp_path / "missing.obj")
    (tmp_path / "z.obj").write_text("v 0 0 0\nf 0 1 1\n")        # zero index
    with pytest.raises(OSError):
        s.load_model_as_prefab(tmp_path / "z.obj")
    (tmp_path / "r.obj").write_text("v 0 0 0\nf 1 2 3\n")        # out of range
    with pytest.raises(OSError):
        s.load_model_as_prefab(tmp_path / "r.obj")
    s.close()


def test_imported_scene_renders(pt, tmp_path):
    """openpbr_as_diffuse import + instancing + packing + oracle render: the
    textured box contributes (OpenPBR would render black)."""
    path = write_model(tmp_path)
    s = pt.Scene.create()
    prefab = s.load_model_as_prefab(path, openpbr_as_diffuse=True)
    e = s.instantiate_prefab(prefab)
    s.set_transform(e, position=(0, 0, 0.5), scale=(0.3, 0.3, 0.3))
    s.pack()
    a = s.arrays()
    assert len(a["shapes"]) == 1 + 3            # plane + three mesh instances
    assert len(a["textures"]) == 2              # checker plane + imported checker
    o = oracle_lib.OracleRenderer(s.packs(), 32, 16, threads=2)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    acc = o.accum()
    o.close()
    assert np.isfinite(acc).all() and acc[..., 3].sum() > 0
    s.close()
