"""JPEG decoding for LoadTexture (stbi_loadf, scene.cpp:294-313; decoder in
csrc/scene/jpeg.cpp).

stb_image cannot be compiled or run here, so parity with it
is unpinned; the decoder is checked three ways:
  1. exact: JPEG files written by the encoder below from chosen quantised
     coefficients (baseline, any sampling factors, restart intervals, 8- and
     16-bit tables, grey / YCbCr / Adobe RGB / CMYK / YCCK) must decode to the
     bytes a numpy restatement of stb_image's integer IDCT, upsamplers and
     colour conversion (stb_image.h:2425-2523, 3455-3526, 3645-3683,
     3858-3982) predicts;
  2. exact: libjpeg's baseline and progressive encodes of one image carry
     the same quantised coefficients, so they must decode identically
     (progressive spectral selection + successive approximation);
  3. close: libjpeg's own decode of libjpeg (Pillow) files, within the
     rounding differences of its IDCT, upsampling and colour tables (and
     stb's swapped last-pair weights in horizontal 2x upsampling, skipped).
"""
from __future__ import annotations

import heapq
import struct

import numpy as np
import pytest

PIL = pytest.importorskip("PIL.Image")

ZIGZAG = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
                   13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52,
                   45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])


# --- a small baseline JPEG encoder (ISO/IEC 10918-1 Annex F, B) -------------------

class BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, code, length):
        for i in range(length - 1, -1, -1):
            self.acc = (self.acc << 1) | ((code >> i) & 1)
            self.n += 1
            if self.n == 8:
                self.out.append(self.acc)
                if self.acc == 0xFF:
                    self.out.append(0)       # byte stuffing
                self.acc = self.n = 0

    def flush(self):
        while self.n:
            self.put(1, 1)                   # pad with 1-bits


def huffman_table(freq, spare):
    """Code lengths (<= 16) from symbol frequencies, plus an unused symbol
    `spare` placed last so that no used code is all 1-bits; returns
    (counts[16], symbols, {sym: (code, len)})."""
    assert spare not in freq
    syms = sorted(freq) + [None]
    w = {s: freq.get(s, 1) for s in syms}
    heap = [(w[s], i, [s]) for i, s in enumerate(syms)]
    heapq.heapify(heap)
    depth = {s: 0 for s in syms}
    if len(heap) == 1:
        depth[syms[0]] = 1
    k = len(heap)
    while len(heap) > 1:
        a, b = heapq.heappop(heap), heapq.heappop(heap)
        for s in a[2] + b[2]:
            depth[s] += 1
        heapq.heappush(heap, (a[0] + b[0], k, a[2] + b[2]))
        k += 1
    assert max(depth.values()) <= 16
    order = sorted(syms, key=lambda s: (depth[s], s is None, s if s is not None else 0))
    counts = [0] * 16
    for s in order:
        counts[depth[s] - 1] += 1
    codes, code, prev = {}, 0, depth[order[0]]
    for s in order:
        code <<= depth[s] - prev
        prev = depth[s]
        codes[s] = (code, depth[s])
        code += 1
    return counts, [spare if s is None else s for s in order], codes


def category(v):
    return 0 if v == 0 else int(abs(v)).bit_length()


def vlc_bits(v, s):
    return v if v >= 0 else v + (1 << s) - 1


def encode_jpeg(planes, comps, quant, restart=0, ids=None, adobe=None, jfif=True):
    """planes[c]: int array (by, bx, 64) of quantised coefficients in
    row-major (natural) order; comps[c] = (h, v, tq).  Interleaved baseline
    scan unless one component."""
    ncomp = len(comps)
    hmax = max(h for h, v, t in comps)
    vmax = max(v for h, v, t in comps)
    mcuy, mcux = planes[0].shape[0] // comps[0][1], planes[0].shape[1] // comps[0][0]
    width, height = encode_jpeg.size
    # symbols for the tables
    order = []
    for j in range(mcuy):
        for i in range(mcux):
            for c, (h, v, t) in enumerate(comps):
                for y in range(v):
                    for x in range(h):
                        order.append((c, j * v + y, i * h + x))
            if ncomp == 1:
                pass
    dfreq, afreq = {}, {}
    pred = [0] * ncomp
    seq = []
    for n, (c, by, bx) in enumerate(order):
        if restart and n % (restart * sum(h * v for h, v, t in comps)) == 0:
            pred = [0] * ncomp
        blk = planes[c][by, bx][ZIGZAG]
        diff = int(blk[0]) - pred[c]
        pred[c] = int(blk[0])
        s = category(diff)
        dfreq[s] = dfreq.get(s, 0) + 1
        acs, run = [], 0
        last = max([k for k in range(1, 64) if blk[k] != 0], default=0)
        for k in range(1, last + 1):
            if blk[k] == 0:
                run += 1
                continue
            while run > 15:
                acs.append((0xF0, 0, 0))
                run -= 16
            sz = category(int(blk[k]))
            acs.append(((run << 4) | sz, int(blk[k]), sz))
            run = 0
        if last < 63:
            acs.append((0x00, 0, 0))
        for sym, _, _ in acs:
            afreq[sym] = afreq.get(sym, 0) + 1
        seq.append((c, diff, s, acs))
    dcnt, dsym, dcode = huffman_table(dfreq, max(set(range(16)) - set(dfreq)))
    acnt, asym, acode = huffman_table(afreq, max(set(range(256)) - set(afreq)))
    out = bytearray(b"\xFF\xD8")
    if jfif:
        out += b"\xFF\xE0" + struct.pack(">H", 16) + b"JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00"
    if adobe is not None:
        out += b"\xFF\xEE" + struct.pack(">H", 14) + b"Adobe\x00" + bytes([100, 0, 0, 0, 0, adobe])
    for t, q in quant.items():
        if q.max() > 255:
            out += b"\xFF\xDB" + struct.pack(">HB", 2 + 129, 0x10 | t) + b"".join(struct.pack(">H", int(x)) for x in q[ZIGZAG])
        else:
            out += b"\xFF\xDB" + struct.pack(">HB", 2 + 65, t) + bytes(int(x) for x in q[ZIGZAG])
    ids = ids or list(range(1, ncomp + 1))
    out += b"\xFF\xC0" + struct.pack(">HBHHB", 8 + 3 * ncomp, 8, height, width, ncomp)
    for c, (h, v, t) in enumerate(comps):
        out += bytes([ids[c], (h << 4) | v, t])
    for tc, (cnt, sym) in enumerate([(dcnt, dsym), (acnt, asym)]):
        out += b"\xFF\xC4" + struct.pack(">HB", 2 + 17 + len(sym), tc << 4) + bytes(cnt) + bytes(sym)
    if restart:
        out += b"\xFF\xDD" + struct.pack(">HH", 4, restart)
    out += b"\xFF\xDA" + struct.pack(">HB", 6 + 2 * ncomp, ncomp)
    for c in range(ncomp):
        out += bytes([ids[c], 0x00])
    out += bytes([0, 63, 0])
    bw = BitWriter()
    blocks_per_mcu = sum(h * v for h, v, t in comps)
    rst = 0
    for n, (c, diff, s, acs) in enumerate(seq):
        if restart and n and n % (restart * blocks_per_mcu) == 0:
            bw.flush()
            bw.out += bytes([0xFF, 0xD0 + rst])
            rst = (rst + 1) & 7
        code, ln = dcode[s]
        bw.put(code, ln)
        if s:
            bw.put(vlc_bits(diff, s), s)
        for sym, val, sz in acs:
            code, ln = acode[sym]
            bw.put(code, ln)
            if sz:
                bw.put(vlc_bits(val, sz), sz)
    bw.flush()
    return bytes(out + bw.out + b"\xFF\xD9")


# --- numpy restatement of stb_image's output stage --------------------------------

def f2f(x):
    return int(np.float32(x) * np.float32(4096) + 0.5)


def idct_1d(s):
    """STBI__IDCT_1D on an array (..., 8) of ints: (x0..x3, t0..t3)."""
    s0, s1, s2, s3, s4, s5, s6, s7 = [s[..., i].astype(np.int64) for i in range(8)]
    p1 = (s2 + s6) * f2f(0.5411961)
    t2 = p1 + s6 * f2f(-1.847759065)
    t3 = p1 + s2 * f2f(0.765366865)
    t0 = (s0 + s4) * 4096
    t1 = (s0 - s4) * 4096
    x0, x3, x1, x2 = t0 + t3, t0 - t3, t1 + t2, t1 - t2
    o0, o1, o2, o3 = s7, s5, s3, s1
    p3, p4, pa, pb = o0 + o2, o1 + o3, o0 + o3, o1 + o2
    p5 = (p3 + p4) * f2f(1.175875602)
    o0 = o0 * f2f(0.298631336)
    o1 = o1 * f2f(2.053119869)
    o2 = o2 * f2f(3.072711026)
    o3 = o3 * f2f(1.501321110)
    pa = p5 + pa * f2f(-0.899976223)
    pb = p5 + pb * f2f(-2.562915447)
    p3 = p3 * f2f(-1.961570560)
    p4 = p4 * f2f(-0.390180644)
    return x0, x1, x2, x3, o0 + pa + p3, o1 + pb + p4, o2 + pb + p3, o3 + pa + p4


def stb_idct(blocks):
    """stbi__idct_block over (..., 64) dequantised coefficients -> (..., 8, 8) uint8."""
    d = blocks.reshape(blocks.shape[:-1] + (8, 8)).astype(np.int64)
    cols = np.swapaxes(d, -1, -2)                      # (..., column, row)
    x0, x1, x2, x3, t0, t1, t2, t3 = idct_1d(cols)
    x0, x1, x2, x3 = x0 + 512, x1 + 512, x2 + 512, x3 + 512
    v = np.stack([(x0 + t3) >> 10, (x1 + t2) >> 10, (x2 + t1) >> 10, (x3 + t0) >> 10,
                  (x3 - t0) >> 10, (x2 - t1) >> 10, (x1 - t2) >> 10, (x0 - t3) >> 10], -1)
    flat = (cols[..., 1:] == 0).all(-1)
    v = np.where(flat[..., None], (cols[..., 0] * 4)[..., None], v)
    rows = np.swapaxes(v, -1, -2)                      # (..., row, column)
    x0, x1, x2, x3, t0, t1, t2, t3 = idct_1d(rows)
    b = 65536 + (128 << 17)
    x0, x1, x2, x3 = x0 + b, x1 + b, x2 + b, x3 + b
    o = np.stack([(x0 + t3) >> 17, (x1 + t2) >> 17, (x2 + t1) >> 17, (x3 + t0) >> 17,
                  (x3 - t0) >> 17, (x2 - t1) >> 17, (x1 - t2) >> 17, (x0 - t3) >> 17], -1)
    return np.clip(o, 0, 255).astype(np.uint8)


def plane_of(coefs, q):
    """Component samples (h2 x w2) from (by, bx, 64) natural-order coefficients."""
    deq = (coefs.astype(np.int64) * q.astype(np.int64)).astype(np.int16)
    px = stb_idct(deq)                                   # (by, bx, 8, 8)
    by, bx = coefs.shape[:2]
    return px.transpose(0, 2, 1, 3).reshape(by * 8, bx * 8)


def upsample(plane, hs, vs, W, H, cy):
    """load_jpeg_image's row loop with the resample_row_* kernels."""
    wl = (W + hs - 1) // hs
    out = np.zeros((H, W), np.int64)
    line0 = line1 = 0
    ystep, ypos = vs >> 1, 0
    for j in range(H):
        bottom = ystep >= (vs >> 1)
        near = plane[line1 if bottom else line0, :wl].astype(np.int64)
        far = plane[line0 if bottom else line1, :wl].astype(np.int64)
        if hs == 1 and vs == 1:
            row = near
        elif hs == 1 and vs == 2:
            row = (3 * near + far + 2) >> 2
        elif hs == 2 and vs == 1:
            row = np.zeros(2 * wl, np.int64)
            if wl == 1:
                row[:] = near[0]
            else:
                row[0] = near[0]
                row[1] = (near[0] * 3 + near[1] + 2) >> 2
                i = np.arange(1, wl - 1)
                row[2 * i] = (3 * near[i] + 2 + near[i - 1]) >> 2
                row[2 * i + 1] = (3 * near[i] + 2 + near[i + 1]) >> 2
                row[2 * (wl - 1)] = (near[wl - 2] * 3 + near[wl - 1] + 2) >> 2
                row[2 * (wl - 1) + 1] = near[wl - 1]
        elif hs == 2 and vs == 2:
            t = 3 * near + far
            row = np.zeros(2 * wl, np.int64)
            if wl == 1:
                row[:] = (t[0] + 2) >> 2
            else:
                row[0] = (t[0] + 2) >> 2
                row[1:2 * wl - 1:2] = (3 * t[:-1] + t[1:] + 8) >> 4
                row[2:2 * wl - 1:2] = (3 * t[1:] + t[:-1] + 8) >> 4
                row[2 * wl - 1] = (t[-1] + 2) >> 2
        else:
            row = np.repeat(near, hs)
        out[j] = row[:W]
        ystep += 1
        if ystep >= vs:
            ystep = 0
            line0 = line1
            ypos += 1
            if ypos < cy:
                line1 += 1
    return out


def f2fixed(x):
    return int(np.float32(x) * np.float32(4096.0) + np.float32(0.5)) << 8


def ycc(y, cb, cr):
    yf = (y << 20) + (1 << 19)
    cr, cb = cr - 128, cb - 128
    r = (yf + cr * f2fixed(1.40200)) >> 20
    # (C: int & 0xffff0000u, back to int: the low 16 bits cleared, the sign kept)
    g = (yf + cr * -f2fixed(0.71414) + ((cb * -f2fixed(0.34414)) & -65536)) >> 20
    b = (yf + cb * f2fixed(1.77200)) >> 20
    return [np.clip(c, 0, 255) for c in (r, g, b)]


def blinn(x, y):
    t = x * y + 128
    return (t + (t >> 8)) >> 8


def stb_expected(planes, comps, quant, W, H, mode):
    hmax = max(h for h, v, t in comps)
    vmax = max(v for h, v, t in comps)
    full = []
    for c, (h, v, t) in enumerate(comps):
        cy = (H * v + vmax - 1) // vmax
        full.append(upsample(plane_of(planes[c], quant[t]), hmax // h, vmax // v, W, H, cy))
    out = np.full((H, W, 4), 255, np.int64)
    if len(comps) == 1:
        out[..., 0] = out[..., 1] = out[..., 2] = full[0]
    elif mode == "rgb":
        out[..., :3] = np.stack(full[:3], -1)
    elif mode == "cmyk":
        for k in range(3):
            out[..., k] = blinn(full[k], full[3])
    else:
        r, g, b = ycc(full[0], full[1], full[2])
        if mode == "ycck":
            r, g, b = [blinn(255 - c, full[3]) for c in (r, g, b)]
        out[..., 0], out[..., 1], out[..., 2] = r, g, b
    return out.astype(np.uint8)


def random_planes(rng, comps, W, H, amp=12, density=0.25):
    hmax = max(h for h, v, t in comps)
    vmax = max(v for h, v, t in comps)
    mcux, mcuy = -(-W // (8 * hmax)), -(-H // (8 * vmax))
    planes = []
    for h, v, t in comps:
        shape = (mcuy * v, mcux * h, 64)
        c = rng.integers(-amp, amp + 1, size=shape)
        c *= rng.random(shape) < density
        c[..., 0] = rng.integers(-40, 41, size=shape[:2])
        # decaying high frequencies, as real images have
        c[..., 1:] = c[..., 1:] // (1 + np.arange(1, 64) // 8)
        planes.append(c)
    return planes


CASES = [
    # (W, H, comps (h, v, tq), mode, restart, q16, ids, adobe)
    (16, 16, [(1, 1, 0)], "grey", 0, False, None, None),
    (37, 21, [(1, 1, 0)], "grey", 3, True, None, None),
    (40, 24, [(1, 1, 0), (1, 1, 1), (1, 1, 1)], "ycc", 0, False, None, None),
    (33, 17, [(2, 2, 0), (1, 1, 1), (1, 1, 1)], "ycc", 2, False, None, None),      # 4:2:0, ragged
    (35, 19, [(2, 1, 0), (1, 1, 1), (1, 1, 1)], "ycc", 0, False, None, None),      # 4:2:2
    (29, 30, [(1, 2, 0), (1, 1, 1), (1, 1, 1)], "ycc", 1, True, None, None),       # 4:4:0
    (45, 9, [(4, 1, 0), (1, 1, 1), (1, 1, 1)], "ycc", 0, False, None, None),       # 4:1:1 (nearest)
    (1, 1, [(2, 2, 0), (1, 1, 1), (1, 1, 1)], "ycc", 0, False, None, None),
    (3, 5, [(2, 1, 0), (1, 1, 1), (1, 1, 1)], "ycc", 0, False, None, None),
    (24, 16, [(1, 1, 0), (1, 1, 0), (1, 1, 0)], "rgb", 0, False, [82, 71, 66], None),   # ids 'R','G','B'
    (24, 16, [(1, 1, 0), (1, 1, 0), (1, 1, 0)], "rgb", 0, False, None, 0),             # Adobe transform 0
    (20, 18, [(1, 1, 0), (1, 1, 0), (1, 1, 0), (1, 1, 0)], "cmyk", 0, False, None, 0),
    (20, 18, [(2, 2, 0), (1, 1, 1), (1, 1, 1), (2, 2, 0)], "ycck", 0, False, None, 2),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_exact_against_stb_restatement(pt, tmp_path, case):
    W, H, comps, mode, restart, q16, ids, adobe = CASES[case]
    rng = np.random.default_rng(100 + case)
    quant = {0: rng.integers(1, 40, 64), 1: rng.integers(1, 60, 64)}
    if q16:
        quant[0][5] = 300          # forces a 16-bit table
    planes = random_planes(rng, comps, W, H)
    encode_jpeg.size = (W, H)
    data = encode_jpeg(planes, comps, quant, restart=restart, ids=ids, adobe=adobe,
                       jfif=mode not in ("rgb", "cmyk", "ycck") or ids is not None)
    p = tmp_path / "t.jpg"
    p.write_bytes(data)
    got = pt.load_image_rgba8(p)
    want = stb_expected(planes, comps, quant, W, H, mode)
    assert got.shape == want.shape
    bad = np.argwhere(got != want)
    assert bad.size == 0, f"{len(bad)} samples differ, first at {bad[:3].tolist()}"


def pil_image(seed, W, H):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:H, 0:W]
    im = np.stack([128 + 100 * np.sin(x / 7.0 + seed), 128 + 90 * np.cos(y / 5.0), (x * y) % 256], -1)
    im += rng.normal(0, 12, im.shape)
    im[: H // 3, : W // 2] = [200, 40, 90]
    return np.clip(im, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("sub", [0, 1, 2])
@pytest.mark.parametrize("W,H", [(61, 43), (128, 96), (9, 7)])
def test_progressive_decodes_like_baseline(pt, tmp_path, sub, W, H):
    """libjpeg's progressive script (DC first + refinement, AC spectral bands
    with successive approximation) stores the baseline encode's coefficients."""
    from PIL import Image
    im = Image.fromarray(pil_image(W + sub, W, H))
    out = {}
    for prog in (False, True):
        p = tmp_path / f"p{int(prog)}.jpg"
        im.save(p, quality=85, subsampling=sub, progressive=prog)
        out[prog] = pt.load_image_rgba8(p)
    assert np.array_equal(out[False], out[True])


@pytest.mark.parametrize("mode,sub", [("L", 0), ("RGB", 0), ("RGB", 1), ("RGB", 2)])
@pytest.mark.parametrize("q,opt,prog", [(95, False, False), (50, True, False), (10, False, True), (75, True, True)])
def test_close_to_libjpeg(pt, tmp_path, mode, sub, q, opt, prog):
    from PIL import Image
    arr = pil_image(q, 83, 57)
    im = Image.fromarray(arr).convert(mode)
    p = tmp_path / "c.jpg"
    kw = {} if mode == "L" else {"subsampling": sub}
    im.save(p, quality=q, optimize=opt, progressive=prog, **kw)
    got = pt.load_image_rgba8(p).astype(int)
    ref = np.asarray(Image.open(p).convert("RGB")).astype(int)
    assert (got[..., 3] == 255).all()
    d = np.abs(got[..., :3] - ref)
    if mode == "RGB" and sub == 1:
        d = d[:, :-2]          # stb weights the last horizontal pair (in[w-2]*3 + in[w-1]), libjpeg the reverse
    assert d.max() <= 4 and d.mean() < 0.35, (d.max(), d.mean())


def test_restart_markers_and_texture_path(pt, tmp_path):
    """libjpeg restart intervals decode like the uninterrupted file, and a
    JPEG goes through LoadTexture (stbi_loadf linearisation)."""
    from PIL import Image
    from test_ingestion import stbi_float, texture_pixels, ulps
    im = Image.fromarray(pil_image(3, 70, 50))
    a, b = tmp_path / "a.jpg", tmp_path / "b.jpg"
    im.save(a, quality=80)
    try:
        im.save(b, quality=80, restart_marker_blocks=3)
    except TypeError:
        pytest.skip("this Pillow cannot write restart markers")
    assert b.read_bytes().count(b"\xFF\xD0") >= 1
    ra, rb = pt.load_image_rgba8(a), pt.load_image_rgba8(b)
    assert np.array_equal(ra, rb)
    s = pt.Scene.empty()
    got, _ = texture_pixels(pt, s, b)
    assert np.max(ulps(got, stbi_float(rb))) <= 1
    s.close()


def test_corrupt_and_truncated_streams(pt, tmp_path):
    from PIL import Image
    im = Image.fromarray(pil_image(5, 64, 48))
    p = tmp_path / "t.jpg"
    im.save(p, quality=80)
    data = p.read_bytes()
    q = tmp_path / "trunc.jpg"
    q.write_bytes(data[: len(data) * 2 // 3])      # no EOI: the decoded part is kept
    t = pt.load_image_rgba8(q)
    full = pt.load_image_rgba8(p)
    assert t.shape == full.shape and np.array_equal(t[:8], full[:8])
    r = tmp_path / "bad.jpg"
    r.write_bytes(b"\xFF\xD8\xFF\xC0\x00\x0B\x0C")   # 12-bit precision
    with pytest.raises(ValueError):
        pt.load_image_rgba8(r)
    r.write_bytes(b"\xFF\xD8" + b"\x00" * 16)
    with pytest.raises(ValueError):
        pt.load_image_rgba8(r)
