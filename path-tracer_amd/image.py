"""Image writers for resolved frames (the reference presents to a window;
these write the same pixels to disk).

  write_png(path, rgba8)   8-bit RGBA (e.g. SampleBuffer.read_srgb8()), zlib-compressed
  write_ppm(path, rgba8)   binary P6, alpha dropped
  write_pfm(path, rgb)     float32 PFM (e.g. read_resolved() or raw XYZ), bottom-up rows
  read_png(path)           reader for the files write_png produces (tests)
"""
from __future__ import annotations

import struct
import zlib
from pathlib import Path

import numpy as np

_PNG_SIG = b"\x89PNG\r\n\x1a\n"


def _chunk(kind: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + kind + data + struct.pack(">I", zlib.crc32(kind + data) & 0xFFFFFFFF)


def write_png(path, rgba8: np.ndarray, level: int = 6) -> None:
    a = np.ascontiguousarray(rgba8, dtype=np.uint8)
    if a.ndim != 3 or a.shape[2] not in (3, 4):
        raise ValueError("expected (H, W, 3|4) uint8")
    h, w, c = a.shape
    raw = np.zeros((h, 1 + w * c), dtype=np.uint8)     # filter type 0 per row
    raw[:, 1:] = a.reshape(h, w * c)
    ihdr = struct.pack(">IIBBBBB", w, h, 8, 6 if c == 4 else 2, 0, 0, 0)
    data = _PNG_SIG + _chunk(b"IHDR", ihdr) + _chunk(b"IDAT", zlib.compress(raw.tobytes(), level)) + _chunk(b"IEND", b"")
    Path(path).write_bytes(data)


def read_png(path) -> np.ndarray:
    data = Path(path).read_bytes()
    if data[:8] != _PNG_SIG:
        raise ValueError("not a PNG")
    pos, idat, hdr = 8, b"", None
    while pos < len(data):
        (n,) = struct.unpack(">I", data[pos:pos + 4])
        kind, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        (crc,) = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        if zlib.crc32(kind + body) & 0xFFFFFFFF != crc:
            raise ValueError(f"bad CRC in {kind!r}")
        if kind == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif kind == b"IDAT":
            idat += body
        pos += 12 + n
    w, h, depth, ctype = hdr[0], hdr[1], hdr[2], hdr[3]
    if depth != 8 or ctype not in (2, 6):
        raise ValueError("only 8-bit RGB/RGBA written by write_png")
    c = 4 if ctype == 6 else 3
    raw = np.frombuffer(zlib.decompress(idat), dtype=np.uint8).reshape(h, 1 + w * c)
    if np.any(raw[:, 0] != 0):
        raise ValueError("only filter type 0 supported")
    return raw[:, 1:].reshape(h, w, c).copy()


def write_ppm(path, rgba8: np.ndarray) -> None:
    a = np.ascontiguousarray(rgba8, dtype=np.uint8)[..., :3]
    h, w = a.shape[:2]
    Path(path).write_bytes(f"P6\n{w} {h}\n255\n".encode() + a.tobytes())


def write_pfm(path, rgb: np.ndarray) -> None:
    a = np.ascontiguousarray(rgb, dtype=np.float32)[..., :3]
    h, w = a.shape[:2]
    body = np.ascontiguousarray(a[::-1]).astype("<f4").tobytes()   # PFM stores rows bottom-up
    Path(path).write_bytes(f"PF\n{w} {h}\n-1.0\n".encode() + body)
