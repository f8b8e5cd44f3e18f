"""Pixel partitioning for one-process-per-GPU rendering.

The image is cut into 16-row bands; band b belongs to rank b % nranks
(interleaved for load balance).  RNG streams are keyed on the
global pixel coordinate (basic_scatter.glsl:315-318), so the union of the
ranks' renders is bit-identical to a single-GPU render and the frame-end sum
over ranks is exact (disjoint supports).
"""
from __future__ import annotations

import numpy as np

BAND_ROWS = 16


def band_rows(height: int, rank: int, nranks: int) -> np.ndarray:
    """Image rows owned by `rank`."""
    rows = np.arange(height)
    return rows[(rows // BAND_ROWS) % nranks == rank]


def owned_pixels(width: int, height: int, rank: int, nranks: int) -> np.ndarray:
    """Boolean (height, width) mask of the pixels owned by `rank`."""
    mask = np.zeros((height, width), dtype=bool)
    mask[band_rows(height, rank, nranks)] = True
    return mask
