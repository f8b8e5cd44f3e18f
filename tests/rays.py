"""Random ray batches for the hit-record parity checks (test infrastructure)."""
from __future__ import annotations

import numpy as np

import oracle_lib


def random_rays(arrays, n, seed):
    rng = np.random.default_rng(seed)
    shapes = arrays["shape_nodes"]
    lo = np.array([-6.0, -12.0, -1.0])
    hi = np.array([6.0, 12.0, 7.0])
    if len(shapes):
        mn = shapes[0]["Minimum"].astype(np.float64)
        mx = shapes[0]["Maximum"].astype(np.float64)
        lo = np.maximum(lo, mn - 1.0)
        hi = np.minimum(hi, mx + 1.0)
    o = rng.uniform(lo, hi, size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    # exercise the slab test's special cases: axis-aligned directions (zero
    # velocity components: infinite reciprocals, 0 * inf = NaN planes), zero
    # and tiny origin components
    axes = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1],
                     [0.6, 0.8, 0], [0, -0.6, 0.8], [1e-20, 1, 0.5]])
    d[: 9 * 32] = np.repeat(axes, 32, axis=0)
    o[64:128, 0] = 0.0
    o[128:192, 1] = 1e-30
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    vel = oracle_lib.pack_unit_vectors(d.astype(np.float32))
    dur = np.full(n, 1048576.0, dtype=np.float32)
    dur[: n // 8] = rng.uniform(0.1, 5.0, size=n // 8).astype(np.float32)
    return o, vel, dur
