"""Regenerates the fixtures in tests/golden/.

  pcg.json            Random() streams from the numpy restatement (tests/kat.py)
  unit_vectors.npz    PackUnitVector / UnpackUnitVector of 64 directions (kat.py)
  fp_convention.npz   bit patterns of the pt_fp.h transcendentals (oracle)
  scene_packs.json    sha256 of every packed buffer of configs 1,2,3,5 (packer)
  c1_oracle.npz       C1 at 48x32: slot state + accumulator after Reset, Run(2),
                      Run(1) (oracle)

The reference cannot be built or run here and ships no fixtures (SURVEY.md
§8(c)), so pcg/unit_vectors are known answers from the published formulas and
the rest pin this build's own oracle and packer against regressions.
Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
import conftest  # noqa: E402,F401  (package loader + spectrum table path)
import kat  # noqa: E402
import oracle_lib  # noqa: E402

PCG_SEEDS = [0, 1, 277803737, 0xFFFFFFFF, kat.seed(17, 5, 3)]
FP_RANGES = {"exp": (-80, 80), "log": (1e-30, 1e30), "sin": (-100, 100), "cos": (-100, 100), "asin": (-1, 1)}


def directions():
    d = [[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]]
    d += [[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]
    n = 64 - len(d)
    i = np.arange(n) + 0.5
    phi = np.arccos(1 - 2 * i / n)
    th = np.pi * (1 + 5 ** 0.5) * i
    d += np.stack([np.cos(th) * np.sin(phi), np.sin(th) * np.sin(phi), np.cos(phi)], 1).tolist()
    d = np.array(d, dtype=np.float64)
    return (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)


def scene_hashes(pt):
    out = {}
    for cfg in (1, 2, 3, 5):
        s = pt.Scene.config(cfg)
        arr = s.arrays()
        out[str(cfg)] = {k: hashlib.sha256(v.tobytes()).hexdigest() for k, v in arr.items()}
        out[str(cfg)]["counts"] = {k: int(len(v)) for k, v in arr.items()}
        s.close()
    return out


def c1_oracle(pt):
    s = pt.Scene.config(1)
    o = oracle_lib.OracleRenderer(s.packs(), 48, 32, threads=4)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    o.run(1)
    return o.state(), o.accum()


def main():
    pt = conftest.load_package()
    (HERE / "pcg.json").write_text(json.dumps(
        {"source": "common.glsl.inc:189-196", "streams": [{"seed": s, "outputs": kat.pcg_stream(s, 16)}
                                                          for s in PCG_SEEDS]}, indent=1) + "\n")
    d = directions()
    p = kat.pack_unit_vector(d)
    np.savez(HERE / "unit_vectors.npz", directions=d, packed=p, unpacked=kat.unpack_unit_vector(p))
    rng = np.random.default_rng(2024)
    fp = {}
    L = oracle_lib.lib()
    for name, (lo, hi) in FP_RANGES.items():
        if name == "log":
            x = np.exp(rng.uniform(np.log(lo), np.log(hi), 256)).astype(np.float32)
        else:
            x = rng.uniform(lo, hi, 256).astype(np.float32)
        f = getattr(L, f"oracle_fp_{name}")
        fp[f"{name}_x"] = x
        fp[f"{name}_y"] = np.array([f(float(v)) for v in x], dtype=np.float32)
    np.savez(HERE / "fp_convention.npz", **fp)
    (HERE / "scene_packs.json").write_text(json.dumps(scene_hashes(pt), indent=1, sort_keys=True) + "\n")
    state, accum = c1_oracle(pt)
    np.savez_compressed(HERE / "c1_oracle.npz", state=state.view(np.uint8), accum=accum)
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
