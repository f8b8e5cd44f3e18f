"""Filtered-slab-test ambiguity rate on real path rays (CPU experiment).

Renders C3 (or --config) with the CPU oracle for a few rounds, takes the
slots' current rays (world space == object space: the room mesh instance has
the identity transform) and runs tools/exp_filter.cpp over them: the share of
internal BLAS steps whose box-pair decision a one-FMA-per-plane slab test
with an error margin could not certify (the kernel's fallback rate).
usage: python tools/exp_filter.py [--config 3] [--w 320 --h 180] [--rounds 6]
"""
import argparse
import ctypes as C
import importlib.util
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--w", type=int, default=320)
    ap.add_argument("--h", type=int, default=180)
    ap.add_argument("--rounds", type=int, default=6)
    args = ap.parse_args()
    so = "/tmp/exp_filter.so"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-o", so,
                    str(ROOT / "tools" / "exp_filter.cpp")], check=True)
    spec = importlib.util.spec_from_file_location("path_tracer_amd", ROOT / "path-tracer_amd" / "__init__.py",
                                                  submodule_search_locations=[str(ROOT / "path-tracer_amd")])
    pt = importlib.util.module_from_spec(spec)
    sys.modules["path_tracer_amd"] = pt
    spec.loader.exec_module(pt)
    import oracle_lib
    import kat
    s = pt.Scene.config(args.config)
    arr = s.arrays()
    nodes = np.ascontiguousarray(arr["mesh_nodes"])
    faces = np.ascontiguousarray(arr["mesh_faces"])
    shapes = arr["shapes"]
    mesh = [sh for sh in shapes if sh["Type"] == 3] if False else list(shapes)
    root = int(shapes[0]["MeshRootNodeIndex"])
    o = oracle_lib.OracleRenderer(s.packs(), args.w, args.h)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    lib = C.CDLL(so)
    lib.exp_filter.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_float,
                               C.c_float, C.c_void_p]
    for K in (8.0, 16.0):
        tot = np.zeros(9, dtype=np.uint64)
        o2 = oracle_lib.OracleRenderer(s.packs(), args.w, args.h)
        o2.RenderFlags = 3
        o2.reset()
        o2.run(2)
        for rr in range(args.rounds):
            st = o2.state().reshape(-1)
            O = np.ascontiguousarray(st["origin"], dtype=np.float32)
            V = np.ascontiguousarray(kat.unpack_unit_vector(st["packed_velocity"]), dtype=np.float32)
            stats = np.zeros(9, dtype=np.uint64)
            lib.exp_filter(nodes.ctypes.data, faces.ctypes.data, root, len(O), O.ctypes.data, V.ctypes.data,
                           np.float32(1e30), K, stats.ctypes.data)
            tot += stats
            o2.run(1)
        o2.close()
        t = tot.astype(float)
        print(f"K={K:g}: rays {int(t[7])}, internal steps {int(t[0])} ({t[0]/t[7]:.1f}/ray), "
              f"ambiguous {t[1]/t[0]*100:.3f} % (order {t[3]/t[0]*100:.3f} %, x-e {t[4]/t[0]*100:.3f} %, "
              f"x {t[5]/t[0]*100:.3f} %, reach-e {t[6]/t[0]*100:.3f} %), exact TA==TB ties {t[8]/t[0]*100:.3f} %, "
              f"ROBUST-BUT-WRONG {int(t[2])}")
    o.close()


if __name__ == "__main__":
    main()
