"""Build the native libraries in-tree (no JIT cache: the .so files travel with
the repository snapshot to the GPU box).

  libptscene.so     host scene API + PackSceneData + spectrum table (g++)
  libpathtracer.so  HIP kernels for gfx950 + C-ABI runtime + RCCL (hipcc)

The oracle (test infrastructure) is built separately by oracle/Makefile.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"

SCENE_SRC = sorted((CSRC / "scene").glob("*.cpp"))
SCENE_HDR = sorted((CSRC / "scene").glob("*.hpp")) + sorted(INCLUDE.glob("*.h"))
HIP_SRC = [CSRC / "hip" / "kernels.hip", CSRC / "hip" / "resolve.hip", CSRC / "hip" / "preview.hip",
           CSRC / "hip" / "runtime.hip"]
HIP_HDR = sorted((CSRC / "hip").glob("*.hpp")) + sorted(INCLUDE.glob("*.h"))

SCENE_LIB = PKG / "libptscene.so"
HIP_LIB = PKG / "libpathtracer.so"

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("PT_OFFLOAD_ARCH", "gfx950")


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], check=True)


def build_scene(force=False, verbose=True):
    if not force and not _stale(SCENE_LIB, SCENE_SRC + SCENE_HDR + [Path(__file__)]):
        return SCENE_LIB
    cmd = ["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-Wall",
           "-Wno-unused-function", "-o", SCENE_LIB] + SCENE_SRC + ["-lpthread", "-lz"]
    _run(cmd, verbose)
    return SCENE_LIB


def build_hip(force=False, verbose=True, out=None, extra=()):
    out = Path(out) if out else HIP_LIB
    if not force and not _stale(out, HIP_SRC + HIP_HDR + [Path(__file__)]):
        return out
    flags = [f"--offload-arch={ARCH}", "-std=c++17", "-O3", "-fPIC",
             # -fno-slp-vectorize: no v_pk_* f32 packing (and its operand moves);
             # shade 0.164 -> 0.156 ms on C3, extend unchanged (tools/gpu_ab.sh).
             "-ffp-contract=off", "-fno-gpu-rdc", "-munsafe-fp-atomics", "-fno-slp-vectorize",
             "-Wno-unused-result", *extra]
    # One object per source, compiled concurrently, then one link.
    import concurrent.futures
    import tempfile
    with tempfile.TemporaryDirectory(prefix="pt_build_") as tmp:
        objs = [Path(tmp) / (src.stem + ".o") for src in HIP_SRC]
        with concurrent.futures.ThreadPoolExecutor(max_workers=min(len(HIP_SRC), os.cpu_count() or 1)) as ex:
            jobs = [ex.submit(_run, [HIPCC, *flags, "-c", str(src), "-o", str(obj)], verbose)
                    for src, obj in zip(HIP_SRC, objs)]
            for j in jobs:
                j.result()
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fno-gpu-rdc", "-o", str(out), *map(str, objs),
              f"-L{ROCM}/lib", "-lrccl"], verbose)
    return out


def build_all(force=False, verbose=True):
    build_scene(force, verbose)
    build_hip(force, verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
