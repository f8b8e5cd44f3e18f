"""Build an alternative libpathtracer.so with extra compiler flags for A/B
timing on the GPU box (load it with PT_HIP_LIB=<path>).

usage: python tools/build_variant.py NAME [hipcc flags...]
       -> build/variants/NAME.so
"""
import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
spec = importlib.util.spec_from_file_location("pt_build", ROOT / "path-tracer_amd" / "build.py")
b = importlib.util.module_from_spec(spec)
spec.loader.exec_module(b)
name, flags = sys.argv[1], sys.argv[2:]
out = ROOT / "build" / "variants" / f"{name}.so"
out.parent.mkdir(parents=True, exist_ok=True)
b.build_hip(force=True, out=out, extra=flags)
print(out)
