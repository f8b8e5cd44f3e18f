"""Writes profiles/traffic.json (read by bench.py) from a committed PMC summary.

usage: python tools/update_traffic.py profiles/<run>   (expects pmc_summary.json)
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
run = Path(sys.argv[1])
s = json.loads((ROOT / run / "pmc_summary.json").read_text())
out = {"profile": str(run), "command": "tools/gpu_profile.sh (bench.py --gpus 1 --steps 20 --warmup 5: C3 1920x1080, N=1)", "kernels": {}, "issue": {}}
for k in ("extend", "raygen", "shade", "round"):
    if k not in s:
        continue
    out["kernels"][k] = {x: int(s[k][x]) for x in ("hbm_bytes", "hbm_read_bytes", "hbm_write_bytes") if x in s[k]}
    iss = {x: s[k][x] for x in ("valu_issue_frac", "valu_active_lanes") if x in s[k]}
    for x in ("SQ_INSTS_VALU", "SQ_INSTS_SALU"):
        if x in s[k]:
            iss[x.lower()] = int(s[k][x])
    if iss:
        out["issue"][k] = iss
(ROOT / "profiles" / "traffic.json").write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out, indent=1))
