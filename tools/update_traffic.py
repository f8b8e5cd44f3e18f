"""Writes one config's entry of profiles/traffic.json (read by bench.py:
roofline.traffic and limiter of that config's line) from a committed PMC
summary.

usage: python tools/update_traffic.py KEY profiles/<run> ["command"] [ROUNDS_PER_BATCH]
       (profiles/<run>/pmc_summary.json from profiles/pmc_summary.py)
KEY: the config ("3"), or a band partition "CONFIG:bandsNxK" (rank 0 of N with
K path streams).  ROUNDS_PER_BATCH: rounds each round-batch launch of the
profile covered; the batch kernel's ("rounds") bytes and instruction counts
are then stored per round, as bench.py reports its time.
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
config, run = sys.argv[1], Path(sys.argv[2])
command = sys.argv[3] if len(sys.argv) > 3 else f"tools/gpu_profile.sh (bench.py --config {config}, N=1)"
per_batch = int(sys.argv[4]) if len(sys.argv) > 4 else 1
s = json.loads((ROOT / run / "pmc_summary.json").read_text())
entry = {"profile": str(run), "command": command, "kernels": {}, "issue": {}}
if per_batch > 1:
    entry["rounds_per_batch_launch"] = per_batch
for k in ("extend", "raygen", "shade", "round", "rounds"):
    if k not in s:
        continue
    div = per_batch if k == "rounds" else 1    # per round
    entry["kernels"][k] = {x: int(s[k][x] / div) for x in ("hbm_bytes", "hbm_read_bytes", "hbm_write_bytes")
                           if x in s[k]}
    if "dispatch_ms" in s[k]:
        entry["kernels"][k]["dispatch_ms"] = s[k]["dispatch_ms"] / div   # the profiled, serialised dispatch
    iss = {x: s[k][x] for x in ("valu_issue_frac", "valu_active_lanes", "l2_hit_rate") if x in s[k]}
    for x in ("SQ_INSTS_VALU", "SQ_INSTS_SALU"):
        if x in s[k]:
            iss[x.lower()] = int(s[k][x] / div)
    if iss:
        entry["issue"][k] = iss
path = ROOT / "profiles" / "traffic.json"
d = json.loads(path.read_text()) if path.exists() else {}
d.setdefault("configs", {})[str(config)] = entry
path.write_text(json.dumps(d, indent=1) + "\n")
print(json.dumps(entry, indent=1))
