"""Matches the extend dispatches of a `rocprofv3 --kernel-trace` run of
tools/exp_reorder.py to its ray orders and prints mean duration per order."""
import csv
import glob
import json
import sys
from collections import defaultdict

d = sys.argv[1]
orders = json.load(open("gpurun_out/exp_reorder_orders.json"))
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "extend_kernel" in row["Kernel_Name"] and "ray_source_arrays" in row["Kernel_Name"]:
            rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
rows.sort()
print(len(rows), "extend(arrays) dispatches,", len(orders), "trace calls")
rows = rows[-len(orders):]
acc = defaultdict(list)
for o, (s, e) in zip(orders, rows):
    acc[o["order"]].append((e - s) / 1e6)
base = min(acc["slot"] + acc.get("slot_again", []))
for k, v in acc.items():
    print(f"{k:26s} best {min(v):.4f} ms  mean {sum(v)/len(v):.4f} ms  vs slot {min(v)/base:.3f}")
