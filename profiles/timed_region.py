"""Per-kernel durations of the timed region from a rocprofv3 kernel trace.

usage: python profiles/timed_region.py run_kernel_trace.csv STEPS [OUT_JSON]

bench.py runs Reset + Run(2), SETTLE_ROUNDS, the warm-up steps, the timed
steps, then one diagnostic extend_stats launch.  The --stats summary averages
every launch of the process (the settle rounds included); this picks the
last STEPS extend / shade / round launches before the diagnostic one -- the
launches inside bench.py's timed region -- for comparison with the bench
line's HIP-event averages (roofline.launch_avg_ms).
"""
import csv
import json
import sys


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    out = {}
    for k in ("extend_kernel", "shade_kernel", "round_kernel"):
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
             if k in r["Kernel_Name"] and "stats" not in r["Kernel_Name"]]
        if d:
            last = d[-steps:]
            out[k.replace("_kernel", "")] = {"launches": len(last), "avg_ms": round(sum(last) / len(last), 4),
                                             "all_launches": len(d), "all_avg_ms": round(sum(d) / len(d), 4)}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
