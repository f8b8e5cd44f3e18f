"""Per-kernel durations of bench.py's timed frames from a rocprofv3 kernel trace.

usage: python profiles/timed_region.py run_kernel_trace.csv BENCH_JSON [OUT_JSON]

bench.py runs the warm-up frames, the timed frames (sum of the line's
frame.rounds_per_frame_rank0 rounds, one extend + shade or one fused round
launch each), then the steady-state secondary measurement (steady_state:
2 + after_rounds-2 + rounds launches, if present) and one diagnostic
extend_stats launch.  The --stats summary averages every launch of the
process; this picks the launches inside the timed frames, for comparison
with the line's HIP-event averages (roofline.launch_avg_ms, sampled every
profile_period-th round of the same frames).
"""
import csv
import json
import sys


def main():
    path, bench = sys.argv[1], json.load(open(sys.argv[2]))
    timed = sum(bench["frame"]["rounds_per_frame_rank0"])
    st = bench.get("steady_state") or {}
    tail = (st.get("after_rounds", 0) + st.get("rounds", 0)) if st else 0
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    out = {"timed_rounds": timed, "skipped_tail_rounds": tail}
    for k in ("extend_kernel", "shade_kernel", "round_kernel"):
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
             if k in r["Kernel_Name"] and "stats" not in r["Kernel_Name"]]
        if d:
            sel = d[len(d) - tail - timed:len(d) - tail]
            out[k.replace("_kernel", "")] = {"launches": len(sel), "avg_ms": round(sum(sel) / max(len(sel), 1), 4),
                                             "all_launches": len(d), "all_avg_ms": round(sum(d) / len(d), 4)}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
