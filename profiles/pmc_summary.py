"""Summarises rocprofv3 --pmc CSVs per kernel and derives HBM traffic.

usage: python profiles/pmc_summary.py OUT_JSON counter_collection.csv [...]

Per kernel: every counter summed over its dimensions within a dispatch, then
averaged over dispatches.  HBM bytes per launch follow MI355X_MICROARCH.md
§HBM: FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half
the bytes of wide (16 B/lane) coalesced reads, so it is doubled; WRITE_SIZE is
exact for 16-B/lane stores.  Both come from separate --pmc passes.
"""
import collections
import csv
import json
import sys


def load(path):
    per = collections.defaultdict(float)
    names = {}
    span = {}
    for r in csv.DictReader(open(path)):
        key = (r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            span[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (d, c), v in per.items():
        agg[names[d]][c].append(v)
    # The profiled dispatches' own durations (rocprofv3 serialises them):
    # the time the counters of the same dispatches accrued in.
    for d, ns in span.items():
        agg[names[d]]["dispatch_ns"].append(float(ns))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


def short(name):
    for k in ("class_list", "shade_classq", "extend", "shade", "raygen", "finalize", "rounds", "round"):
        if f"{k}_kernel" in name:
            return k
    return name[:40]


def main():
    out_path, paths = sys.argv[1], sys.argv[2:]
    kernels = {}
    for p in paths:
        for k, d in load(p).items():
            kernels.setdefault(short(k), {}).update(d)
    # Class-pure shade (a class_list launch, then a shade_classq launch, per
    # round and tile group): "shade" is the pair -- counters summed -- so
    # bench.py's shade time (both launches) meets its bytes.
    if "class_list" in kernels and "shade_classq" in kernels and "shade" not in kernels:
        a, b = kernels["class_list"], kernels["shade_classq"]
        kernels["shade"] = {c: a.get(c, 0.0) + b[c] for c in b}   # dispatch_ns too: the pair's time
    result = {}
    for k, d in kernels.items():
        e = {c: round(v, 1) for c, v in d.items()}
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            rd = 2.0 * d["FETCH_SIZE"] * 1024
            wr = d["WRITE_SIZE"] * 1024
            e["hbm_read_bytes"] = round(rd)
            e["hbm_write_bytes"] = round(wr)
            e["hbm_bytes"] = round(rd + wr)
        # VALU issue: a wave64 VALU instruction holds its SIMD 2 cycles
        # (MI355X_MICROARCH.md constants table); 256 CUs x 4 SIMDs; the
        # GRBM_GUI_ACTIVE sum over the 8 XCDs / 8 = the dispatch's cycles.
        if "SQ_INSTS_VALU" in d and "GRBM_GUI_ACTIVE" in d:
            cycles = d["GRBM_GUI_ACTIVE"] / 8
            e["valu_issue_frac"] = round(d["SQ_INSTS_VALU"] * 2 / (1024 * max(cycles, 1)), 4)
        if "SQ_THREAD_CYCLES_VALU" in d and "SQ_ACTIVE_INST_VALU" in d:
            e["valu_active_lanes"] = round(d["SQ_THREAD_CYCLES_VALU"] / max(d["SQ_ACTIVE_INST_VALU"], 1), 1)
        if "dispatch_ns" in d:
            e["dispatch_ms"] = round(d["dispatch_ns"] * 1e-6, 5)
            if "hbm_bytes" in e:
                # HBM GB/s of the profiled (serialised) dispatches: bytes and
                # time from the same dispatches.
                e["hbm_gbps_serialised"] = round(e["hbm_bytes"] / d["dispatch_ns"], 2)
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
            e["l2_hit_rate"] = round(d["TCC_HIT_sum"] / max(d["TCC_HIT_sum"] + d["TCC_MISS_sum"], 1), 4)
        result[k] = e
        print(k, json.dumps(e))
    json.dump(result, open(out_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
