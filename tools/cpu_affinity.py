"""Where the CPU baseline's two placement clusters come from:
the C3 oracle at 16 threads, after a 34-round settle, timed over a few
consecutive rounds under different CPU masks for its worker threads (the
oracle's std::thread workers are created per round and inherit the calling
thread's mask):
  all        the process's whole affinity mask (what bench.py's cpu_baseline uses)
  cores16    16 logical CPUs on 16 distinct physical cores (one SMT sibling each)
  smt8x2     8 physical cores, both SMT siblings of each (16 logical CPUs)
  cores16b   another 16 distinct cores (the other package when there are two)
Prints one JSON object: the host topology summary, /proc/loadavg, and the
per-mask rates of each repetition.

usage: python tools/cpu_affinity.py OUT.json [--reps 2] [--rounds 6] [--settle 34]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def topology():
    cpus = sorted(os.sched_getaffinity(0))
    info = {}
    for c in cpus:
        base = Path(f"/sys/devices/system/cpu/cpu{c}/topology")
        try:
            pkg = int((base / "physical_package_id").read_text())
            core = int((base / "core_id").read_text())
        except OSError:
            pkg, core = 0, c
        info[c] = (pkg, core)
    return cpus, info


def masks(cpus, info):
    by_core = {}
    for c in cpus:
        by_core.setdefault(info[c], []).append(c)
    cores = sorted(by_core)           # (package, core)
    first = [by_core[k][0] for k in cores]
    out = {"all": set(cpus), "cores16": set(first[:16])}
    pairs = [k for k in cores if len(by_core[k]) >= 2][:8]
    if len(pairs) == 8:
        out["smt8x2"] = {c for k in pairs for c in by_core[k][:2]}
    pk = sorted({k[0] for k in cores})
    other = [by_core[k][0] for k in cores if k[0] == pk[-1]] if len(pk) > 1 else first[len(first) // 2:]
    if len(other) >= 16:
        out["cores16b"] = set(other[:16])
    return out, len(cores), pk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--settle", type=int, default=34)
    a = ap.parse_args()
    import bench
    import oracle_lib  # test infrastructure: the CPU baseline, never the product path
    pt = bench.load_package()
    scene = pt.Scene.config(3)
    info = scene.info
    cpus, topo = topology()
    ms, ncores, pkgs = masks(cpus, topo)
    home = os.sched_getaffinity(0)
    o = oracle_lib.OracleRenderer(scene.packs(), info.width, info.height, threads=16)
    o.RenderFlags = info.render_flags
    o.reset()
    o.run(2)
    for _ in range(a.settle):
        o.run(1)
    rows = []
    try:
        for rep in range(a.reps):
            for name, m in ms.items():
                os.sched_setaffinity(0, m)
                r0, _ = o.counters()
                t0 = time.perf_counter()
                c0 = time.process_time()
                for _ in range(a.rounds):
                    o.run(1)
                dt = time.perf_counter() - t0
                cpu = time.process_time() - c0
                r1, _ = o.counters()
                rows.append({"rep": rep, "mask": name, "cpus": len(m), "seconds": round(dt, 3),
                             "mrays_per_s": round((r1 - r0) / dt / 1e6, 3), "cpu_seconds": round(cpu, 2)})
                print(json.dumps(rows[-1]), flush=True)
    finally:
        os.sched_setaffinity(0, home)
        o.close()
    out = {"cpu_model": bench.cpu_model(), "affinity_cpus": len(cpus), "physical_cores": ncores,
           "packages": pkgs, "loadavg": Path("/proc/loadavg").read_text().strip(),
           "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "threads": 16, "rounds_per_sample": a.rounds,
           "settle_rounds": a.settle, "masks": {k: sorted(v)[:20] for k, v in ms.items() if k != "all"},
           "rows": rows}
    Path(a.out).write_text(json.dumps(out, indent=1))
    print(json.dumps({k: v for k, v in out.items() if k != "rows"}))


if __name__ == "__main__":
    main()
