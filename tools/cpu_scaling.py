"""Thread scaling of the CPU baseline (the oracle: scalar C++ restatement of
the integrator, std::thread over pixel rows) on the C3 frame, 1..T threads.

VERDICT r03 #8 asked for an all-core run beside bench.py's 16-thread
cpu_baseline.  On the GPU box a job's CPU share is 16 threads (OMP_NUM_THREADS)
of a 256-CPU host shared with the other GPUs' jobs, so this measures the
oracle's scaling up to that share and reports the per-thread rate from which
an all-core figure is extrapolated (stated as such, not measured).

usage: python tools/cpu_scaling.py OUT.json [--threads 1,2,4,8,16] [--rounds 2]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--config", type=int, default=3)
    a = ap.parse_args()
    import bench
    import oracle_lib  # test infrastructure: the CPU baseline, never the product path
    pt = bench.load_package()
    scene = pt.Scene.config(a.config)
    info = scene.info
    rows = []
    for t in [int(x) for x in a.threads.split(",")]:
        o = oracle_lib.OracleRenderer(scene.packs(), info.width, info.height, threads=t)
        o.RenderFlags = info.render_flags
        o.reset()
        o.run(2)
        r0, s0 = o.counters()
        t0 = time.perf_counter()
        for _ in range(a.rounds):
            o.run(1)
        dt = time.perf_counter() - t0
        r1, s1 = o.counters()
        o.close()
        row = {"threads": t, "rounds": a.rounds, "seconds": round(dt, 3), "mrays_per_s": round((r1 - r0) / dt / 1e6, 4)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    base = rows[0]["mrays_per_s"] / rows[0]["threads"]
    for r in rows:
        r["efficiency_vs_1_thread"] = round(r["mrays_per_s"] / (base * r["threads"]), 3)
    host = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except OSError:
        aff = host
    last = rows[-1]
    out = {"config": f"C{a.config} {info.width}x{info.height}", "cpu_model": bench.cpu_model(), "host_cpus": host,
           "affinity_cpus": aff, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "rows": rows,
           "extrapolated_all_host_cpus_mrays_per_s": round(last["mrays_per_s"] / last["threads"] * host, 1),
           "extrapolation": f"{last['threads']}-thread rate per thread x {host} host CPUs (linear; not measured: "
                            "the job's CPU share is its OMP_NUM_THREADS)"}
    Path(a.out).write_text(json.dumps(out, indent=1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
