"""Thread scaling of the CPU baseline (the oracle: scalar C++ restatement of
the integrator, std::thread over pixels) on the C3 frame, 1..T threads, over
SETTLED rounds: one oracle is reset, run through Run(2) + `settle` rounds at
the largest thread count (the path population past its first rounds, where
the per-round cost is stationary), then each thread count times `rounds`
consecutive rounds of the same render (oracle_set_threads between them).

VERDICT r04 #6: round 4 timed 2 rounds right after Reset (the shortest paths)
per thread count.  Each thread count runs pinned to that many distinct
physical cores of one package (bench.pick_cores), as bench.py's cpu_baseline
does.  On the GPU box a job's CPU share is 16 threads
(OMP_NUM_THREADS) of a 256-CPU host shared with the other GPUs' jobs; this
tool stays inside that share, and states the all-core figure as an
extrapolation of the measured per-thread rate, not a measurement.

usage: python tools/cpu_scaling.py OUT.json [--threads 1,2,4,8,16] [--settle 34] [--rounds 32]
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
    ap.add_argument("--settle", type=int, default=34)
    ap.add_argument("--rounds", type=int, default=32)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--init-gpu", action="store_true",
                    help="create a HIP device first, as bench.py's process has when it times its cpu_baseline")
    a = ap.parse_args()
    import bench
    import oracle_lib  # test infrastructure: the CPU baseline, never the product path
    pt = bench.load_package()
    dev = pt.Device(0) if a.init_gpu else None
    scene = pt.Scene.config(a.config)
    info = scene.info
    counts = [int(x) for x in a.threads.split(",")]
    o = oracle_lib.OracleRenderer(scene.packs(), info.width, info.height, threads=max(counts))
    o.RenderFlags = info.render_flags
    o.reset()
    o.run(2)
    t0 = time.perf_counter()
    for _ in range(a.settle):
        o.run(1)
    settle_s = time.perf_counter() - t0
    print(json.dumps({"settle_rounds": a.settle, "settle_s": round(settle_s, 2), "threads": max(counts)}), flush=True)
    rows = []
    home = os.sched_getaffinity(0)
    allowed = len(home)
    for t in counts:
        o.set_threads(t)
        # The same placement as bench.py's cpu_baseline: t threads pinned to
        # t distinct, least busy physical cores of one package.
        pinned, placement = bench.pick_cores(t) if t < allowed else (None, "every affinity CPU, unpinned")
        os.sched_setaffinity(0, pinned if pinned else home)
        r0, s0 = o.counters()
        t0 = time.perf_counter()
        c0 = time.process_time()
        per_round = []
        for _ in range(a.rounds):
            t1 = time.perf_counter()
            o.run(1)
            per_round.append(time.perf_counter() - t1)
        dt = time.perf_counter() - t0
        cpu_s = time.process_time() - c0
        r1, s1 = o.counters()
        per_round.sort()
        row = {"threads": t, "rounds": a.rounds, "seconds": round(dt, 3),
               "mrays_per_s": round((r1 - r0) / dt / 1e6, 4),
               "msamples_per_s": round((s1 - s0) / dt / 1e6, 4),
               "median_round_s": round(per_round[len(per_round) // 2], 4),
               "min_round_s": round(per_round[0], 4), "max_round_s": round(per_round[-1], 4),
               "cpu_seconds": round(cpu_s, 2),
               "mrays_per_cpu_s_x_threads": round((r1 - r0) / max(cpu_s, 1e-9) * t / 1e6, 4),
               "placement": placement, "pinned_cpus": sorted(pinned) if pinned else None}
        os.sched_setaffinity(0, home)
        rows.append(row)
        print(json.dumps(row), flush=True)
    o.close()
    if dev is not None:
        dev.close()
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
           "affinity_cpus": aff, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
           "hip_device_initialised": a.init_gpu,
           "method": f"one render: Reset, Run(2), {a.settle} settle rounds at {max(counts)} threads, then "
                     f"{a.rounds} timed consecutive rounds per thread count",
           "rows": rows,
           "extrapolated_all_host_cpus_mrays_per_s": round(last["mrays_per_s"] / last["threads"] * host, 1),
           "extrapolation": f"{last['threads']}-thread rate per thread x {host} host CPUs (linear; not measured: "
                            "the job's CPU share is its OMP_NUM_THREADS, the rest of the host belongs to the "
                            "other GPUs' jobs)"}
    Path(a.out).write_text(json.dumps(out, indent=1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
