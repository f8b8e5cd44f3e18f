"""Thread scaling of the CPU baseline (the oracle: scalar C++ restatement of
the integrator, std::thread over pixels) on the C3 frame, 1..T threads.

One code path with bench.py's CPU leg: bench.pin_cores (the
threads' distinct physical cores of one package, pinned from the oracle's
creation on), bench.settled_oracle (Reset, Run(2), 34 settle rounds) and
bench.time_oracle_rounds (at least 32 rounds, more while under 15 s).  The table's first row IS the bench leg: a fresh oracle at
the job's thread count, settled and timed exactly as bench.py times it.  The
other thread counts then time the rounds that follow on the same render
(oracle_set_threads), largest first.

On the GPU box a job's CPU share is 16 threads (OMP_NUM_THREADS) of a
256-CPU host shared with the other GPUs' jobs; this tool stays inside that
share, and states the all-core figure as an extrapolation of the measured
per-thread rate, not a measurement.

usage: python tools/cpu_scaling.py OUT.json [--threads 16,8,4,2,1] [--rounds 32] [--max-seconds 30]
"""
import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--threads", default="", help="comma list (default: the bench leg's count, then halvings to 1)")
    ap.add_argument("--rounds", type=int, default=32, help="minimum timed rounds per thread count")
    ap.add_argument("--max-seconds", type=float, default=30.0)
    ap.add_argument("--config", type=int, default=3)
    a = ap.parse_args()
    import bench
    pt = bench.load_package()
    scene = pt.Scene.config(a.config)
    info = scene.info
    lead, allowed, omp = bench.cpu_threads()
    if a.threads:
        counts = [int(x) for x in a.threads.split(",")]
    else:
        counts, t = [lead], lead
        while t > 1:
            t //= 2
            counts.append(t)
    counts = sorted(set(counts), reverse=True)
    # The bench leg's placement: pinned from creation on (first touch on the
    # package the threads run on); smaller counts take the first cores of
    # that set, so every row runs on the package that holds the state.
    cores, placement = bench.pin_cores(counts[0])
    home = os.sched_getaffinity(0)
    if cores:
        os.sched_setaffinity(0, set(cores))
    o = bench.settled_oracle(scene, info.width, info.height, counts[0], 3)
    os.sched_setaffinity(0, home)
    rows = []
    for i, t in enumerate(counts):
        # The first row: bench.py's CPU leg exactly (fresh settled render,
        # its round minimum and time bound); the smaller counts time fewer
        # rounds when a round is slow (a 1-thread C3 round takes ~2.4 s).
        mx = a.max_seconds if i == 0 else min(a.max_seconds, 20.0)
        est = rows[0]["median_round_s"] * counts[0] / t if rows else 0.0   # this count's round, predicted
        mn = a.rounds if i == 0 else max(4, min(a.rounds, int(mx / max(est, 1e-3))))
        row = bench.time_oracle_rounds(o, t, mn, mx, cores, placement if i == 0 else None)
        row["bench_leg"] = i == 0 and t == lead
        rows.append(row)
        print(json.dumps(row), flush=True)
    o.close()
    base = rows[-1]["mrays_per_s"] / rows[-1]["threads"]
    for r in rows:
        r["efficiency_vs_fewest_threads"] = round(r["mrays_per_s"] / (base * r["threads"]), 3)
    host = os.cpu_count() or 1
    top = rows[0]
    out = {"config": f"C{a.config} {info.width}x{info.height}", "cpu_model": bench.cpu_model(), "host_cpus": host,
           "affinity_cpus": allowed, "omp_num_threads": omp or None,
           "method": f"bench.settled_oracle (Reset, Run(2), {bench.CPU_SETTLE_ROUNDS} settle rounds at {counts[0]} "
                     "threads), then bench.time_oracle_rounds per thread count, largest first, on the same render",
           "rows": rows,
           "extrapolated_all_host_cpus_mrays_per_s": round(top["mrays_per_s"] / top["threads"] * host, 1),
           "extrapolation": f"{top['threads']}-thread rate per thread x {host} host CPUs (linear; NOT measured: "
                            "the job's CPU share is its OMP_NUM_THREADS, the rest of the host belongs to the "
                            "other GPUs' jobs)"}
    Path(a.out).write_text(json.dumps(out, indent=1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
