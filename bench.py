"""Benchmark: Mrays/s of the wavefront integrator on the C3 room scene
(BASELINE.json metric "Mrays/s + Msamples/s, Viking Room 1920x1080 1024spp,
1/2/4/8 GPUs"; --config 4 for C4, 3840x2160 over 8 GPUs).

A step is one integrator round (extend + shade over every pixel slot, i.e.
one RunBasicRenderer(1)).  Inputs (scene, slot state) are resident in HBM
before timing starts.  For N GPUs (one process per GPU, launched by
torch.distributed.run) the job is sharded one of two ways (--shard):

* samples (default, all single-GPU configs): north_star's "pixels/samples
  shard embarrassingly ... RCCL reduce of the per-pixel radiance and
  sample-count buffers at frame end".  Every rank renders the whole frame with
  its own RNG stream (FrameIndex offset rank << 24), so the frame's spp
  target is split over the ranks; the frame-end ncclReduce of the XYZ sums and
  sample counts into rank 0's total buffer (ptCommReduceSampleBufferInto) is
  inside the timed region.  Per-GPU work per step is fixed: "weak".
* bands (default for C4, "pixel-tiled across 8xMI355X"): the frame is split
  into 16-row bands, band b on rank b % N (strong scaling: each rank traces
  1/N of the frame); the frame-end RCCL point-to-point gather of every rank's
  bands to rank 0 (ptCommGatherSampleBuffer) is inside the timed region.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
PKG_DIR = ROOT / "path-tracer_amd"

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
# Algorithmic bytes per ray per launch, SURVEY.md §8(d) (the reference's SoA
# records, independent of this build's layout): extend reads the 20-B ray and
# writes the 24-B hit; shade reads path 60 + ray/hit 44 and writes ray 20 +
# path vertex 52.  Sum = the 220 B/ray whole-path figure.
ALG_BYTES = {"extend": 44, "shade": 176, "round": 220}   # round: fused extend + shade (small partitions)
L2_PEAK_GBPS = 34500.0   # aggregate L2 bandwidth (MI355X_MICROARCH.md § L2)
PATH_BYTES_PER_RAY = 220  # SURVEY.md §8(d) whole-path definition


def load_package():
    spec = importlib.util.spec_from_file_location("path_tracer_amd", PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["path_tracer_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


SETTLE_ROUNDS = 32   # untimed rounds after Reset + Run(2), before the warm-up steps


def measured_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC profile
    (profiles/traffic.json <- profiles/pmc_summary.py over separate
    FETCH_SIZE / WRITE_SIZE passes of this bench, gfx950-corrected), or None."""
    p = ROOT / "profiles" / "traffic.json"
    if not p.exists():
        return None, None
    d = json.loads(p.read_text())
    k = d.get("kernels", {}).get(kernel, {})
    return k.get("hbm_bytes"), d.get("profile")


def measured_issue(kernel):
    """VALU issue utilisation of `kernel` from the committed PMC profile
    (profiles/traffic.json "issue"): the bound that actually limits the
    traversal and shading kernels, which are far below the HBM roofline."""
    p = ROOT / "profiles" / "traffic.json"
    if not p.exists():
        return None
    return json.loads(p.read_text()).get("issue", {}).get(kernel)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(pt, scene, width, height, max_seconds=12.0, max_rounds=200):
    """Time the CPU oracle (scalar C++ restatement, std::thread over host
    cores) on the same scene and frame.  Bounded: Reset + Run(2) warm-up, then
    single rounds until max_seconds of timed work or max_rounds.

    Threads: every CPU this process may run on (its affinity mask), capped by
    OMP_NUM_THREADS when set -- on the GPU box that is the job's CPU share
    (16) of a machine whose nproc counts every GPU's share."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    host_cpus = os.cpu_count() or 1
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = host_cpus
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(allowed, omp) if omp > 0 else allowed)
    o = oracle_lib.OracleRenderer(scene.packs(), width, height, threads=threads)
    o.RenderFlags = 3
    o.reset()
    o.run(2)
    r0, s0 = o.counters()
    t0 = time.perf_counter()
    rounds = 0
    while rounds < max_rounds:
        o.run(1)
        rounds += 1
        if time.perf_counter() - t0 > max_seconds:
            break
    dt = time.perf_counter() - t0
    r1, s1 = o.counters()
    o.close()
    return {
        "value": round((r1 - r0) / dt / 1e6, 4),
        "unit": "Mrays/s",
        "cores": threads,
        "threads": threads,
        "host_cpus": host_cpus,
        "affinity_cpus": allowed,
        "omp_num_threads": omp or None,
        "cpu_model": cpu_model(),
        "kind": "port",
        "sample": f"C3 {width}x{height}, {rounds} rounds after Reset+Run(2) warm-up "
                  f"({(r1 - r0)} rays, {(s1 - s0)} samples, {dt:.1f} s)",
        "msamples_per_s": round((s1 - s0) / dt / 1e6, 4),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--profile-period", type=int, default=4,
                    help="time the kernels of every N-th step (HIP events) inside the timed loop")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--one-gpu-flow-check", action="store_true",
                    help="every rank on device 0 (multi-rank flow check on a one-GPU box; timings not meaningful)")
    ap.add_argument("--shard", choices=("auto", "samples", "bands"), default="auto",
                    help="multi-GPU split: samples (whole frame per rank, own RNG stream) or 16-row pixel bands; "
                         "auto = bands for C4 (pixel-tiled by its config), samples otherwise")
    args = ap.parse_args()
    shard = args.shard if args.shard != "auto" else ("bands" if args.config == 4 else "samples")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")

    pt = load_package()
    scene = pt.Scene.config(args.config)
    info = scene.info
    width, height = info.width, info.height

    # One GPU per rank: LOCAL_RANK indexes the visible devices; a launcher
    # that leaves each rank a single visible device gets device 0.
    ndev = max(pt.device_count(), 1)
    dev = pt.Device(0 if args.one_gpu_flow_check else local_rank % ndev)
    dscene = pt.DeviceScene(dev)
    dscene.update(scene)
    sb = pt.SampleBuffer(dev, width, height)
    part_rank, part_n = (rank, world) if shard == "bands" else (0, 1)
    r = pt.BasicRenderer(dev, dscene, sb, rank=part_rank, nranks=part_n)
    r.RenderFlags = info.render_flags
    r.PathTerminationProbability = info.termination_probability
    # Sample shards: rank r's RNG stream starts at FrameIndex r << 24 (seeds
    # are hashed from (x, y, FrameIndex), scene.glsl.inc / basic.cpp:285-332).
    if shard == "samples":
        r.FrameIndex = rank << 24
    total = pt.SampleBuffer(dev, width, height) if (world > 1 and shard == "samples" and rank == 0) else None
    comm = None
    exchange = None
    if world > 1:
        import torch
        uid = bytearray(pt.Comm.unique_id()) if rank == 0 else bytearray(128)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        dist.broadcast(t, 0)
        # RCCL over xGMI; if the communicator cannot be built (e.g. two ranks
        # on one device, which RCCL refuses) the frame-end exchange falls back
        # to a gloo reduce through host memory, and the line says so.
        try:
            comm = pt.Comm(dev, world, rank, bytes(t.tolist()))
            exchange = "rccl"
        except Exception as e:   # noqa: BLE001
            print(f"bench: RCCL communicator unavailable ({e}); gloo fallback", file=sys.stderr, flush=True)
            exchange = "gloo-fallback"
        ok = torch.tensor([1 if comm is not None else 0], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0 and comm is not None:   # every rank takes the same path
            comm.close()
            comm, exchange = None, "gloo-fallback"

    def frame_end_exchange():
        """The frame-end exchange (inside the timed region)."""
        if world == 1:
            return
        if comm is not None:
            if shard == "samples":
                comm.reduce_sample_buffer_into(sb, total, 0)
            else:
                comm.gather_sample_buffer(sb, 0)
            return
        import torch
        a = sb.read()
        if shard == "bands":
            a[~pt.owned_pixels(width, height, rank, world)] = 0.0
        acc = torch.from_numpy(a)
        dist.reduce(acc, dst=0, op=dist.ReduceOp.SUM)
        if rank == 0:
            (total if shard == "samples" else sb).write(acc.numpy())

    # Reset + Run(2) as after a restart (application.cpp:109-110), then the
    # path population settles (the first ~30 rounds after a restart run ~4 %
    # slower than the rest of a 1024-spp render, tools/exp_trend.py), then the
    # W warm-up steps.
    r.reset()
    r.run(2)
    r.run(SETTLE_ROUNDS)
    for _ in range(args.warmup):
        r.run(1)
    dev.synchronize()
    rays0, samples0 = r.stats()

    def barrier():
        if dist is not None:
            dist.barrier()

    # Kernel durations: HIP events around the extend / shade launches of every
    # profile_period-th step of the timed loop (an event pair per launch costs
    # issue time; sampling keeps the measured loop representative).
    dev.set_profiling(True, period=args.profile_period)
    dev.reset_kernel_stats()
    barrier()
    dev.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r.run(1)
    frame_end_exchange()
    dev.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    n_ext, ms_ext = dev.kernel_stats(1)
    n_sh, ms_sh = dev.kernel_stats(2)
    n_rd, ms_rd = dev.kernel_stats(5)    # fused rounds (a partition that fits the GPU at once)
    dev.set_profiling(False)

    # Traversal counters of one extra extend over the current rays (outside
    # the timed region; the next Run overwrites the same hit records).
    trav = r.extend_stats()
    slots_owned = int(np.sum(pt.owned_pixels(width, height, part_rank, part_n)))
    # Rays traced and paths completed in the timed steps (ptGetStats; the
    # sample count equals the accumulator's alpha increments).
    rays1, samples1 = r.stats()
    rays_local, samples_local = rays1 - rays0, samples1 - samples0
    assert rays_local == slots_owned * args.steps
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        local = torch.tensor([rays_local, samples_local], dtype=torch.float64)
        dist.all_reduce(local, op=dist.ReduceOp.SUM)
        rays, samples = float(local[0]), float(local[1])
    else:
        rays, samples = float(rays_local), float(samples_local)

    def shutdown():
        for x in (r, sb, dscene) + ((total,) if total is not None else ()):
            x.close()
        if comm is not None:
            comm.close()
        dev.close()
        if dist is not None:
            dist.destroy_process_group()

    if rank != 0:
        shutdown()
        return

    mrays = rays / dt / 1e6
    avg_ext = ms_ext / max(n_ext, 1) if n_ext else ms_rd / max(n_rd, 1)   # traversal-level cache rate below
    kernels = {}
    for name, n_k, ms_k in (("extend", n_ext, ms_ext), ("shade", n_sh, ms_sh), ("round", n_rd, ms_rd)):
        if n_k:
            avg = ms_k / n_k
            kernels[name] = {"avg_ms": avg, "gbps": ALG_BYTES[name] * slots_owned / (avg * 1e-3) / 1e9}
    dom = max(kernels, key=lambda k: kernels[k]["avg_ms"])
    achieved = kernels[dom]["gbps"]
    traffic, traffic_src = measured_traffic(dom)
    xname = "RCCL" if exchange == "rccl" else "gloo (host-memory fallback)"
    metric = ("Mrays/s + Msamples/s, Viking Room 1920x1080 1024spp, 1/2/4/8 GPUs" if args.config == 3 else
              f"Mrays/s + Msamples/s, C{args.config} {info.width}x{info.height} {info.spp}spp")
    out = {
        "metric": metric,
        "value": round(mrays, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak" if shard == "samples" else "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic (procedural {info.mesh_face_count}-triangle room mesh + 1024^2 texture; "
                "Viking Room asset absent)",
        "config": {
            "workload": (f"C{args.config} scene, {width}x{height} px frame split in 16-row bands over {world} GPU(s) "
                         f"({slots_owned} px on rank 0), one round (extend+shade of every pixel's path) per step"
                         if shard == "bands" else
                         f"C{args.config} scene, {width}x{height} px frame; each of {world} GPU(s) renders every pixel "
                         f"with its own RNG stream (the spp target split over the GPUs), one round (extend+shade of "
                         f"every pixel's path) per step per GPU"),
            "shard": shard,
            "exchange": exchange,
            "spp_target": info.spp,
            "settle_rounds": SETTLE_ROUNDS,
            "mesh_faces": info.mesh_face_count,
            "parallelism": (f"pixel-bands x{world}" + (f" + {xname} band gather to rank 0" if world > 1 else "")
                            if shard == "bands" else
                            f"sample-shards x{world}" + (f" + {xname} reduce of radiance + sample counts to rank 0"
                                                         if world > 1 else "")),
        },
        "msamples_per_s": round(samples / dt / 1e6, 3),
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 5),
            "traffic": traffic,
            "traffic_unit": "bytes per launch (HBM, PMC)",
            "traffic_source": traffic_src,
            "alg_bytes_per_launch": ALG_BYTES[dom] * slots_owned,
            "alg_bytes_per_slot": ALG_BYTES[dom],
            "launch_avg_ms": {k: round(v["avg_ms"], 4) for k, v in kernels.items()},
            "launches_timed": {"extend": n_ext, "shade": n_sh, "round": n_rd, "every_nth_step": args.profile_period},
            "path_gbps_220B_per_ray": round(PATH_BYTES_PER_RAY * rays / dt / 1e9, 2),
        },
        # What bounds the dominant kernel instead of HBM (PMC, same profile):
        # fraction of the chip's VALU issue slots used, and active lanes per
        # VALU instruction (of 64; divergence).
        "limiter": {"kind": "valu_issue", "kernel": dom, **(measured_issue(dom) or {}),
                    "per_kernel": {k: measured_issue(k) for k in ("extend", "shade")},
                    "source": traffic_src},
    }
    # Node/face bytes the traversal pulls through L1/L2 per ray (BVH + faces
    # are cache-resident): internal node = both child boxes (64 B), face 48 B,
    # stack pop = 2 index words (8 B).
    cache_bytes = (64 * trav["internal_nodes"] + 48 * trav["faces"] + 8 * trav["pops"]) / max(trav["rays"], 1)
    out["traversal"] = {
        "simd_efficiency": round(trav["simd_efficiency"], 4),
        "steps_per_ray": round(trav["lane_steps_per_ray"], 2),
        "internal_nodes_per_ray": round(trav["internal_nodes_per_ray"], 2),
        "leaves_per_ray": round(trav["blas_leaves_per_ray"], 2),
        "faces_per_ray": round(trav["faces_per_ray"], 2),
        "pops_per_ray": round(trav["pops_per_ray"], 2),
        "cache_bytes_per_ray": round(cache_bytes, 1),
        "cache_gbps": round(cache_bytes * slots_owned / (avg_ext * 1e-3) / 1e9, 1),
        "l2_peak_gbps": L2_PEAK_GBPS,
    }
    if not args.no_cpu_baseline and world == 1:   # rank 0 at N=1 only
        out["cpu_baseline"] = cpu_baseline(pt, scene, info.width, info.height)
    print(json.dumps(out), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
