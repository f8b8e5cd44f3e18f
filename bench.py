"""Benchmark: Mrays/s of the wavefront integrator over whole frames of the
BASELINE.json metric "Mrays/s + Msamples/s, Viking Room 1920x1080 1024spp,
1/2/4/8 GPUs" (C3; --config 4 for C4, 3840x2160 4096spp over 8 GPUs).

A step is one frame in SURVEY.md §8(d)'s benchmark mode: Reset, Run(2), then
Run(1) rounds until the paths completed since the Reset reach the config's spp
target x pixels (ptRenderFrame; the application's frame loop,
application.cpp:100-115, basic.cpp:285-332), plus the frame-end exchange for
N GPUs.  `value` = rays traced by all ranks / the max over ranks of the timed
frames' wall time.  Inputs (scene, buffers) are resident in HBM before timing
starts.

N GPUs, one process per GPU.  `bench.py --gpus N` without a launcher starts
`torch.distributed.run --nproc-per-node N` over itself (before any GPU call);
under a launcher WORLD_SIZE must equal --gpus.  The frame is split one of two
ways (--shard), total work fixed either way ("strong" scaling):

* samples (default, every config that fits one GPU): north_star's
  "pixels/samples shard embarrassingly ... RCCL reduce of the per-pixel
  radiance and sample-count buffers at frame end".  Every rank renders the
  whole frame with its own RNG stream (FrameIndex offset rank << 24) to
  1/N of the spp target; the frame-end ncclReduce of the XYZ sums and sample
  counts into rank 0's total buffer (ptCommReduceSampleBufferInto) is inside
  the step.
* bands (default for C4, "pixel-tiled across 8xMI355X"): 16-row bands, band b
  on rank b % N, each rank to the full spp target on its own pixels; the
  frame-end RCCL point-to-point gather of the bands to rank 0
  (ptCommGatherSampleBuffer) is inside the step.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import math
import os
import socket
import subprocess
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
# round: fused extend + shade (small partitions); rounds: a round batch (per round it covers)
ALG_BYTES = {"extend": 44, "shade": 176, "round": 220, "rounds": 220}
KERNEL_IDS = {"extend": 1, "shade": 2, "round": 5, "rounds": 6}   # pt_api.h PT_KERNEL_*
L2_PEAK_GBPS = 34500.0   # aggregate L2 bandwidth (MI355X_MICROARCH.md § L2)
PATH_BYTES_PER_RAY = 220  # SURVEY.md §8(d) whole-path definition
STEADY_ROUNDS = 64        # secondary key: steady-state rounds timed after the frames
FILL_SLOTS = 1 << 21      # slots per launch a band partition is filled to with path streams (C3 frame: 2.07 M)
SETTLE_ROUNDS = 32        # ... after this many rounds past a restart


def load_package():
    spec = importlib.util.spec_from_file_location("path_tracer_amd", PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["path_tracer_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def profile_for(key):
    """The committed PMC summary of this workload (profiles/traffic.json,
    keyed by config, or "CONFIG:bandsNxK" for rank 0 of N band partitions
    with K path streams; tools/update_traffic.py), or None."""
    p = ROOT / "profiles" / "traffic.json"
    if not p.exists():
        return None
    return json.loads(p.read_text()).get("configs", {}).get(str(key))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def pick_cores(n, sample_s=0.25):
    """n logical CPUs of this process's affinity mask on n distinct physical
    cores of one package, the least busy over a /proc/stat sample (the host
    is shared with other GPUs' jobs), and a description; (None, reason) when
    the topology is unreadable or too small.  Unpinned, the oracle's threads
    (created per round) land across both packages and ran 5.9-7.1 Mrays/s
    against 9.9-11.3 pinned to 16 distinct cores (tools/cpu_affinity.py,
    profiles/r05_aff): the placement, not the host's load, made round 4's
    and round 5's two clusters."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
        topo = {}
        for c in cpus:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            topo[c] = (int(open(base + "physical_package_id").read()), int(open(base + "core_id").read()))

        def stat():
            out = {}
            for line in open("/proc/stat"):
                f = line.split()
                if f[0].startswith("cpu") and f[0] != "cpu":
                    v = [int(x) for x in f[1:]]
                    out[int(f[0][3:])] = (sum(v), v[3] + (v[4] if len(v) > 4 else 0))
            return out
        a = stat()
        time.sleep(sample_s)
        b = stat()
    except (OSError, ValueError, AttributeError, KeyError):
        return None, "topology unreadable: threads unpinned"

    def busy(c):
        dt = b[c][0] - a[c][0]
        return 1.0 - (b[c][1] - a[c][1]) / dt if dt > 0 else 1.0
    cores = {}
    for c in cpus:
        cores.setdefault(topo[c], []).append(c)
    # A core's load: its busiest sibling; its CPU: its least busy sibling.
    load = {k: max(busy(c) for c in v) for k, v in cores.items()}
    best = None
    for pkg in sorted({k[0] for k in cores}):
        ks = sorted((k for k in cores if k[0] == pkg), key=lambda k: load[k])[:n]
        if len(ks) == n and (best is None or sum(load[k] for k in ks) < best[0]):
            best = (sum(load[k] for k in ks), pkg, ks)
    if best is None:
        return None, f"fewer than {n} physical cores in one package: threads unpinned"
    _, pkg, ks = best
    chosen = sorted(min(cores[k], key=busy) for k in ks)
    return set(chosen), (f"{n} threads pinned to {n} distinct physical cores of package {pkg}, the least busy "
                         f"over a {sample_s} s /proc/stat sample (mean busy {best[0] / n:.2f})")


CPU_SETTLE_ROUNDS = 34   # the CPU leg's settled window starts after Reset + Run(2) + this many rounds


def cpu_threads():
    """The CPU leg's thread count: every CPU this process may run on (its
    affinity mask), capped by OMP_NUM_THREADS when set -- on the GPU box that
    is the job's CPU share (16) of a machine whose nproc counts every GPU's
    share.  Returns (threads, affinity CPUs, OMP_NUM_THREADS or 0)."""
    host_cpus = os.cpu_count() or 1
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = host_cpus
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(allowed, omp) if omp > 0 else allowed), allowed, omp


def settled_oracle(scene, width, height, threads, flags, settle_rounds=CPU_SETTLE_ROUNDS):
    """The CPU oracle on the frame, past its first rounds: Reset, Run(2) and
    `settle_rounds` untimed rounds (the path population past its first,
    shortest paths; the per-round cost is then stationary)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib  # test infrastructure: the CPU baseline, never the product path
    o = oracle_lib.OracleRenderer(scene.packs(), width, height, threads=threads)
    o.RenderFlags = flags
    o.reset()
    o.run(2)
    for _ in range(settle_rounds):
        o.run(1)
    return o


def pin_cores(threads):
    """(cores, placement): `threads` distinct physical cores of one package
    for the CPU leg (pick_cores), as a sorted list, or (None, reason) when
    that is every affinity CPU or the topology is unreadable."""
    if threads >= len(os.sched_getaffinity(0)):
        return None, "every affinity CPU, unpinned"
    pinned, placement = pick_cores(threads)
    return (sorted(pinned) if pinned else None), placement


def time_oracle_rounds(o, threads, min_rounds=32, max_seconds=30.0, cores=None, placement=None):
    """Time consecutive single rounds of a settled oracle at `threads`
    threads, pinned to `cores` (distinct physical cores of one package:
    pin_cores; the first `threads` of them) or unpinned when None: at least
    min_rounds, more while under max_seconds / 2, never past max_seconds.
    The one timing code path of bench.py's CPU leg and tools/cpu_scaling.py's
    table."""
    home = os.sched_getaffinity(0)
    o.set_threads(threads)
    # The oracle's worker threads are created per round and inherit this
    # thread's mask.
    pinned = set(cores[:threads]) if cores else None
    if placement is None:
        placement = (f"{threads} threads pinned to {threads} distinct physical cores" if pinned
                     else "every affinity CPU, unpinned")
    try:
        if pinned:
            os.sched_setaffinity(0, pinned)
        r0, s0 = o.counters()
        t0 = time.perf_counter()
        c0 = time.process_time()
        rounds, per_round = 0, []
        while rounds < min_rounds or time.perf_counter() - t0 < max_seconds / 2:
            t1 = time.perf_counter()
            o.run(1)
            per_round.append(time.perf_counter() - t1)
            rounds += 1
            if time.perf_counter() - t0 > max_seconds:
                break
        dt = time.perf_counter() - t0
        cpu_s = time.process_time() - c0
        r1, s1 = o.counters()
    finally:
        os.sched_setaffinity(0, home)
    per_round.sort()
    return {"threads": threads, "rounds": rounds, "seconds": round(dt, 3), "rays": r1 - r0, "samples": s1 - s0,
            "mrays_per_s": round((r1 - r0) / dt / 1e6, 4), "msamples_per_s": round((s1 - s0) / dt / 1e6, 4),
            "median_round_s": round(per_round[len(per_round) // 2], 4),
            "min_round_s": round(per_round[0], 4), "max_round_s": round(per_round[-1], 4),
            # CPU seconds the process's threads actually ran (= threads x
            # wall time when the pinned cores were not shared).
            "cpu_seconds": round(cpu_s, 2),
            "mrays_per_cpu_s_x_threads": round((r1 - r0) / max(cpu_s, 1e-9) * threads / 1e6, 4),
            "placement": placement, "pinned_cpus": sorted(pinned) if pinned else None}


def cpu_baseline(pt, scene, width, height, config, settle_rounds=CPU_SETTLE_ROUNDS, min_rounds=32, max_seconds=30.0):
    """Time the CPU oracle (scalar C++ restatement, std::thread over host
    cores) on the same scene and frame: settled_oracle, then
    time_oracle_rounds at the job's thread count (cpu_threads).  Bounded:
    about 15-30 s of CPU work."""
    threads, allowed, omp = cpu_threads()
    host_cpus = os.cpu_count() or 1
    # Pinned from the oracle's creation on, so its worker threads first-touch
    # the path state on the package they then run on (settling it unpinned
    # left pages on the other package of the NUMA host: 8.98 against 11.76
    # Mrays/s on one box, profiles/r06_final).
    cores, placement = pin_cores(threads)
    home = os.sched_getaffinity(0)
    try:
        if cores:
            os.sched_setaffinity(0, set(cores))
        o = settled_oracle(scene, width, height, threads, 3, settle_rounds)
        try:
            row = time_oracle_rounds(o, threads, min_rounds, max_seconds, cores, placement)
        finally:
            o.close()
    finally:
        os.sched_setaffinity(0, home)
    share = "the job's CPU share (OMP_NUM_THREADS)" if omp > 0 and omp < allowed else "every affinity CPU"
    return {
        "value": row["mrays_per_s"],
        "unit": "Mrays/s",
        "cores": threads,
        "threads": threads,
        "threads_used": f"{threads} threads = {share}; {allowed} affinity CPUs, {host_cpus} host CPUs",
        "host_cpus": host_cpus,
        "affinity_cpus": allowed,
        "omp_num_threads": omp or None,
        "placement": row["placement"],
        "pinned_cpus": row["pinned_cpus"],
        "cpu_model": cpu_model(),
        "kind": "port",
        "sample": f"C{config} {width}x{height}, {row['rounds']} consecutive rounds after Reset + Run(2) + "
                  f"{settle_rounds} settle rounds ({row['rays']} rays, {row['samples']} samples, "
                  f"{row['seconds']:.1f} s timed)",
        "msamples_per_s": row["msamples_per_s"],
        "median_round_s": row["median_round_s"],
        "cpu_seconds": row["cpu_seconds"],
        "mrays_per_cpu_s_x_threads": row["mrays_per_cpu_s_x_threads"],
    }


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n):
    """`bench.py --gpus N` without a launcher: run torch.distributed.run over
    this script as a child (no exec: nothing here has touched the GPU yet) and
    exit with its status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(Path(__file__).resolve())] + sys.argv[1:]
    return subprocess.call(cmd)


def launch_check(args, world, rank):
    """--launch-check: the N-rank plumbing without a GPU (CPU test of the
    launcher): process group, world size, the max-over-ranks reduction and a
    frame-end-sized gloo reduce; rank 0 prints the line's rank fields."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    if args.inject_failure == rank:
        # A rank failing mid-frame (a device fault, an RCCL abort, a bad
        # argument): it raises here, before the exchange its peers block in;
        # the launcher then stops the other ranks and the launch exits non-zero.
        raise RuntimeError(f"bench: injected failure on rank {rank}")
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    acc = torch.ones(4 * 64 * 64, dtype=torch.float32)
    dist.reduce(acc, dst=0, op=dist.ReduceOp.SUM)
    ok = (rank != 0) or bool(torch.all(acc == float(world)).item())
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "world_size": dist.get_world_size(),
                          "max_over_ranks": float(t.item()), "reduce_ok": ok,
                          "config": {"exchange": "gloo", "comm_ranks": dist.get_world_size()}}), flush=True)
    dist.destroy_process_group()
    return 0 if ok else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed frames")
    ap.add_argument("--warmup", type=int, default=1, help="untimed frames")
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--spp", type=int, default=0, help="frame spp target (default: the config's)")
    ap.add_argument("--profile-period", type=int, default=8,
                    help="time the kernels of every N-th round (HIP events) inside the timed frames")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-steady", action="store_true", help="skip the steady-state secondary measurement")
    ap.add_argument("--one-gpu-flow-check", action="store_true",
                    help="every rank on device 0 (multi-rank flow check on a one-GPU box; timings not meaningful)")
    ap.add_argument("--launch-check", action="store_true",
                    help="N-rank launch plumbing only (gloo, no GPU): CPU test of the launcher")
    ap.add_argument("--split", type=int, default=0,
                    help="tile groups on concurrent streams (ptSetBasicRendererSplit): 0 automatic, 1 off, K")
    ap.add_argument("--class-lists", type=int, default=0,
                    help="class-pure shade in tile groups (ptSetBasicRendererClassLists): 0 automatic, 1 off")
    ap.add_argument("--streams", type=int, default=0,
                    help="path streams per owned pixel (0: auto -- bands fill ~2^21 slots per launch, samples 1)")
    ap.add_argument("--inject-failure", type=int, default=-1, metavar="RANK",
                    help="with --launch-check: this rank raises before the exchange (tests the failure path)")
    ap.add_argument("--shard", choices=("auto", "samples", "bands"), default="auto",
                    help="multi-GPU split: samples (whole frame per rank, own RNG stream) or 16-row pixel bands; "
                         "auto = bands for C4 (pixel-tiled by its config), samples otherwise")
    args = ap.parse_args()

    # N ranks: launch them first (before anything touches the GPU), or check
    # the launcher's world size against --gpus.
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(self_launch(args.gpus))
        world, rank, local_rank = 1, 0, 0
    else:
        world = int(os.environ["WORLD_SIZE"])
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if world != args.gpus:
            print(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr, flush=True)
            sys.exit(2)
    if args.launch_check:
        sys.exit(launch_check(args, world, rank))

    shard = args.shard if args.shard != "auto" else ("bands" if args.config == 4 else "samples")
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")

    pt = load_package()
    scene = pt.Scene.config(args.config)
    info = scene.info
    width, height = info.width, info.height
    spp = args.spp or info.spp

    # One GPU per rank: LOCAL_RANK indexes the visible devices; a launcher
    # that leaves each rank a single visible device gets device 0.
    ndev = max(pt.device_count(), 1)
    dev = pt.Device(0 if args.one_gpu_flow_check else local_rank % ndev)
    dscene = pt.DeviceScene(dev)
    dscene.update(scene)
    sb = pt.SampleBuffer(dev, width, height)
    part_rank, part_n = (rank, world) if shard == "bands" else (0, 1)
    px_owned = int(np.sum(pt.owned_pixels(width, height, part_rank, part_n)))
    # Path streams per owned pixel (bands): a partition smaller than one GPU's
    # fill carries several independent paths per pixel so that each launch
    # still holds about FILL_SLOTS slots.
    streams = args.streams if args.streams > 0 else (
        max(1, round(FILL_SLOTS / max(px_owned, 1))) if shard == "bands" else 1)
    r = pt.BasicRenderer(dev, dscene, sb, rank=part_rank, nranks=part_n, streams=streams)
    r.RenderFlags = info.render_flags
    r.PathTerminationProbability = info.termination_probability
    # Sample shards: rank r's RNG stream starts at FrameIndex r << 24 (seeds
    # are hashed from (x, y, FrameIndex), scene.glsl.inc / basic.cpp:285-332).
    if shard == "samples":
        r.FrameIndex = rank << 24
    slots_owned = px_owned * streams    # paths (rays) per round
    # Tile groups on concurrent streams (ptSetBasicRendererSplit): profiling
    # times group 0's launches, which cover timed_tiles of the tiles.
    r.set_split(args.split)
    try:
        r.set_class_lists(args.class_lists)
        class_lists = r.class_lists()
    except AttributeError:   # an older library under PT_HIP_LIB (A/B builds)
        class_lists = None
    split = r.split()
    launch_slots = slots_owned * split["timed_tiles"] / max(split["tiles"], 1) if split["groups"] > 1 else slots_owned
    # This rank's frame target (Σ alpha): samples -> 1/N of spp x frame,
    # bands -> spp x its own pixels.
    target = math.ceil(spp * width * height / world) if shard == "samples" else spp * px_owned
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
        """The frame-end exchange (inside the step)."""
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

    def barrier():
        if dist is not None:
            dist.barrier()

    frames = []   # (rounds, samples) per timed frame

    # A frame that has not reached its target after 64x the rounds the spp
    # target needs at one completed path per slot and round is broken: stop.
    max_rounds = 64 * spp + 64

    last_note = [time.perf_counter()]

    def frame(record):
        rounds, samples = r.render_frame(target, max_rounds)
        # A progress note on stderr at most every 20 s (long configs such as
        # C5's 8192-spp frames), so a watcher sees the run is alive.
        now = time.perf_counter()
        if rank == 0 and now - last_note[0] > 20.0:
            print(f"bench: frame done ({rounds} rounds, {samples} samples)", file=sys.stderr, flush=True)
            last_note[0] = now
        if samples < target:
            raise RuntimeError(f"frame stopped at {rounds} rounds with {samples} of {target} samples")
        r.merge_streams()    # path streams -> the sample buffer (no-op for one stream)
        frame_end_exchange()
        if record:
            frames.append((rounds, samples))

    for _ in range(args.warmup):
        frame(False)
    dev.synchronize()

    # Kernel durations: HIP events around the extend / shade launches of every
    # profile_period-th round of the timed frames (an event pair per launch
    # costs issue time; sampling keeps the measured loop representative).
    dev.set_profiling(True, period=args.profile_period)
    dev.reset_kernel_stats()
    barrier()
    dev.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame(True)
    dev.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    # Per kernel: timed launches, rounds they covered (a round batch covers
    # several) and their total time.
    kstats = {k: (*dev.kernel_stats(i), dev.kernel_rounds(i)) for k, i in KERNEL_IDS.items()}
    dev.set_profiling(False)

    rounds_local = sum(f[0] for f in frames)
    samples_local = sum(f[1] for f in frames)
    rays_local = rounds_local * slots_owned
    assert all(f[1] >= target for f in frames), "a frame ended short of its spp target"

    # Secondary: the steady-state rate (rounds after the path population
    # settled, no Reset in the window), outside the timed frames.
    steady = None
    if not args.no_steady:
        r.reset()
        r.run(2)
        r.run_rounds(SETTLE_ROUNDS)     # consecutive Run(1) rounds, as the frames run them
        dev.synchronize()
        s0 = time.perf_counter()
        r.run_rounds(STEADY_ROUNDS)
        dev.synchronize()
        sdt = time.perf_counter() - s0
        steady = {"rounds": STEADY_ROUNDS, "after_rounds": SETTLE_ROUNDS + 2,
                  "ms_per_round": round(sdt / STEADY_ROUNDS * 1e3, 4),
                  "mrays_per_s_per_gpu": round(slots_owned * STEADY_ROUNDS / sdt / 1e6, 3)}

    # Traversal counters of one extra extend over the current rays (outside
    # the timed region; the next Run overwrites the same hit records).
    trav = r.extend_stats()
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        local = torch.tensor([rays_local, samples_local, rounds_local], dtype=torch.float64)
        dist.all_reduce(local, op=dist.ReduceOp.SUM)
        rays, samples, rounds_all = float(local[0]), float(local[1]), float(local[2])
        comm_ranks = world if comm is not None else None
    else:
        rays, samples, rounds_all = float(rays_local), float(samples_local), float(rounds_local)
        comm_ranks = None

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
    kernels = {}
    for name, (n_k, ms_k, rounds_k) in kstats.items():
        if n_k:
            avg = ms_k / max(rounds_k, 1)   # per round (= per launch except for round batches)
            kernels[name] = {"avg_ms": avg, "gbps": ALG_BYTES[name] * launch_slots / (avg * 1e-3) / 1e9,
                             "launches": n_k, "rounds": rounds_k}
    # traversal-level cache rate below: extend's time per round, or the fused kernels'
    avg_ext = next(kernels[k]["avg_ms"] for k in ("extend", "round", "rounds") if k in kernels)
    # The dominant kernel: the most device time over the timed rounds (C1's
    # frames are mostly round batches, with two single fused rounds each).
    dom = max(kernels, key=lambda k: kernels[k]["avg_ms"] * kernels[k]["rounds"])
    achieved = kernels[dom]["gbps"]
    wall_round_ms = dt / max(rounds_local, 1) * 1e3
    ksum = {k: v["avg_ms"] * (split["groups"] if k in ("extend", "shade") else 1) for k, v in kernels.items()
            if k in ("extend", "shade", "round", "rounds")}
    share_ms = wall_round_ms * ksum[dom] / max(sum(ksum.values()), 1e-12) if dom in ksum else None
    apportioned = ({"ms_per_round": round(share_ms, 4), "wall_ms_per_round": round(wall_round_ms, 4),
                    "achieved": round(ALG_BYTES[dom] * slots_owned / (share_ms * 1e-3) / 1e9, 2),
                    "frac": round(ALG_BYTES[dom] * slots_owned / (share_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5)}
                   if share_ms else None)
    # The committed PMC profile of this workload: the whole frame's launches
    # (N = 1 and sample shards), or rank 0's band partition with its path
    # streams (a launch over other slots than the whole frame's).
    pkey = str(args.config) if part_n == 1 else f"{args.config}:bands{part_n}x{streams}"
    prof = profile_for(pkey) or {}
    kprof = prof.get("kernels", {}).get(dom, {})
    traffic = kprof.get("hbm_bytes")
    # The roofline that binds the dominant kernel,
    # from the committed PMC of this workload, every figure in ONE machine
    # state -- the profiled dispatches, which rocprofv3 serialises:
    #   issue_frac   = VALU issue fraction x active lanes / 64 (the chip's
    #                  lane-issue capacity doing useful work),
    #   traffic_frac = the dispatches' HBM bytes / their own duration / peak.
    # Whichever resource is closer to its peak in that state binds; `bound`
    # says which, and the line's frac stays priced against HBM.
    dissue = (prof.get("issue") or {}).get(dom) or {}
    issue_frac = (round(dissue["valu_issue_frac"] * dissue["valu_active_lanes"] / 64.0, 4)
                  if "valu_issue_frac" in dissue and "valu_active_lanes" in dissue else None)
    dispatch_ms = kprof.get("dispatch_ms")
    traffic_frac = (round(traffic / (dispatch_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
                    if traffic is not None and dispatch_ms else None)
    if "valu_issue_frac" not in dissue or traffic_frac is None:
        binding = None
    elif dissue["valu_issue_frac"] > traffic_frac:
        binding = "valu_issue"
    else:
        binding = "hbm"
    # Which image property the N-GPU frame keeps (VERDICT r04 #7 / ADVICE r04):
    # band partitions with one path stream are the one-GPU frame bit for bit;
    # sample shards and band path streams add independent RNG streams
    # (FrameIndex offsets), the same estimator with the same sample count.
    if world == 1 and streams == 1:
        identity = ("bit-identical to the oracle's frame (the CPU restatement of the reference integrator; "
                    "tests/test_gpu_bench_path.py checks this schedule at full size)")
    elif shard == "bands" and streams == 1:
        identity = "bit-identical to the 1-GPU frame (disjoint bands, same seeds)"
    else:
        identity = (f"same estimator as the 1-GPU frame, not bit-identical: "
                    + (f"{streams} path streams per pixel seeded FrameIndex + (k << 24)" if shard == "bands"
                       else "each rank's RNG stream starts at FrameIndex + (rank << 24)"))
    xname = "RCCL" if exchange == "rccl" else "gloo (host-memory fallback)"
    metric = ("Mrays/s + Msamples/s, Viking Room 1920x1080 1024spp, 1/2/4/8 GPUs" if args.config == 3 and spp == 1024
              else f"Mrays/s + Msamples/s, C{args.config} {info.width}x{info.height} {spp}spp")
    out = {
        "metric": metric,
        "value": round(mrays, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic (procedural {info.mesh_face_count}-triangle room mesh + 1024^2 texture; "
                "Viking Room asset absent)",
        "config": {
            "workload": (f"C{args.config} scene, one {width}x{height} {spp}-spp frame per step (Reset, Run(2), "
                         f"Run(1) until the frame's sample count reaches {spp} x pixels), split in 16-row bands over "
                         f"{world} GPU(s) ({px_owned} px on rank 0, {streams} path stream(s) per pixel) + the bands' "
                         f"gather to rank 0"
                         if shard == "bands" else
                         f"C{args.config} scene, one {width}x{height} {spp}-spp frame per step (Reset, Run(2), "
                         f"Run(1) until the frame's sample count reaches {spp} x pixels); each of {world} GPU(s) "
                         f"renders every pixel with its own RNG stream to 1/{world} of the samples, then the "
                         f"reduce of radiance + sample counts to rank 0"),
            "shard": shard,
            "exchange": exchange,
            "comm_ranks": comm_ranks,
            "spp_target": spp,
            "streams": streams,
            "slots_per_launch_rank0": slots_owned,
            "split": split["groups"],
            "class_lists": class_lists,
            "frame_target_samples_rank0": target,
            "mesh_faces": info.mesh_face_count,
            "image_identity": identity,
            "parallelism": (f"pixel-bands x{world}" + (f" + {xname} band gather to rank 0" if world > 1 else "")
                            if shard == "bands" else
                            f"sample-shards x{world}" + (f" + {xname} reduce of radiance + sample counts to rank 0"
                                                         if world > 1 else "")),
        },
        "msamples_per_s": round(samples / dt / 1e6, 3),
        "frame": {
            "frame_s": round(dt / args.steps, 4),
            "rounds_per_frame_rank0": [f[0] for f in frames],
            "rounds_all_ranks": int(rounds_all),
            "samples_per_frame_rank0": [f[1] for f in frames],
            "rays": int(rays),
            "samples": int(samples),
        },
        "steady_state": steady,
        "roofline": {
            # The limiter of the dominant kernel in its profiled state (HBM
            # or VALU issue); peak / frac are the HBM roofline either way.
            "bound": binding or "hbm",
            "priced_against": "hbm",
            "kernel": dom,
            # The dominant kernel's share of the chip: the frame's wall time
            # per round apportioned among the kernels by their summed launch
            # time per round (tile groups run K launches of each kernel
            # concurrently), its algorithmic bytes per round over that share.
            # Kernel time <= step time by construction.
            "achieved": apportioned["achieved"] if apportioned else round(achieved, 2),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": apportioned["frac"] if apportioned else round(achieved / HBM_PEAK_GBPS, 5),
            "frac_basis": "apportioned chip share per round" if apportioned else "per launch",
            "traffic": traffic,
            "traffic_unit": "bytes per launch (HBM, PMC)",
            "traffic_source": prof.get("profile") if traffic is not None else None,
            "alg_bytes_per_launch": round(ALG_BYTES[dom] * launch_slots),
            "alg_bytes_per_round": round(ALG_BYTES[dom] * slots_owned),
            "split_groups": split["groups"],
            "slots_per_timed_launch": round(launch_slots),
            "apportioned": apportioned,
            # One timed launch's own rate: its bytes over its own duration.
            # With tile groups, `split_groups` such launches overlap, so this
            # is not a share of the chip (secondary).
            "per_launch": {"avg_ms": round(kernels[dom]["avg_ms"], 4), "achieved": round(achieved, 2),
                           "frac": round(achieved / HBM_PEAK_GBPS, 5)},
            "alg_bytes_per_slot": ALG_BYTES[dom],
            "launch_avg_ms": {k: round(v["avg_ms"], 4) for k, v in kernels.items()},
            "launches_timed": {**{k: v[0] for k, v in kstats.items()}, "every_nth_round": args.profile_period},
            "rounds_timed": {k: v[2] for k, v in kstats.items()},
            "path_gbps_220B_per_ray": round(PATH_BYTES_PER_RAY * rays / dt / 1e9, 2),
            # BASELINE.md's whole-path definition: 220 B per ray over the frame time.
            "path_frac": round(PATH_BYTES_PER_RAY * rays / dt / 1e9 / HBM_PEAK_GBPS, 5),
            # Both from the committed PMC's serialised dispatches (above).
            "traffic_frac": traffic_frac,
            "issue_frac": issue_frac,
            "pmc_state": "serialised profiled dispatches (rocprofv3 --pmc): counters and durations of the same dispatches",
            "pmc_dispatch_ms": dispatch_ms,
            "binding": binding,
        },
        # What bounds the dominant kernel instead of HBM (PMC of this config's
        # committed profile): fraction of the chip's VALU issue slots used and
        # active lanes per VALU instruction (of 64; divergence).  null when no
        # profile of this config is committed.
        "limiter": ({"kind": "valu_issue", "kernel": dom, **(prof.get("issue", {}).get(dom) or {}),
                     "per_kernel": {k: prof.get("issue", {}).get(k) for k in ("extend", "shade", "round", "rounds")
                                    if prof.get("issue", {}).get(k)},
                     "source": prof.get("profile"), "profile_key": pkey} if prof else None),
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
        "cache_gbps": round(cache_bytes * launch_slots / (avg_ext * 1e-3) / 1e9, 1),
        "l2_peak_gbps": L2_PEAK_GBPS,
    }
    if not args.no_cpu_baseline and world == 1:   # rank 0 at N=1 only
        out["cpu_baseline"] = cpu_baseline(pt, scene, info.width, info.height, args.config)
    print(json.dumps(out), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
