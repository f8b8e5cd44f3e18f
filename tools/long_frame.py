"""A whole benchmark frame against the oracle: ptRenderFrame at a config's
full size and spp target with every scheduling mode automatic (the bench's
schedule: tile groups, class lists, split batches, the guarded end), then the
oracle running Reset, Run(2) and Run(1) rounds to the same round count.
Checks that the frame ended at the first round whose completed-path total
reaches the target (one round earlier the oracle is short of it), the
sample count, and every accumulated pixel and slot state bit for bit.
Prints progress to stderr and one JSON line.

usage: python tools/long_frame.py [CONFIG] [SPP]   (default C3, its 1024 spp)
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    import __graft_entry__ as ge
    import oracle_lib
    from test_gpu_parity import compare_state
    pt = ge._load_package()
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    s = pt.Scene.config(config)
    info = s.info
    W, H = info.width, info.height
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else info.spp
    target = spp * W * H
    dev = pt.Device(0)
    ds = pt.DeviceScene(dev)
    ds.update(s)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = info.render_flags
    r.PathTerminationProbability = info.termination_probability
    split, lists = r.split(), r.class_lists()
    t0 = time.time()
    rounds, samples = r.render_frame(target)
    gpu_s = time.time() - t0
    ga, gs = sb.read(), r.read_state()
    for x in (r, sb, ds, dev):
        x.close()
    print(f"gpu frame: {rounds} rounds, {samples} samples, {gpu_s:.2f} s", file=sys.stderr, flush=True)
    o = oracle_lib.OracleRenderer(s.packs(), W, H)
    o.RenderFlags = info.render_flags
    o.PathTerminationProbability = info.termination_probability
    t0 = time.time()
    o.reset()
    o.run(2)
    for i in range(rounds - 3):
        o.run(1)
        if i % 100 == 99:
            print(f"oracle round {i + 3} of {rounds}, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    _, before = o.counters()
    o.run(1)
    _, osamples = o.counters()
    oa = o.accum()
    state_ok = True
    try:
        compare_state(gs, o.state())
    except AssertionError as e:   # noqa: PERF203
        state_ok = str(e)
    o.close()
    diff = int(np.count_nonzero(np.any(ga.view(np.uint32) != oa.view(np.uint32), axis=-1)))
    out = {"config": config, "W": W, "H": H, "spp": spp, "target": target, "split": split, "class_lists": lists,
           "rounds": rounds, "gpu_samples": samples, "oracle_samples": osamples,
           "oracle_before_last_round": before, "ends_at_first_round_reaching_target": before < target <= osamples,
           "samples_equal": samples == osamples, "differing_pixels": diff, "state_bit_exact": state_ok,
           "gpu_s": round(gpu_s, 2), "oracle_s": round(time.time() - t0, 1)}
    print(json.dumps(out), flush=True)
    ok = out["ends_at_first_round_reaching_target"] and out["samples_equal"] and diff == 0 and state_ok is True
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
