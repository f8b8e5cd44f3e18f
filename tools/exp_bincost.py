"""Experiment: can a cheap cost predictor recover the perfect longest-first
gain of the global ray sort?  (GPU; run under rocprofv3 --kernel-trace,
durations matched by tools/exp_reorder_report.py.)

tools/exp_gsort.py measured, on C3's settled rays, the (octant, origin cell)
sorted order at 0.64x of slot order when 256-ray blocks run longest-first by
their OWN step counts, but only 0.78x with the previous round's block costs
taken by block index.  Here the previous round's costs are attached to the
sort KEYS instead (per-bin cost), which a renderer can keep per bin:

  stale        key order, blocks longest-first by the previous round's cost
               of the block with the same index (exp_gsort's "stale");
  binmean      key bins ordered by the previous round's mean steps of the
               bin's rays (descending), key order inside; no block permutation
               (dispatch order = position order, so the order IS longest-first);
  binwave      the same with the bin cost from per-WAVE maxima of the previous
               round's sorted order (what an extend wave can store: its
               steps), a wave credited to the bin of its first ray;
  binwavemean / binwavemax   the bin cost from per-wave step sums (maxima
               x 64) of the previous round's sorted order, interpolated over
               the bin's position range (one store per wave), log-bucketed;
  binlpt       key order, blocks longest-first by the max predicted (binmean)
               cost of their rays;
  slotpred     rays ordered by the previous-round step count of their own
               slot's ray (log2 bucket, descending), then key;
  perfect      blocks longest-first by their own step counts (bound).
Rounds A -> B and B -> C are both measured.  Hits are identical in every
order (checked).
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "tools"))
import kat  # noqa: E402
from exp_gsort import keys, load  # noqa: E402


def main():
    pt = load()
    scene = pt.Scene.config(3)
    info = scene.info
    W, H = info.width, info.height
    dev = pt.Device(0)
    ds = pt.DeviceScene(dev)
    ds.update(scene)
    sb = pt.SampleBuffer(dev, W, H)
    r = pt.BasicRenderer(dev, ds, sb)
    r.RenderFlags = info.render_flags
    r.reset()
    r.run(2)
    for _ in range(30):
        r.run(1)
    dev.synchronize()
    y, x = np.divmod(np.arange(W * H), W)
    slot = ((y // 16) * (W // 16) + x // 16) * 256 + (y % 16) * 16 + x % 16
    base = np.argsort(slot, kind="stable")
    rays = []
    for _ in range(3):
        st = r.read_state().reshape(-1)
        rays.append((st["origin"][base].astype(np.float32), st["packed_velocity"][base].astype(np.uint32)))
        r.run(1)
        dev.synchronize()
    n = len(rays[0][1])
    dur = np.full(n, 1048576.0, np.float32)
    lo = np.minimum.reduce([o.min(0) for o, _ in rays])
    hi = np.maximum.reduce([o.max(0) for o, _ in rays])
    steps, K = [], []
    for O, PV in rays:
        steps.append(ds.trace_rays_stats(O, PV, dur)[1].astype(np.int64))
        K.append(keys(O, kat.unpack_unit_vector(PV), lo, hi))
    nb = (n + 255) // 256
    idx = np.arange(n)

    def block_cost(st):
        pad = np.zeros(nb * 256, np.int64)
        pad[:n] = st
        return pad.reshape(nb, 256).max(1)

    def by_blocks(p, cost):
        blocks = np.argsort(-cost, kind="stable")
        q = (blocks[:, None] * 256 + np.arange(256)[None, :]).reshape(-1)
        return p[q[q < n]]

    def bin_mean(k, st, nbins):
        c = np.bincount(k.astype(np.int64), weights=st, minlength=nbins)
        m = np.bincount(k.astype(np.int64), minlength=nbins)
        return np.where(m > 0, c / np.maximum(m, 1), 0.0)

    def bin_wave(k_sorted, st_sorted, nbins):
        nw = (n + 63) // 64
        pad = np.zeros(nw * 64, np.int64)
        pad[:n] = st_sorted
        wmax = pad.reshape(nw, 64).max(1)
        first = k_sorted[np.arange(nw) * 64].astype(np.int64)
        c = np.bincount(first, weights=wmax, minlength=nbins)
        m = np.bincount(first, minlength=nbins)
        return np.where(m > 0, c / np.maximum(m, 1), -1.0)   # unseen bins: last (would be any)

    def bin_wave_interp(k_sorted, st_sorted, nbins, use_max=False):
        """Per-wave sums (or max x 64) of the previous round's sorted order, a
        bin's cost = the interpolated prefix over its position range / count
        (what the renderer computes from one store per extend wave)."""
        nw = (n + 63) // 64
        pad = np.zeros(nw * 64, np.int64)
        pad[:n] = st_sorted
        w = pad.reshape(nw, 64)
        ws = (w.max(1) * 64) if use_max else w.sum(1)
        P = np.concatenate([[0], np.cumsum(ws)]).astype(np.float64)
        cnt = np.bincount(k_sorted.astype(np.int64), minlength=nbins)
        start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
        end = start + cnt

        def at(pos):
            wi = pos // 64
            return P[wi] + (P[np.minimum(wi + 1, nw)] - P[wi]) * (pos % 64) / 64.0

        c = (at(end) - at(start)) / np.maximum(cnt, 1)
        q = np.where(cnt > 0, np.floor(np.log2(np.maximum(c, 1.0)) * 32), -1)   # 32 buckets per octave
        return q

    orders = {}
    stats = {"corr_slot_steps": []}
    for a, b in ((0, 1), (1, 2)):
        sa, sb_ = steps[a], steps[b]
        stats["corr_slot_steps"].append(round(float(np.corrcoef(sa, sb_)[0, 1]), 3))
        for name in ("oct_cell8", "oct_cell8_dir4"):
            ka, kb = K[a][name], K[b][name]
            nbins = int(max(ka.max(), kb.max())) + 1
            pa = np.argsort(ka, kind="stable")
            pb = np.argsort(kb, kind="stable")
            tag = f"{name}|{a}{b}"
            orders[f"{tag}|stale"] = by_blocks(pb, block_cost(sa[pa]))
            cm = bin_mean(ka, sa, nbins)
            orders[f"{tag}|binmean"] = np.lexsort((idx, kb, -cm[kb.astype(np.int64)]))
            cw = bin_wave(ka[pa], sa[pa], nbins)
            orders[f"{tag}|binwave"] = np.lexsort((idx, kb, -cw[kb.astype(np.int64)]))
            cwi = bin_wave_interp(ka[pa], sa[pa], nbins)
            orders[f"{tag}|binwavemean"] = np.lexsort((idx, kb, -cwi[kb.astype(np.int64)]))
            cwx = bin_wave_interp(ka[pa], sa[pa], nbins, use_max=True)
            orders[f"{tag}|binwavemax"] = np.lexsort((idx, kb, -cwx[kb.astype(np.int64)]))
            pred = cm[kb[pb].astype(np.int64)]
            orders[f"{tag}|binlpt"] = by_blocks(pb, block_cost(np.round(pred * 16).astype(np.int64)))
            bucket = np.floor(np.log2(np.maximum(sa, 1))).astype(np.int64)
            orders[f"{tag}|slotpred"] = np.lexsort((idx, kb, -bucket))
            orders[f"{tag}|perfect"] = by_blocks(pb, block_cost(sb_[pb]))
            for o in ("binmean", "binwavemean", "slotpred"):
                w = np.zeros(((n + 63) // 64) * 64, np.int64)
                w[:n] = sb_[orders[f"{tag}|{o}"]]
                stats[f"{tag}|{o}|simd_eff"] = round(float(sb_.sum() / (w.reshape(-1, 64).max(1).sum() * 64)), 4)
    orders["slot_b"] = np.arange(n)
    print(json.dumps(stats, indent=1), flush=True)
    refs = {}
    log = []
    for name, p in orders.items():
        rb = 2 if "|12|" in name else 1
        O, PV = rays[rb]
        for k in range(3):
            h = ds.trace_rays(O[p], PV[p], dur)
            back = np.empty_like(h)
            back[p] = h
            if rb not in refs:
                refs[rb] = back
            same = bool(np.array_equal(back.view(np.uint8), refs[rb].view(np.uint8)))
            log.append({"order": name if name != "slot_b" else "slot", "rep": k, "identical": same})
            if not same:
                print("MISMATCH", name, flush=True)
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "exp_reorder_orders.json").write_text(json.dumps(log))
    (ROOT / "gpurun_out" / "exp_bincost_stats.json").write_text(json.dumps(stats, indent=1))
    for o in (r, sb, ds):
        o.close()
    dev.close()


if __name__ == "__main__":
    main()
