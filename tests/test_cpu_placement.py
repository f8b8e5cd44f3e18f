"""CPU: bench.pick_cores, the CPU baseline's thread placement (DESIGN §4
"CPU baseline"): n logical CPUs of the affinity mask on n distinct physical
cores of one package, or None with a reason."""
from __future__ import annotations

import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def topo(c):
    base = Path(f"/sys/devices/system/cpu/cpu{c}/topology")
    return int((base / "physical_package_id").read_text()), int((base / "core_id").read_text())


def test_pick_cores_distinct_cores_one_package():
    allowed = os.sched_getaffinity(0)
    n = max(1, min(2, len(allowed)))
    cpus, why = bench.pick_cores(n, sample_s=0.05)
    if cpus is None:
        assert "unpinned" in why
        return
    assert len(cpus) == n and cpus <= allowed
    t = [topo(c) for c in cpus]
    assert len(set(t)) == n, "two threads on one physical core"
    assert len({p for p, _ in t}) == 1, "threads on two packages"
    assert f"{n} threads pinned" in why


def test_pick_cores_too_many():
    allowed = os.sched_getaffinity(0)
    cpus, why = bench.pick_cores(len(allowed) + 1, sample_s=0.05)
    assert cpus is None and "unpinned" in why
