"""bench.py's N-rank launch path on the CPU (`bench.py --gpus N`
must produce an N-rank line without an external launcher).  --launch-check
runs the launcher, the gloo process group, the max-over-ranks reduction and a
frame-end reduce without touching a GPU."""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def run_bench(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True, env=env,
                       timeout=300)
    return p


def test_gpus2_self_launches_two_ranks():
    p = run_bench(["--gpus", "2", "--launch-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout          # one JSON line, from rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and d["config"]["comm_ranks"] == 2
    assert d["max_over_ranks"] == 2.0 and d["reduce_ok"]


def test_gpus8_self_launches_eight_ranks():
    """The driver's N = 8 launch: eight self-launched gloo
    ranks, one line from rank 0 with n_gpus 8 and the max over all ranks."""
    p = run_bench(["--gpus", "8", "--launch-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["world_size"] == 8 and d["config"]["comm_ranks"] == 8
    assert d["max_over_ranks"] == 8.0 and d["reduce_ok"]


def test_world_size_must_match_gpus():
    p = run_bench(["--gpus", "4", "--launch-check"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2 and "WORLD_SIZE=2 but --gpus 4" in p.stderr


def test_failing_rank_ends_launch_nonzero():
    """Failure path: a rank that raises before the
    frame-end exchange, while its peer is blocked in it, ends the whole
    N-rank launch with a non-zero status within a bound (the launcher stops
    the surviving rank; nothing waits for a collective that cannot finish)."""
    import time
    t0 = time.perf_counter()
    p = run_bench(["--gpus", "2", "--launch-check", "--inject-failure", "1"])
    dt = time.perf_counter() - t0
    assert p.returncode != 0
    assert "injected failure on rank 1" in p.stderr
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]   # no result line
    assert dt < 90.0, f"failed launch took {dt:.1f} s to end"
