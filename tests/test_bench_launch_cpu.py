"""bench.py's rank launch (reference: one process per GPU, main_train_psnr.py:52-54,122-130,
utils/utils_dist.py:13-28): `--gpus N` either is one rank of an N-process launch (torchrun) or
spawns the N ranks itself; a count that disagrees with WORLD_SIZE is refused."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launch_plan():
    assert bench.launch_plan(1, {}) == ("run", 1)
    assert bench.launch_plan(8, {}) == ("spawn", 8)
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}) == ("run", 4)
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == ("run", 1)
    with pytest.raises(SystemExit):
        bench.launch_plan(8, {"WORLD_SIZE": "1"})    # a scaling run must not time fewer GPUs silently
    with pytest.raises(SystemExit):
        bench.launch_plan(2, {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {})


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=240, env=env)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    """`python bench.py --gpus N` (no torchrun) starts N ranks that rendezvous on 127.0.0.1; rank 0 reports
    the world it measured (gloo dry run: no GPU is touched)."""
    r = _run(["--gpus", str(n), "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["ranks"] == list(range(n))


def test_mismatch_refused():
    r = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
