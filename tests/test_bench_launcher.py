"""bench.py's rank launcher (CPU, no GPU).

`python bench.py --gpus N` started without torch.distributed.run (WORLD_SIZE unset)
starts its N rank processes itself, with the environment the driver's launcher would
give them, and rank 0 prints the one JSON line.  `--plumbing` stops each rank right
after the gloo group is up, so the wiring (ranks, world size, the max-over-ranks
reduction bench.py times with) is checked without a GPU.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env,
                          cwd=ROOT)


@pytest.mark.parametrize("n", [2, 3])
def test_bare_bench_spawns_its_ranks(n):
    r = _run(["--gpus", str(n), "--plumbing"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]   # gloo logs its own lines
    assert len(lines) == 1, r.stdout   # rank 0 alone prints the JSON line
    out = json.loads(lines[0])
    assert out["world"] == n and out["rank"] == 0 and out["local_rank"] == 0
    assert out["max_rank"] == n - 1   # the max-over-ranks reduction saw every rank


def test_single_gpu_needs_no_launcher():
    r = _run(["--gpus", "1", "--plumbing"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out == {"rank": 0, "world": 1, "local_rank": 0, "max_rank": 0.0}


def test_launcher_env_mismatch_fails_loudly():
    # under a launcher (WORLD_SIZE set) --gpus must agree with it
    r = _run(["--gpus", "2", "--plumbing"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in (r.stderr + r.stdout)
