"""bench.py's launcher: `--gpus N` starts N rank processes itself (RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_* set, before anything touches a GPU); checked
on the CPU with the --dry-run rendezvous over gloo."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env=None):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout  # only rank 0 prints
    return lines[0]


def test_gpus_2_launches_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = _run("--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1", env=env)
    assert out["n_gpus"] == 2 and out["ranks_sum"] == 3.0 and out["steps"] == 3


def test_gpus_1_single_process():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = _run("--dry-run", env=env)
    assert out["n_gpus"] == 1
