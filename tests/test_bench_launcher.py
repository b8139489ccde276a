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


def test_compact_line_fits_the_driver_tail():
    """The stdout line stays a few KB (round 4's 20 KB line overflowed the driver's
    tail): rebuilt from round 4's full record, it keeps the contract's fields, the
    roofline, the CPU baseline, parity, latency and one summary per leg."""
    sys.path.insert(0, ROOT)
    import bench
    with open(os.path.join(ROOT, "profiles", "archive", "r04_bench.json")) as f:
        full = json.load(f)
    full["build"] = bench.source_identity()
    line = bench.compact_line(full, "profiles/bench_detail_x.json")
    s = json.dumps(line)
    assert len(s) <= 6000, len(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
              "roofline", "cpu_baseline", "parity_sample", "latency_ms", "legs", "detail"):
        assert k in line, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in line["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"], k
    assert set(line["legs"]) == {"C3", "C4", "C5_custom", "C5_date"}
    assert all("ms_per_step" in v and "frac" in v for v in line["legs"].values())


def test_line_reports_the_shard_transport():
    """world > 1: the line names how the shards' collectives travelled and the RCCL
    communicators' rank counts (min / max over the ranks, from yrwi_shard_info), so
    an 8-GPU record shows that RCCL saw 8 ranks -- or that it did not."""
    sys.path.insert(0, ROOT)
    import bench
    with open(os.path.join(ROOT, "profiles", "archive", "r04_bench.json")) as f:
        full = json.load(f)
    info = lambda r, t, n, peers: {"transport": t, "rank": r, "world": 8, "rccl_ranks": n, "lanes": 8,
                                   "lanes_own_comm": 8 if n else 0, "device_peers": peers, "mailbox": 1,
                                   "pci_bus_id": f"0000:{r:02x}:00.0"}
    full["shard_transport"] = bench.transport_summary([info(r, "rccl", 8, 0) for r in range(8)])
    line = bench.compact_line(full, "profiles/bench_detail_x.json")
    assert len(json.dumps(line)) <= 6000
    assert line["transport"] == "rccl" and line["rccl_ranks"] == {"min": 8, "max": 8}
    assert "k_compact" in line["roofline_kernels"] and "frac" in line["roofline_kernels"]["k_compact"]
    mixed = bench.transport_summary([info(0, "rccl", 2, 0), info(1, "host-staged", 0, 1)])
    assert mixed["transport"] == ["rccl", "host-staged"] and mixed["rccl_ranks"] == {"min": 0, "max": 2}
    assert mixed["ranks_sharing_a_device"] == 1
    assert bench.transport_summary([None, None]) is None
    # one GPU: no transport keys
    full.pop("shard_transport")
    assert "transport" not in bench.compact_line(full, "x")
