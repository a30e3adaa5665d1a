"""bench.py's N-rank path on CPU: `--gpus N` outside torchrun spawns N ranks
through torch.distributed.run (127.0.0.1 rendezvous); each rank runs the same
timed region (barriers, max-over-ranks time) and the totals are all-reduced
before rank 0 prints the one JSON line.  --dry-run swaps the GPU work for a
synthetic stand-in on gloo, so this checks the launcher and collectives only."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                         timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_launcher_ranks(gpus):
    """The headline shape (BASELINE config 4, the north star): one batch per
    step split over the ranks (strong scaling), totals all-reduced."""
    j = _bench("--dry-run", "--gpus", str(gpus), "--steps", "3", "--warmup", "1", "--instances", "500")
    assert j["n_gpus"] == gpus and j["config"]["rccl_world"] == gpus and j["scaling"] == "strong"
    assert j["config"]["instances_per_gpu_per_step"] * gpus == j["config"]["instances_per_step"] == 500 // gpus * gpus
    assert j["counters"]["instances"] == 500 // gpus * gpus * 3     # all-reduced over the ranks
    assert j["steps"] == 3 and j["ms_per_step"] > 0 and j["value"] > 0
    assert "config 4 (north star)" in j["config"]["workload"]
    # the default batch: the dry-run stand-in for 2^26
    j = _bench("--dry-run", "--gpus", str(gpus), "--steps", "2", "--warmup", "0")
    assert j["config"]["instances_per_step"] == 1 << 12 and j["counters"]["instances"] == 2 << 12


def test_bench_defaults_to_north_star():
    sys.path.insert(0, ROOT)
    import bench
    import argparse
    old = sys.argv
    sys.argv = ["bench.py"]
    try:
        a = bench.parse()
    finally:
        sys.argv = old
    assert isinstance(a, argparse.Namespace) and a.config == 4 and a.gpus == 1


def test_bench_rejects_world_mismatch():
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--gpus", "2"],
                         capture_output=True, text=True, timeout=120, env={**os.environ, **env}, cwd=ROOT)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr


def test_step_instances_sized_from_world():
    """Configs 4 and 5 are one batch over the node (64M over 8 GPUs, 256M):
    each rank's share is that batch / world; config 2 is a fixed batch per GPU."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.step_instances(4, 0, 1) == 1 << 26 and bench.step_instances(4, 0, 8) == 1 << 23
    assert bench.step_instances(5, 0, 8) == 1 << 25 and bench.step_instances(5, 0, 2) == 1 << 27
    assert bench.step_instances(2, 0, 1) == bench.step_instances(2, 0, 8) == 1 << 28
    assert bench.scaling_of(4) == "strong" and bench.scaling_of(2) == "weak"
