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
    j = _bench("--dry-run", "--gpus", str(gpus), "--steps", "3", "--warmup", "1", "--instances", "500")
    assert j["n_gpus"] == gpus and j["rccl_world"] == gpus
    assert j["counters"]["instances"] == 500 * 3 * gpus     # all-reduced over the ranks
    assert j["steps"] == 3 and j["ms_per_step"] > 0


def test_bench_rejects_world_mismatch():
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--gpus", "2"],
                         capture_output=True, text=True, timeout=120, env={**os.environ, **env}, cwd=ROOT)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr
