"""Multi-rank sharding on CPU (gloo, world_size 2 and 4): the all-reduced
totals of the sharded run equal the single-process totals, and the shards
tile the batch exactly.  The per-rank compute here is the CPU oracle (no GPU
in this container); on GPUs bench.py runs the same shard/all-reduce code
with the HIP path and RCCL."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import dist as pdist
import oracle_c
import pxb


def test_shard_ranges_tile_the_batch():
    for world in (1, 2, 3, 8):
        for first, n in ((0, 1000), (7, 1), (5, 0), (1 << 40, 12345)):
            cur = first
            for r in range(world):
                lo, hi = pdist.shard_range(r, world, first, n)
                assert lo == cur and hi >= lo
                cur = hi
            assert cur == first + n


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, c, first, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def run_fn(cfg, lo, count):
        _, _, _, cnt = oracle_c.run_cpu(cfg, lo, count, threads=1)
        return [cnt[k] for k in pxb.COUNTER_NAMES]

    tot = pdist.run_sharded(run_fn, pxb.CONFIGS[c], first, n, rank, world)
    if rank == 0:
        q.put(tot.tolist())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,c", [(2, 3), (4, 5)])
def test_gloo_sharded_totals_match_single_process(world, c):
    first, n = 1000, 3000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, c, first, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, _, _, exp = oracle_c.run_cpu(pxb.CONFIGS[c], first, n, threads=2)
    assert got == [exp[k] for k in pxb.COUNTER_NAMES]
