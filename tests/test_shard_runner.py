"""pxb_run_multi's phase order (csrc/shard_runner.h) under injected shard
failures, with a fake backend on the host (tests/native/shard_host.cpp): the
call returns the failing shard's error promptly, the collective is issued for
all devices or for none, and every shard is torn down."""
import ctypes as C
import os
import subprocess
import time

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "shard_host.cpp")
HDR = os.path.join(HERE, "..", "cloud-haskell-paxos_amd", "csrc", "shard_runner.h")
OUT = os.path.join(HERE, "native", "_build", "libshard_host.so")


def lib():
    if not os.path.exists(OUT) or max(os.path.getmtime(SRC), os.path.getmtime(HDR)) > os.path.getmtime(OUT):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", OUT, SRC], check=True)
    return C.CDLL(OUT)


def run(G, phase, shard):
    counts = (C.c_int * 6)()
    t0 = time.perf_counter()
    rc = lib().shard_test(G, phase, shard, counts)
    return rc, dict(zip(("setup", "compute", "reduce", "abort", "fetch", "teardown"), counts)), time.perf_counter() - t0


@pytest.mark.parametrize("G", [1, 2, 8])
def test_clean_run(G):
    rc, c, _ = run(G, 0, 0)
    assert rc == 0
    assert c == dict(setup=G, compute=G, reduce=1, abort=0, fetch=G, teardown=G)


@pytest.mark.parametrize("G,shard", [(2, 0), (2, 1), (8, 5)])
def test_setup_failure_skips_everything_after(G, shard):
    rc, c, dt = run(G, 1, shard)
    assert rc == -2 and dt < 5
    assert c["compute"] == 0 and c["reduce"] == 0 and c["teardown"] == G


@pytest.mark.parametrize("G,shard", [(2, 1), (8, 0), (8, 7)])
def test_compute_failure_issues_no_collective(G, shard):
    rc, c, dt = run(G, 2, shard)
    assert rc == -3 and dt < 5
    assert c["compute"] == G and c["reduce"] == 0 and c["fetch"] == 0 and c["teardown"] == G


def test_collective_failure_aborts():
    rc, c, _ = run(4, 3, 0)
    assert rc == -5 and c["reduce"] == 1 and c["abort"] == 1 and c["fetch"] == 0 and c["teardown"] == 4


def test_fetch_failure_reported():
    rc, c, _ = run(4, 4, 2)
    assert rc == -2 and c["fetch"] == 4 and c["teardown"] == 4
