"""GPU-vs-oracle fuzz over the per-lane kernel's shapes (a checker run by hand
on the GPU box, not collected by pytest: it takes minutes).

Draws schedules around the BASELINE configs so that every routing is hit
often: the simple-schedule shape (loss-free, skew-free single decree with
delays <= 4, layout 6), the compact 4-step and 8-step layouts, the slim
three-proposer split (fuzzed P), faulty log mode, and the general kernel
beyond them.  Every batch is compared with the C oracle instance by instance
(results, digests) and in its run totals.

    python tests/fuzz_gpu.py [n_configs] [instances_per_config] [seed] [kinds]

kinds: a comma list to cycle through (default simple,simple,compact,split,log,any,
the rounds 4-6 runs; p3 adds three-proposer schedules that are not fuzzed per
instance).
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "cloud-haskell-paxos_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_c  # noqa: E402
import pxb  # noqa: E402


def draw(rng, kind):
    P = int(rng.integers(1, 3))
    N = int(rng.integers(2, 10))
    crash = int(rng.choice([0, rng.integers(1, 400000), 1000000]))
    common = dict(seed=int(rng.integers(0, 1 << 63)), n_proposers=P, n_acceptors=N, crash_ppm=crash,
                  crash_len_max=int(rng.integers(1, 40)), crash_start_max=int(rng.integers(0, 30)),
                  step_cap=int(rng.choice([int(rng.integers(1, 64)), 256, 300, 1024])))
    if kind == "simple":              # layout 6: no loss, no skew, delays <= 4
        return pxb.Config(loss_ppm=0, delay_max=int(rng.integers(1, 5)), skew_max=0, **common)
    if kind == "compact":             # compact 4- and 8-step layouts (loss and skew)
        return pxb.Config(loss_ppm=int(rng.integers(0, 400000)), delay_max=int(rng.integers(1, 9)),
                          skew_max=int(rng.integers(0, 6)), **common)
    if kind == "split":               # fuzzed P (the two-proposer kernel, then the three-proposer one)
        common.update(n_proposers=3, n_acceptors=int(rng.integers(5, 10)))
        return pxb.Config(loss_ppm=int(rng.integers(0, 400000)), delay_max=int(rng.integers(1, 9)),
                          skew_max=int(rng.integers(0, 4)), randomize=True, **common)
    if kind == "p3":                  # three proposers on every instance (not fuzzed): slim / compact / general
        common.update(n_proposers=3)
        return pxb.Config(loss_ppm=int(rng.integers(0, 400000)), delay_max=int(rng.integers(1, 9)),
                          skew_max=int(rng.integers(0, 4)), **common)
    if kind == "log":                 # faulty log mode (the per-lane LG shape, delays <= 8)
        return pxb.Config(loss_ppm=int(rng.integers(0, 200000)), delay_max=int(rng.integers(1, 9)),
                          skew_max=int(rng.integers(0, 4)), n_ticks=int(rng.integers(2, 12)),
                          tick_period=int(rng.integers(1, 16)), **common)
    return pxb.Config(loss_ppm=int(rng.integers(0, 1000001)), delay_max=int(rng.integers(1, 16)),
                      skew_max=int(rng.integers(0, 12)), **common)     # anything (general kernel too)


def main():
    n_cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    rng = np.random.default_rng(int(sys.argv[3]) if len(sys.argv) > 3 else 0xF022)
    kinds = sys.argv[4].split(",") if len(sys.argv) > 4 else ["simple", "simple", "compact", "split", "log", "any"]
    t0 = time.time()
    bad = 0
    for i in range(n_cfg):
        kind = kinds[i % len(kinds)]
        cfg = draw(rng, kind)
        first = int(rng.integers(0, 1 << 40))
        res, dig, _, cnt = pxb.run(cfg, first, n)
        eres, edig, _, ecnt = oracle_c.run_cpu(cfg, first, n, threads=16)
        ok = np.array_equal(res, eres) and np.array_equal(dig, edig) and cnt == ecnt
        if not ok:
            bad += 1
            d = np.nonzero((res != eres).any(1) | (dig != edig).any(1))[0]
            print("MISMATCH %s first=%d %s: %d instances differ (first %s); totals equal: %s" % (
                kind, first, cfg, d.size, d[:3].tolist(), cnt == ecnt), flush=True)
        if i % 20 == 19:
            print("%d configs, %d mismatches, %.0f s" % (i + 1, bad, time.time() - t0), flush=True)
    print("done: %d configs x %d instances, %d mismatches" % (n_cfg, n, bad), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
