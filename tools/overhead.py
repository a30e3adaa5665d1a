"""Diagnostic: per-launch cost of the config-2 kernel with and without its
output stream, and of a tiny launch (fixed overhead).
    python tools/overhead.py [lib.so]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cloud-haskell-paxos_amd"))
import torch  # noqa: E402
import pxb  # noqa: E402

if len(sys.argv) > 1:
    pxb.load(os.path.join(ROOT, sys.argv[1]))
cfg = pxb.CONFIGS[2]
n = 1 << 20
out = torch.empty((n, 4), dtype=torch.int32, device="cuda")
dig = torch.empty((n, 5), dtype=torch.int32, device="cuda")
tot = torch.zeros(16, dtype=torch.int64, device="cuda")


def timeit(label, m, outputs, reps=20):
    for k in range(3):
        pxb.run_device(cfg, k * m, m, d_results=out if outputs else None, d_digests=dig if outputs else None,
                       d_totals=tot)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(reps):
        pxb.run_device(cfg, (k + 3) * m, m, d_results=out if outputs else None,
                       d_digests=dig if outputs else None, d_totals=tot)
    e1.record()
    torch.cuda.synchronize()
    print("%-34s %9.1f us per launch" % (label, e0.elapsed_time(e1) * 1e3 / reps), flush=True)


timeit("config 2, 2^20, with outputs", n, True)
timeit("config 2, 2^20, totals only", n, False)
timeit("config 2, 2^19, with outputs", n // 2, True)
timeit("config 2, 2^18, with outputs", n // 4, True)
timeit("config 2, 12 x 4096 (1 gen/wave)", 12 * 4096, True)
timeit("config 2, 1 instance", 1, True)
