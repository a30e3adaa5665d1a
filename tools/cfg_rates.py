"""Throughput and canonical-roofline fraction per BASELINE config (diagnostic).
    python tools/cfg_rates.py [lib.so]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cloud-haskell-paxos_amd"))
import torch  # noqa: E402
import pxb  # noqa: E402

if len(sys.argv) > 1:
    pxb.load(os.path.join(ROOT, sys.argv[1]))
CASES = ((2, 1 << 20, 10), (3, 1 << 22, 2), (4, 1 << 23, 2), (4, 1 << 26, 1), (5, 1 << 22, 1), (6, 1 << 20, 3))
if os.environ.get("PXB_RATES_QUICK"):
    CASES = tuple(c for c in CASES if c[1] <= (1 << 23))
if os.environ.get("PXB_RATES_CONFIGS"):
    keep = [int(x) for x in os.environ["PXB_RATES_CONFIGS"].split(",")]
    CASES = tuple(c for c in CASES if c[0] in keep)
for c, n, reps in CASES:
    cfg = pxb.CONFIGS[c]
    N = cfg.n_acceptors
    out = torch.empty((n, 4), dtype=torch.int32, device="cuda")
    dig = torch.empty((n, N), dtype=torch.int32, device="cuda")
    tot = torch.zeros(16, dtype=torch.int64, device="cuda")
    pxb.run_device(cfg, 0, min(n, 1 << 20), d_results=out, d_digests=dig, d_totals=tot)
    torch.cuda.synchronize()
    tot.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(reps):
        pxb.run_device(cfg, (k + 1) * n, n, d_results=out, d_digests=dig, d_totals=tot)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    t = pxb.counters_dict(tot.cpu().tolist())
    gbs = t["canon_bytes"] / reps / (ms * 1e-3) / 1e9
    print("config %d  n=%-9d %9.3f ms  %8.1f Minst/s  %7.1f Mdecided/s  canon %6.0f B/inst  %6.0f GB/s = %.3f of 8 TB/s  "
          "steps/inst %.1f  msgs/inst %.1f" % (c, n, ms, n / ms / 1e3, t["decided"] / reps / ms / 1e3,
                                               t["canon_bytes"] / t["instances"], gbs, gbs / 8000,
                                               t["steps"] / t["instances"], t["messages"] / t["instances"]), flush=True)
