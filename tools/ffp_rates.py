"""Fault-free per-lane kernel for duelling proposers / log mode vs the general
fault-free kernel (PXB_NO_FFP=1): ms per batch on this GPU.
    python3 tools/ffp_rates.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cloud-haskell-paxos_amd"))
import pxb  # noqa: E402

CASES = {
    "log_mode (P2 N2, 16 Ticks)": (pxb.LOG_CONFIG, 1 << 22),
    "duel P2 N5 skew2": (pxb.Config(seed=0xD0E1, n_proposers=2, n_acceptors=5, skew_max=2, step_cap=600), 1 << 22),
    "duel P3 N9 skew2": (pxb.Config(seed=0xD0E2, n_proposers=3, n_acceptors=9, skew_max=2, step_cap=600), 1 << 22),
    "log P1 N5 8 Ticks": (pxb.Config(seed=0x5EED0006, n_proposers=1, n_acceptors=5, n_ticks=8, tick_period=6), 1 << 22),
}
tot = torch.zeros(16, dtype=torch.int64, device="cuda")
for name, (cfg, n) in CASES.items():
    line = []
    for mode, env in (("per_lane", {}), ("general", {"PXB_NO_FFP": "1"})):
        os.environ.pop("PXB_NO_FFP", None)
        os.environ.update(env)
        pxb.reload_hooks()
        pxb.run_device(cfg, 1 << 36, 1 << 16, d_totals=tot)
        torch.cuda.synchronize()
        tot.zero_()
        t0 = time.perf_counter()
        pxb.run_device(cfg, 0, n, d_totals=tot)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0)
        c = pxb.counters_dict(tot.cpu().tolist())
        line.append("%s %.2f ms (%.0f M/s, executes %d)" % (mode, ms, n / ms / 1e3, c["executes"]))
    print("%-28s %s" % (name, "   ".join(line)), flush=True)
