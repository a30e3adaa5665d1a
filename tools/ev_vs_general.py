"""Routing experiment (GPU): per-lane vs general kernel on fuzzed / long-delay
topologies whose per-lane layout fits few waves per CU.  Prints ms per batch
for each routing forced through the PXB_* environment switches.
    python3 tools/ev_vs_general.py [n_instances]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cloud-haskell-paxos_amd"))
import pxb  # noqa: E402

N_INST = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
CASES = {
    "c5": pxb.CONFIGS[5],
    "c5_d12": pxb.Config(seed=0x5EED0005, n_proposers=3, n_acceptors=9, loss_ppm=300000, delay_max=12,
                         crash_ppm=200000, crash_len_max=16, crash_start_max=16, skew_max=3, step_cap=512,
                         randomize=True),
    "p3n9_d8": pxb.Config(seed=0x77, n_proposers=3, n_acceptors=9, loss_ppm=100000, delay_max=8,
                          crash_ppm=200000, crash_len_max=16, crash_start_max=16, skew_max=3, step_cap=512),
    "p3n9_d12": pxb.Config(seed=0x78, n_proposers=3, n_acceptors=9, loss_ppm=100000, delay_max=12,
                           crash_ppm=200000, crash_len_max=16, crash_start_max=16, skew_max=3, step_cap=512),
    "p2n9_d12": pxb.Config(seed=0x79, n_proposers=2, n_acceptors=9, loss_ppm=100000, delay_max=12,
                           crash_ppm=200000, crash_len_max=16, crash_start_max=16, skew_max=3, step_cap=512),
    "p3n6_d6": pxb.Config(seed=0x7A, n_proposers=3, n_acceptors=6, loss_ppm=100000, delay_max=6,
                          crash_ppm=200000, crash_len_max=16, crash_start_max=16, skew_max=3, step_cap=512),
}
MODES = {"default": {}, "general": {"PXB_NO_EV": "1"}, "no_split": {"PXB_NO_SPLIT": "1"}}

tot = torch.zeros(16, dtype=torch.int64, device="cuda")
for name, cfg in CASES.items():
    line = []
    for mode, env in MODES.items():
        for k in ("PXB_NO_EV", "PXB_NO_SPLIT"):
            os.environ.pop(k, None)
        os.environ.update(env)
        pxb.reload_hooks()
        pxb.run_device(cfg, 1 << 36, 1 << 16, d_totals=tot)        # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pxb.run_device(cfg, 0, N_INST, d_totals=tot)
        torch.cuda.synchronize()
        line.append("%s %.1f ms" % (mode, 1e3 * (time.perf_counter() - t0)))
    print("%-10s %s" % (name, "   ".join(line)), flush=True)
