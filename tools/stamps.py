"""Diagnostic: per-section cycle shares of the batch kernel (variants/stamps.so,
built with -DPXB_STAMPS).  Never a timing number: read the shares only."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PXB_LIB", os.path.join(ROOT, "variants", "stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "cloud-haskell-paxos_amd"))
import torch  # noqa
import pxb  # noqa

NAMES = ["refill", "acceptor", "prop_tick+count", "prop_fast", "prop_multi", "endstep", "finish", "exit"]
CNAMES = ["wave-steps", "acc-iters", "fast-rounds", "multi-calls", "multi-rounds", "philox-sites", "max-slot-rounds", "active-slots"]
lib = pxb.load()
lib.pxb_debug_stamps.argtypes = [C.c_void_p]
for c, n in ((2, 1 << 20), (3, 1 << 22), (4, 1 << 22), (5, 1 << 20)):
    cfg = pxb.CONFIGS[c]
    out = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    tot = torch.zeros(16, dtype=torch.int64, device="cuda")
    pxb.run_device(cfg, 0, n, d_results=out, d_totals=tot)
    buf = (C.c_ulonglong * 16)()
    lib.pxb_debug_stamps(C.cast(buf, C.c_void_p))   # discard warmup
    pxb.run_device(cfg, n, n, d_results=out, d_totals=tot)
    lib.pxb_debug_stamps(C.cast(buf, C.c_void_p))
    total = sum(buf[:8])
    ws = max(buf[8], 1)
    steps = tot.cpu().tolist()[12] / 2
    print("config %d: %s" % (c, "  ".join("%s %.1f%%" % (NAMES[i], 100.0 * buf[i] / total) for i in range(8))))
    print("   total wave-cycles %.3g, per instance-step %.1f" % (total, total / steps))
    print("   per wave-step: " + "  ".join("%s %.3f" % (CNAMES[i], buf[8 + i] / ws) for i in range(1, 8)))
