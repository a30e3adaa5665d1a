"""Diagnostic (never a bench number): per-wave timeline of one per-lane-kernel
launch from a library built with -DPXB_WAVE_TIMES (tools/build_wt.sh):
start, end and last work-queue grab of every wave (s_memrealtime, 100 MHz),
so the launch's tail -- how long waves sit finished while others still run --
can be measured instead of guessed.

    python tools/ev_wave_times.py variants/v_wt.so <config> <instances> [first]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cloud-haskell-paxos_amd"))
import torch  # noqa: E402
import pxb  # noqa: E402


def main():
    lib_path, c, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    first = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 36
    lib = pxb.load(os.path.join(ROOT, lib_path))
    lib.pxb_debug_wave_times.argtypes = [C.c_void_p, C.c_uint]
    lib.pxb_debug_wave_times.restype = C.c_int
    cfg = pxb.CONFIGS[c]
    tot = torch.zeros(16, dtype=torch.int64, device="cuda")
    pxb.run_device(cfg, first, min(n, 1 << 20), d_totals=tot)      # warm
    torch.cuda.synchronize()
    tot.zero_()
    pxb.run_device(cfg, first + n, n, d_totals=tot)
    torch.cuda.synchronize()
    buf = np.zeros((65536, 6), dtype=np.uint64)
    nw = lib.pxb_debug_wave_times(C.c_void_p(buf.ctypes.data), 65536)
    w = buf[:nw].astype(np.float64)
    t0 = w[:, 0].min()
    start, end, grab, taken = (w[:, 0] - t0) * 10e-6, (w[:, 1] - t0) * 10e-6, (w[:, 2] - t0) * 10e-6, w[:, 3]
    span = end.max()
    print("config %d, %d instances, %d waves: span %.3f ms" % (c, n, nw, span))
    print("wave start: max %.3f ms" % start.max())
    pct = np.percentile(end, [0, 10, 50, 90, 99, 100])
    print("wave end   ms: min %.3f p10 %.3f p50 %.3f p90 %.3f p99 %.3f max %.3f" % tuple(pct))
    print("last grab  ms: p50 %.3f p90 %.3f max %.3f" % tuple(np.percentile(grab, [50, 90, 100])))
    print("idle wave-time after each wave's end: %.2f %% of waves x span" % (100 * (span - end).sum() / (nw * span)))
    print("instances grabbed per wave: min %d mean %.1f max %d" % (taken.min(), taken.mean(), taken.max()))
    late = end > np.percentile(end, 90)
    print("the last 10 %% of waves to end: last grab at %.3f ms (median), end %.3f ms (median)" % (
        np.median(grab[late]), np.median(end[late])))
    print("totals", pxb.counters_dict(tot.cpu().tolist())["instances"])
    # placement: HW_ID = wave [3:0] simd [5:4] cu [11:8] sh [12] se [15:13]; XCC_ID [3:0]
    hw = buf[:nw, 4].astype(np.int64)
    xcc = buf[:nw, 5].astype(np.int64) & 15
    simd = (hw >> 4) & 3
    cu = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
    key = cu * 4 + simd
    _, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    per_simd = cnt[inv]                     # waves sharing this wave's SIMD
    ncu = len(np.unique(cu))
    print("CUs used %d, SIMDs used %d; waves per CU: %s" % (ncu, len(cnt), np.bincount(np.unique(cu, return_counts=True)[1])))
    for k in sorted(set(per_simd.tolist())):
        m = per_simd == k
        print("waves on SIMDs shared by %d: %4d waves, instances per wave mean %.0f (min %d max %d), "
              "per-SIMD rate %.0f" % (k, m.sum(), taken[m].mean(), taken[m].min(), taken[m].max(), k * taken[m].mean()))


if __name__ == "__main__":
    main()
