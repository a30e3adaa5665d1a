"""Diagnostic: per-wave run time spread of one launch (variants/wt.so, built
with -DPXB_WAVE_TIMES).  Shows how long the slowest waves keep the kernel
alive after the others have finished.
    python tools/wave_times.py [config ...]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PXB_LIB", os.path.join(ROOT, "variants", "wt.so"))
sys.path.insert(0, os.path.join(ROOT, "cloud-haskell-paxos_amd"))
import numpy as np  # noqa
import torch  # noqa
import pxb  # noqa

lib = pxb.load()
lib.pxb_debug_wave_times.argtypes = [C.c_void_p, C.c_uint]
SIZES = {2: 1 << 20, 3: 1 << 22, 4: 1 << 23, 5: 1 << 22, 6: 1 << 20}
for c in [int(x) for x in sys.argv[1:]] or [2, 3, 4, 5, 6]:
    cfg = pxb.CONFIGS[c]
    n = SIZES[c]
    out = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    tot = torch.zeros(16, dtype=torch.int64, device="cuda")
    for k in range(2):
        pxb.run_device(cfg, k * n, n, d_results=out, d_totals=tot)
    buf = np.zeros(6 * 65536, dtype=np.uint64)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    pxb.run_device(cfg, 2 * n, n, d_results=out, d_totals=tot)
    e1.record()
    torch.cuda.synchronize()
    nw = lib.pxb_debug_wave_times(buf.ctypes.data, 65536)
    r = buf[:6 * nw].reshape(nw, 6).astype(np.int64)
    mhz = (r[:, 5] - r[:, 4]) / np.maximum(r[:, 1] - r[:, 0], 1) * 100.0
    print("config %d: event time %.1f us; shader clock over wave lifetimes: mean %.0f MHz (p1 %.0f p99 %.0f)" % (
        c, e0.elapsed_time(e1) * 1e3, mhz.mean(), *np.percentile(mhz, [1, 99])))
    t = r[:, :2].copy()
    hw, xcc = r[:, 2], r[:, 3] & 15
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    cu_key = ((xcc * 8 + se) * 16 + cu)
    t -= t[:, 0].min()
    st, en = t[:, 0] * 10e-3, t[:, 1] * 10e-3          # 100 MHz ticks -> us
    dur = en - st
    xcd = np.arange(nw) % 8
    print("config %d: %d waves, kernel span %.1f us; start max %.1f us; end p1 %.1f p50 %.1f p99 %.1f max %.1f us; "
          "busy fraction %.3f" % (c, nw, en.max(), st.max(), *np.percentile(en, [1, 50, 99]), en.max(),
                                  dur.sum() / (nw * en.max())))
    print("   mean end by XCC: " + " ".join("%.1f" % en[xcc == k].mean() for k in range(8)))
    # spread of the end time inside a CU and inside a SIMD vs across CUs
    cus = np.unique(cu_key)
    cu_mean = np.array([en[cu_key == k].mean() for k in cus])
    cu_max = np.array([en[cu_key == k].max() for k in cus])
    within_cu = np.concatenate([en[cu_key == k] - en[cu_key == k].mean() for k in cus])
    sk = cu_key * 4 + simd
    sids = np.unique(sk)
    simd_max = np.array([en[sk == k].max() for k in sids])
    simd_mean_end = np.array([en[sk == k].mean() for k in sids])
    print("   %d CUs, %d SIMDs; CU mean end p1 %.1f p99 %.1f; CU max end p1 %.1f p50 %.1f; within-CU std %.1f; "
          "SIMD last-wave end p1 %.1f p50 %.1f; waves/SIMD %s" % (
              len(cus), len(sids), *np.percentile(cu_mean, [1, 99]), *np.percentile(cu_max, [1, 50]),
              within_cu.std(), *np.percentile(simd_max, [1, 50]),
              np.bincount(np.bincount(np.searchsorted(sids, sk)))))
    order = np.argsort(st, kind="stable")
    print("   end time vs dispatch order (deciles): " + " ".join(
        "%.1f" % en[order[i * nw // 10:(i + 1) * nw // 10]].mean() for i in range(10)))
