"""A/B timing of library variants (diagnostic; never the bench number).
    python tools/exp.py lib1.so [lib2.so ...]
For each lib: kernel ms per launch (HIP events on the launch stream) for
config 2 (2^20, with and without outputs), configs 3 and 4 (2^22) config 5 (2^20) and config 6 (log mode, 2^20)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cloud-haskell-paxos_amd"))
import torch  # noqa: E402
import pxb  # noqa: E402


def timeit(cfg, n, outputs, reps, first0):
    N = cfg.n_acceptors
    out = torch.empty((n, 4), dtype=torch.int32, device="cuda") if outputs else None
    dig = torch.empty((n, N), dtype=torch.int32, device="cuda") if outputs else None
    tot = torch.zeros(16, dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        pxb.run_device(cfg, first0, n, d_results=out, d_digests=dig, d_totals=tot, stream=st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for k in range(reps):
            pxb.run_device(cfg, first0 + (k + 1) * n, n, d_results=out, d_digests=dig, d_totals=tot,
                           stream=st.cuda_stream)
        e1.record(st)
        st.synchronize()
    return e0.elapsed_time(e1) / reps, tot.cpu().tolist()


def main():
    for lib in sys.argv[1:]:
        pxb._lib = None
        pxb.load(os.path.join(ROOT, lib))
        row = []
        ms, t = timeit(pxb.CONFIGS[2], 1 << 20, True, 20, 0)
        row.append("c2 %.4f ms (%.2f Ginst/s)" % (ms, (1 << 20) / ms / 1e6))
        ms, t = timeit(pxb.CONFIGS[2], 1 << 20, False, 20, 0)
        row.append("c2-noout %.4f" % ms)
        ms, t = timeit(pxb.CONFIGS[3], 1 << 22, True, 3, 0)
        row.append("c3 %.2f ms (%.1f Minst/s, %.1f ps/inst-step, %.1f ps/msg)" % (
            ms, (1 << 22) / ms / 1e3, ms * 1e9 * 4 / t[12], ms * 1e9 * 4 / t[7]))
        ms, t = timeit(pxb.CONFIGS[4], 1 << 22, True, 2, 0)
        row.append("c4 %.2f ms (%.1f Minst/s, %.1f ps/inst-step, %.1f ps/msg)" % (
            ms, (1 << 22) / ms / 1e3, ms * 1e9 * 3 / t[12], ms * 1e9 * 3 / t[7]))
        ms, t = timeit(pxb.CONFIGS[5], 1 << 20, True, 2, 0)
        row.append("c5 %.2f ms (%.1f Minst/s, %.1f ps/inst-step, %.1f ps/msg)" % (
            ms, (1 << 20) / ms / 1e3, ms * 1e9 * 3 / t[12], ms * 1e9 * 3 / t[7]))
        ms, t = timeit(pxb.CONFIGS[6], 1 << 20, True, 5, 0)
        row.append("c6 %.3f ms (%.1f Minst/s)" % (ms, (1 << 20) / ms / 1e3))
        print("%-28s %s" % (lib, " | ".join(row)), flush=True)


if __name__ == "__main__":
    main()
