"""A/B timing of per-lane-kernel library variants (diagnostic; never the bench
number).  python tools/ab_ev.py lib1.so[@PXB_X=1] [lib2.so ...]
Per lib: configs 4 (2^23), 3 (2^22), 5 (2^22): kernel ms per launch (HIP
events on the launch stream) and the run totals, which must equal the first
lib's (every variant is exact)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cloud-haskell-paxos_amd"))
import torch  # noqa: E402
import pxb  # noqa: E402

CASES = [(4, 1 << 23, 1), (3, 1 << 22, 2), (5, 1 << 22, 1)]
if os.environ.get("AB_CASES"):
    CASES = [tuple(int(x) for x in c.split(":")) for c in os.environ["AB_CASES"].split(",")]


def timeit(cfg, n, reps):
    N = cfg.n_acceptors
    out = torch.empty((n, 4), dtype=torch.int32, device="cuda")
    dig = torch.empty((n, N), dtype=torch.int32, device="cuda")
    tot = torch.zeros(16, dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        pxb.run_device(cfg, 1 << 40, min(n, 1 << 20), d_results=out, d_digests=dig, d_totals=tot, stream=st.cuda_stream)
        st.synchronize()
        tot.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for k in range(reps):
            pxb.run_device(cfg, k * n, n, d_results=out, d_digests=dig, d_totals=tot, stream=st.cuda_stream)
        e1.record(st)
        st.synchronize()
    return e0.elapsed_time(e1) / reps, tot.cpu().tolist()


def main():
    ref = {}
    for arg in sys.argv[1:]:
        # lib.so[@VAR=value,VAR=value]: the variant's environment (routing switches)
        lib, _, envs = arg.partition("@")
        for k in [k for k in os.environ if k.startswith("PXB_")]:
            del os.environ[k]
        for kv in filter(None, envs.split(",")):
            k, _, v = kv.partition("=")
            os.environ[k] = v
        pxb._lib = None
        lib_h = pxb.load(os.path.join(ROOT, lib))
        if hasattr(lib_h, "pxb_reload_hooks"):       # (ABI >= 5: hooks are read once; re-read them)
            lib_h.pxb_reload_hooks()
        row = []
        for c, n, reps in CASES:
            ms, t = timeit(pxb.CONFIGS[c], n, reps)
            ok = ref.setdefault((c, n), t) == t
            row.append("c%d %8.2f ms %6.1f M/s%s" % (c, ms, n / ms / 1e3, "" if ok else " TOTALS DIFFER"))
        print("%-26s %s" % (os.path.basename(lib) + ("@" + envs if envs else ""), " | ".join(row)), flush=True)


if __name__ == "__main__":
    main()
