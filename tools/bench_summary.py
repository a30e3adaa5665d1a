#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (tools/gpu_lease.sh).

    python3 tools/bench_summary.py gpurun_out/<tag>/bench_<k>.json
"""
import json
import sys


def main(path):
    j = json.load(open(path))
    r = j.get("roofline") or {}
    print("headline %.4g %s  ms/step %.2f  kernel ms/step %.2f  VALU frac %s" % (
        j["value"], j["unit"], j["ms_per_step"], j.get("kernel_ms_per_step", 0.0), r.get("frac")))
    for k, v in j.get("extra", {}).items():
        if "instances_per_s" in v:
            fr = (v.get("roofline") or {}).get("frac")
            sp = v.get("speedup_vs_general_kernel")
            print("  %-22s %.4g inst/s  frac %s%s" % (k, v["instances_per_s"], fr,
                                                      "  x%.2f vs general" % sp if sp else ""))
    cb = j.get("cpu_baseline")
    if cb:
        print("  cpu baseline %.4g %s on %s cores (%s)" % (cb["value"], cb["unit"], cb["cores"], cb["kind"]))


if __name__ == "__main__":
    main(sys.argv[1])
