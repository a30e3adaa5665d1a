"""VALU-issue roofline of the batch kernel from a rocprofv3 --pmc pass
(a round-1 profile directory, valu/ pass) and the kernel-trace average duration.

The batch kernel keeps the protocol state on chip, so its real limiter is
VALU issue, not HBM.  A wave64 VALU instruction issues in 2 cycles on a
SIMD-32, 4 SIMDs per CU: the peak is 2 wave-instructions per CU-cycle
(MI355X_MICROARCH.md, "Wave scheduling").  (Round 1 used 1 per CU-cycle, half
the peak, and reported fractions above 1; corrected in round 2.)  The clock is
the in-kernel effective clock, GRBM_GUI_ACTIVE / 8 XCDs / kernel time
(MI355X_MICROARCH.md, DVFS give-back), capped at 2.4 GHz.  tools/roofline.py
is the round-2 tool (whole bench workloads, HBM passes included).
    python tools/valu_roofline.py <prof dir> <instances per launch> [out.json]"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import main as summary  # noqa: E402

CUS = 256


def kernel_avg_ns(root, kernel_sub="paxos_batch_kernel"):
    for f in glob.glob(os.path.join(root, "trace", "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_sub in row["Name"]:
                    return float(row["AverageNs"])
    return None


def roofline(root, instances):
    s = summary(os.path.join(root, "valu"))
    ns = kernel_avg_ns(root)
    # the quotient reads high on dispatches shorter than ~0.3 ms: cap it at
    # the MI355X peak engine clock (2.4 GHz)
    clock_hz = min(s["GRBM_GUI_ACTIVE"] / 8.0 / (ns * 1e-9), 2.4e9)
    rate = s["SQ_INSTS_VALU"] / (ns * 1e-9)               # wave-instructions / s
    peak = CUS * 2.0 * clock_hz                           # 2 wave64 VALU instructions per CU-cycle
    # measured ceiling: tools/micro/valu_peak.hip (independent add/xor chains,
    # 8 waves/SIMD) issues ~1.4 wave-instructions per CU-cycle on gfx950
    emp = None
    pf = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r01_valu_peak.jsonl")
    if os.path.exists(pf):
        rows = [json.loads(line) for line in open(pf) if line.strip()]
        emp = max(r["G_wave_valu_insts_per_s"] for r in rows if r["kernel"] == "add/xor chains") * 1e9
    return {"kernel_avg_us": ns / 1e3, "effective_clock_MHz": clock_hz / 1e6,
            "valu_insts_per_launch": s["SQ_INSTS_VALU"], "valu_insts_per_instance": s["SQ_INSTS_VALU"] / instances,
            "lds_insts_per_instance": s["SQ_INSTS_LDS"] / instances,
            "salu_insts_per_instance": s["SQ_INSTS_SALU"] / instances,
            "achieved_G_wave_insts_per_s": rate / 1e9, "peak_G_wave_insts_per_s": peak / 1e9,
            "valu_frac": rate / peak,
            "microbench_G_wave_insts_per_s": None if emp is None else emp / 1e9,
            "note": "peak = 2 wave64 VALU instructions per CU-cycle (SIMD-32, 2 cycles per wave64 "
                    "instruction, 4 SIMDs); the dependent-chain microbenchmark (tools/micro/valu_peak.hip, "
                    "1.43 per CU-cycle) is not a ceiling; PMC means per dispatch"}


if __name__ == "__main__":
    r = roofline(sys.argv[1], int(sys.argv[2]))
    print(json.dumps(r, indent=1))
    if len(sys.argv) > 3:
        json.dump(r, open(sys.argv[3], "w"), indent=1)
