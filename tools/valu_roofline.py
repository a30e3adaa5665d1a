"""VALU-issue roofline of the batch kernel from a rocprofv3 --pmc pass
(tools/profile_round.sh, valu/) and the kernel-trace average duration.

The batch kernel keeps the protocol state on chip, so its real limiter is
VALU issue, not HBM.  A wave64 VALU instruction occupies its SIMD's 16 lanes
for 4 cycles, so a CU issues at most one wave-instruction per cycle over its 4
SIMDs: peak = CUs x clock.  The clock is the in-kernel effective clock,
GRBM_GUI_ACTIVE / 8 XCDs / kernel time (MI355X_MICROARCH.md, DVFS give-back),
capped at 2.4 GHz.
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
    peak = CUS * clock_hz
    return {"kernel_avg_us": ns / 1e3, "effective_clock_MHz": clock_hz / 1e6,
            "valu_insts_per_launch": s["SQ_INSTS_VALU"], "valu_insts_per_instance": s["SQ_INSTS_VALU"] / instances,
            "lds_insts_per_instance": s["SQ_INSTS_LDS"] / instances,
            "salu_insts_per_instance": s["SQ_INSTS_SALU"] / instances,
            "achieved_G_wave_insts_per_s": rate / 1e9, "peak_G_wave_insts_per_s": peak / 1e9,
            "valu_issue_frac": rate / peak,
            "note": "peak = 256 CUs x effective clock x 1 wave64 VALU instruction per CU-cycle (4 SIMDs x 16 lanes, "
                    "4 cycles per wave64 instruction); PMC means per dispatch"}


if __name__ == "__main__":
    r = roofline(sys.argv[1], int(sys.argv[2]))
    print(json.dumps(r, indent=1))
    if len(sys.argv) > 3:
        json.dump(r, open(sys.argv[3], "w"), indent=1)
