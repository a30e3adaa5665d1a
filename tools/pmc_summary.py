"""Summarise rocprofv3 --pmc CSV output per kernel: mean per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root, kernel_sub="paxos_batch_kernel"):
    agg = defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_sub not in row.get("Kernel_Name", ""):
                    continue
                agg[(row["Counter_Name"], row["Dispatch_Id"])].append(float(row["Counter_Value"]))
    per = defaultdict(list)
    for (name, disp), vals in agg.items():
        per[name].append(sum(vals))
    out = {k: sum(v) / len(v) for k, v in sorted(per.items())}
    for k, v in out.items():
        print("%-28s %16.1f" % (k, v))
    return out


if __name__ == "__main__":
    main(*sys.argv[1:])
