#!/bin/bash
# Kernel trace of one bench workload (per-launch start / end / queue: which
# kernel holds a step's tail).  Runs on the GPU box:
#   bash tools/gpu_ktrace.sh <outdir> <bench.py args...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/bench.py --no-cpu "$@" > $OUT/bench.json 2> $OUT/trace.log || { tail -5 $OUT/trace.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
t0 = min(int(r["Start_Timestamp"]) for r in rows)
for r in rows:
    n = r["Kernel_Name"]
    if "paxos" in n or "finalize" in n:
        s = (int(r["Start_Timestamp"]) - t0) / 1e6
        e = (int(r["End_Timestamp"]) - t0) / 1e6
        print("%-52s q%s %9.3f %9.3f %8.3f" % (n.split("(")[0].replace("void ", "")[-52:], r["Queue_Id"], s, e, e - s))
PY
