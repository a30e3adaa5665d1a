#!/bin/bash
# Kernel-trace stats of one bench config (per-kernel average durations).
#   bash tools/gpu_ktrace.sh <tag> <config> <instances> [env...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; C=$2; NI=$3; shift 3
OUT=$R/gpurun_out/kt_$T
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
env "$@" timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --config $C --instances $NI --steps 2 --warmup 1 > $OUT/bench.json 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, json, sys
d = sys.argv[1]
for f in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("%-60s calls %4s avg %10.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
b = [l for l in open(d + "/bench.json") if l.startswith("{")]
if b:
    j = json.loads(b[-1]); print("value %.2f M/s, ms/step %.2f" % (j["value"] / 1e6, j["ms_per_step"]))
PY
