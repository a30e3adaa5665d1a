#!/bin/bash
# Where a per-lane wave's cycles go (one PMC pass per workload): issue vs
# dependency wait vs parked, config 4 and config 5's P = 3 shape alone.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmcw
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
for w in "4 4194304" "5 4194304 nosplit"; do
  set -- $w
  tag=c$1$3
  env_ns=""; [ "$3" = nosplit ] && export PXB_NO_SPLIT=1 || unset PXB_NO_SPLIT
  timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/pmcw/$tag -o pmc --output-format csv -- python3 $R/bench.py --config $1 --instances $2 --steps 1 --warmup 1 --no-cpu --no-extra > $R/gpurun_out/pmcw/$tag.log 2>&1 || { tail -5 $R/gpurun_out/pmcw/$tag.log; exit 1; }
  f=$(find $R/gpurun_out/pmcw/$tag -name '*counter_collection.csv' | head -1)
  python3 - "$f" $tag <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "paxos_ev_kernel" in r["Kernel_Name"]:
        agg[r["Kernel_Name"].split("(")[0][-40:]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    wc = v["SQ_WAVE_CYCLES"]
    print(sys.argv[2], k, " ".join("%s %.3f" % (n[3:], v[n] / wc) for n in sorted(v) if n != "SQ_WAVE_CYCLES"))
PY
done
