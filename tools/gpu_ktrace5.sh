#!/bin/bash
# Kernel trace of config 5 on the three-proposer shape alone (PXB_NO_SPLIT=1):
# grid, LDS, VGPRs and duration per dispatch.   bash tools/gpu_ktrace5.sh lib...
# (KT_NO_SPLIT=0: the production routing; KT_N: instances)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/kt5
cd /tmp && export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1))
  PXB_NO_SPLIT=${KT_NO_SPLIT:-1} PXB_LIB=$R/$lib timeout -s KILL 200 rocprofv3 --kernel-trace -d $R/gpurun_out/kt5/l$i -o run --output-format csv -- python3 $R/bench.py --config 5 --instances ${KT_N:-8388608} --steps 1 --warmup 1 --no-cpu --no-extra > $R/gpurun_out/kt5/l$i.log 2>&1 || { tail -5 $R/gpurun_out/kt5/l$i.log; exit 1; }
  f=$(find $R/gpurun_out/kt5/l$i -name '*kernel_trace.csv' | head -1)
  python3 - "$f" "$lib" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if "paxos" in r["Kernel_Name"]:
        keys = [k for k in r if k.lower().startswith(("grid", "workgroup", "lds", "vgpr", "sgpr", "scratch", "accum"))]
        print(sys.argv[2], r["Kernel_Name"][:60], {k: r[k] for k in keys}, "ms %.2f" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
PY
done
