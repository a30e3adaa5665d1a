#!/bin/bash
# Wire codec kernel trace (tools/wire_prof.py) -> gpurun_out/wirep
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/wirep
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wirep/trace -o run --output-format csv -- python3 $R/tools/wire_prof.py > $R/gpurun_out/wirep/run.log 2>&1 || { tail -5 $R/gpurun_out/wirep/run.log; exit 1; }
tail -2 $R/gpurun_out/wirep/run.log
cat $(find $R/gpurun_out/wirep/trace -name '*kernel_stats.csv' | head -1) | cut -d, -f1-8
