#!/bin/bash
# Kernel trace of north-star steps (config 4, 2^26 per step, one stream): the
# per-launch time of each kernel of the routing.  Output gpurun_out/r05t/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r05t && cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05t/trace -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu --no-extra --one-stream --config 4 --steps 2 --warmup 1 > $R/gpurun_out/r05t/bench.json \
  2> $R/gpurun_out/r05t/trace.log || { tail -5 $R/gpurun_out/r05t/trace.log; exit 1; }
head -c 300 $R/gpurun_out/r05t/bench.json; echo
find $R/gpurun_out/r05t/trace -name '*kernel_stats.csv' -exec cat {} \;
