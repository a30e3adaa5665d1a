#!/bin/bash
# Kernel trace of one config-5 step (2^25 instances) -> gpurun_out/kt5/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/kt5
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt5/trace -o run --output-format csv -- python3 $R/bench.py --config 5 --instances 33554432 --steps 1 --warmup 1 --no-cpu --no-extra > $R/gpurun_out/kt5/bench.json 2> $R/gpurun_out/kt5/trace.log || { tail -5 $R/gpurun_out/kt5/trace.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/kt5/trace/**/*kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows:
    n = r['Kernel_Name']
    if 'paxos' in n or 'finalize' in n:
        print('%-60s %10.2f ms  grid %s' % (n[:60], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6, r.get('Grid_Size', r.get('Grid_Size_X', '?'))))
PY
