#!/bin/bash
# A/B of library variants (variants/<name>.so via PXB_LIB) on configs 4 and 3,
# two alternating rounds.   bash tools/gpu_ab_ev.sh <name>...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ab
for round in 1 2; do
  for v in "$@"; do
    for c in 4 3; do
      PXB_LIB=$R/variants/$v.so timeout -k 10 120 python3 -u bench.py --config $c --instances 4194304 --steps 2 --warmup 1 --no-cpu --no-extra > gpurun_out/ab/$v.c$c.json 2> gpurun_out/ab/$v.c$c.err || { tail -5 gpurun_out/ab/$v.c$c.err; exit 1; }
      python3 -c "import json; e=json.load(open('gpurun_out/ab/$v.c$c.json')); print('round $round %-12s config $c: %.2f M/s' % ('$v', e['value']/1e6))"
    done
  done
done
