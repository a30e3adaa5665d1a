#!/bin/bash
# config 5 (2^24) and config 4 (2^24) rates of the in-tree library and of each variants/<name>.so
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/abc5
for v in base "$@"; do
  for c in 5 4; do
    if [ $v = base ]; then unset PXB_LIB; else export PXB_LIB=variants/$v.so; fi
    timeout -k 10 200 python3 -u bench.py --config $c --instances 16777216 --steps 1 --warmup 1 --no-cpu --no-extra > gpurun_out/abc5/$v.c$c.json 2> gpurun_out/abc5/$v.c$c.err || { cat gpurun_out/abc5/$v.c$c.err; exit 1; }
    python3 -c "import json; e=json.load(open('gpurun_out/abc5/$v.c$c.json')); print('$v config $c: %.2f M inst/s' % (e['counters']['instances']/e['ms_per_step']/1e3))"
  done
done
