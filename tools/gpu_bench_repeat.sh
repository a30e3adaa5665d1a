#!/bin/bash
# box-to-box / run-to-run spread of the headline and north-star lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/rep
for i in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --no-cpu > gpurun_out/rep/b$i.json 2> gpurun_out/rep/b$i.err || { tail -5 gpurun_out/rep/b$i.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/rep/b$i.json')); print('run $i: config 2 %.2f G/s, north star %.2f M/s, config 3 %.1f M/s, config 5 %.2f M/s, log mode %.2f G/s' % (j['value']/1e9, j['north_star']['instances_per_s']/1e6, j['extra']['config3']['instances_per_s']/1e6, j['extra']['config5']['instances_per_s']/1e6, j['extra']['log_mode']['instances_per_s']/1e9))"
done
