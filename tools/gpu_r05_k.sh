#!/bin/bash
# GPU suite, A/B against variants/base_r05.so, then the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05k
bash tools/gpu_r05_j.sh "$@" || exit 1
cp gpurun_out/r05j/* gpurun_out/r05k/
timeout -k 10 600 python3 -u bench.py > gpurun_out/r05k/bench.json 2> gpurun_out/r05k/bench.err || { tail -20 gpurun_out/r05k/bench.err; exit 1; }
python3 -c "
import json; j=json.load(open('gpurun_out/r05k/bench.json'))
print('headline %.4g %s  ms/step %.2f  roofline frac %s' % (j['value'], j['unit'], j['ms_per_step'], j['roofline']['frac']))
for k, v in j['extra'].items():
    if 'instances_per_s' in v: print(k, '%.4g inst/s' % v['instances_per_s'], 'frac', (v.get('roofline') or {}).get('frac'))
print('cpu', j['cpu_baseline']['value'], j['cpu_baseline']['cores'])"
