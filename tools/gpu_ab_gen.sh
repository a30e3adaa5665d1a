#!/bin/bash
# A/B of library variants (variants/<name>.so via PXB_LIB) on the general
# kernel's workloads: config 2 (the headline: 4 x 2^26-instance steps) and
# config 5 (2^22), two alternating rounds.   bash tools/gpu_ab_gen.sh <name>...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/abg
for round in 1 2; do
  for v in "$@"; do
    PXB_LIB=$R/variants/$v.so timeout -k 10 120 python3 -u bench.py --steps 4 --warmup 1 --no-cpu --no-extra > gpurun_out/abg/$v.c2.json 2> gpurun_out/abg/$v.c2.err || { tail -5 gpurun_out/abg/$v.c2.err; exit 1; }
    PXB_LIB=$R/variants/$v.so timeout -k 10 120 python3 -u bench.py --config 5 --instances 4194304 --steps 2 --warmup 1 --no-cpu --no-extra > gpurun_out/abg/$v.c5.json 2> gpurun_out/abg/$v.c5.err || { tail -5 gpurun_out/abg/$v.c5.err; exit 1; }
    python3 -c "
import json; a=json.load(open('gpurun_out/abg/$v.c2.json')); b=json.load(open('gpurun_out/abg/$v.c5.json'))
print('round $round %-10s config 2: %.3f G/s (%.3f ms/step)   config 5: %.2f M/s' % ('$v', a['value']/1e9, a['ms_per_step'], b['value']/1e6))"
  done
done
