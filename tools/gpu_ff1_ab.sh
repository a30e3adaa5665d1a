#!/bin/bash
# ff1 A/B: parity subset and config-2 rate of the in-tree library, then the
# config-2 rate of each variants/<name>.so given
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && bash tools/gpu_ff1q.sh || exit 1
for v in "$@"; do
  PXB_LIB=variants/$v.so timeout -k 10 120 python3 -u bench.py --config 2 --steps 10 --warmup 2 --no-cpu --no-extra > gpurun_out/ff1q/c2_$v.json 2> gpurun_out/ff1q/c2_$v.err || { cat gpurun_out/ff1q/c2_$v.err; exit 1; }
  python3 -c "import json; e=json.load(open('gpurun_out/ff1q/c2_$v.json')); print('variant $v config 2: %.3f G/s  %.3f ms/step' % (e['value']/1e9, e['ms_per_step']))"
done
