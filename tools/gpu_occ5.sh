#!/bin/bash
# Residency sweep of config 5 on the three-proposer per-lane shape alone
# (PXB_NO_SPLIT=1), K blocks (= waves) per CU.   bash tools/gpu_occ5.sh lib...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/occ5
for lib in "$@"; do
  for k in ${OCC_KS:-3 4 5 0}; do
    PXB_NO_SPLIT=1 PXB_LIB=$R/$lib PXB_BLOCKS_PER_CU=$k timeout -k 10 120 python3 -u bench.py --config 5 --instances 8388608 --steps 1 --warmup 1 --no-cpu --no-extra > gpurun_out/occ5/k$k.json 2> gpurun_out/occ5/k$k.err || { tail -5 gpurun_out/occ5/k$k.err; exit 1; }
    python3 -c "import json; e=json.load(open('gpurun_out/occ5/k$k.json')); print('$lib waves/CU cap $k: %.2f M/s' % (e['value']/1e6))"
  done
done
