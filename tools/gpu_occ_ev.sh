#!/bin/bash
# Residency sweep of the per-lane kernel: config 4 (and 3; OCC_KS, OCC_CS choose) with the launch
# capped at K blocks (= waves) per CU (PXB_BLOCKS_PER_CU).   bash tools/gpu_occ_ev.sh [lib]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/occ
LIB=${1:-$R/cloud-haskell-paxos_amd/csrc/libpaxos_batch.so}
for k in ${OCC_KS:-5 6 7 8 9}; do
  for c in ${OCC_CS:-4 3}; do
    PXB_LIB=$LIB PXB_BLOCKS_PER_CU=$k timeout -k 10 120 python3 -u bench.py --config $c --instances 4194304 --steps 2 --warmup 1 --no-cpu --no-extra > gpurun_out/occ/k$k.c$c.json 2> gpurun_out/occ/k$k.c$c.err || { tail -5 gpurun_out/occ/k$k.c$c.err; exit 1; }
    python3 -c "import json; e=json.load(open('gpurun_out/occ/k$k.c$c.json')); print('waves/CU $k config $c: %.2f M/s' % (e['value']/1e6))"
  done
done
