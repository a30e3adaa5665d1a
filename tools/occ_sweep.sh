#!/bin/bash
# throughput vs resident blocks per CU (64-thread blocks = waves per CU)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; shift
for k in "$@"; do
  echo "== blocks_per_cu=$k" >> $OUT
  PXB_BLOCKS_PER_CU=$k timeout -k 10 120 python3 $R/bench.py --no-cpu --no-extra --steps 10 >> $OUT 2>&1 || exit 1
done
