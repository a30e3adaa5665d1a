#!/bin/bash
# A/B timing of library variants: bash tools/ab.sh out.txt lib1.so lib2.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; shift
for lib in "$@"; do
  echo "== $lib" >> $OUT
  PXB_VERBOSE=1 PXB_LIB=$R/$lib timeout -k 10 120 python3 $R/bench.py --no-cpu --steps 20 >> $OUT 2>&1 || { echo "FAILED $lib" >> $OUT; exit 1; }
done
