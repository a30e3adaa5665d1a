#!/bin/bash
# Per-config rates of several library variants (tools/cfg_rates.py, quick set).
#   bash tools/ab_rates.sh <outdir> lib1.so [lib2.so ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; shift
mkdir -p $OUT
for lib in "$@"; do
  name=$(basename $lib .so)
  PXB_RATES_QUICK=1 timeout -k 10 200 python3 -u $R/tools/cfg_rates.py $lib > $OUT/$name.txt 2>&1 || { cat $OUT/$name.txt; exit 1; }
  echo "== $name"; grep config $OUT/$name.txt
done
