#!/bin/bash
# Config 2/6 rates of several variants, twice each in alternation (box noise).
#   bash tools/ab_c2.sh <outdir> lib1.so [lib2.so ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; shift
mkdir -p $OUT
for rep in 1 2; do
  for lib in "$@"; do
    name=$(basename $lib .so)
    PXB_RATES_CONFIGS=2,6 timeout -k 10 100 python3 -u $R/tools/cfg_rates.py $lib > $OUT/$name.$rep.txt 2>&1 || { cat $OUT/$name.$rep.txt; exit 1; }
    echo "== $name ($rep)"; grep config $OUT/$name.$rep.txt | cut -c1-60
  done
done
