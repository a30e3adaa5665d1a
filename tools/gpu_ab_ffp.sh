#!/bin/bash
# fault-free duelling / log-mode rates (tools/ffp_rates.py) of the in-tree library and variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in base "$@"; do
  if [ $v = base ]; then unset PXB_LIB; else export PXB_LIB=variants/$v.so; fi
  echo "== $v"; timeout -k 10 200 python3 -u tools/ffp_rates.py 2>&1 | grep -v amdgpu.ids || exit 1
done
