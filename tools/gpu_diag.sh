#!/bin/bash
# Diagnostics: section stamps + instruction-mix PMC pass + cycle PMC pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-diag}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 200 python3 tools/stamps.py > $O/stamps.log 2>&1 || { echo stamps failed; tail $O/stamps.log; exit 1; }
cat $O/stamps.log
timeout -k 10 300 bash tools/profile_pmc.sh gpurun_out/$TAG/pmc || { echo pmc failed; exit 1; }
for d in inst cyc lds; do echo "== $d"; python3 tools/pmc_summary.py $O/pmc/$d; done
