#!/bin/bash
# A/B the variant libraries given as arguments (tools/ab_ev.py), twice each, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ab
for l in "$@"; do test -f "$l" || { echo "missing $l"; exit 1; }; done
timeout -k 10 600 python3 -u tools/ab_ev.py "$@" "$@" > gpurun_out/ab/ab.txt 2>&1; rc=$?
cat gpurun_out/ab/ab.txt; exit $rc
