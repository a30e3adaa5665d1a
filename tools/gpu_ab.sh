#!/bin/bash
# A/B of per-lane-kernel library variants (tools/ab_ev.py), two passes:
#   bash tools/gpu_ab.sh lib1.so lib2.so ...   (AB_CASES as in ab_ev.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ab
for l in "$@"; do test -f "$l" || { echo "missing $l"; exit 1; }; done
# AB_PASSES passes over the libs, interleaved (default 2)
LIBS=(); for p in $(seq ${AB_PASSES:-2}); do LIBS+=("$@"); done
AB_CASES=${AB_CASES:-4:8388608:1,3:4194304:2} timeout -k 10 600 python3 -u tools/ab_ev.py "${LIBS[@]}" > gpurun_out/ab/ab.txt 2>&1 || { cat gpurun_out/ab/ab.txt; exit 1; }
cat gpurun_out/ab/ab.txt
