#!/bin/bash
# Round 5 A/B of per-lane variants against the current library (tools/ab_ev.py),
# two passes: bash tools/gpu_r05_ab.sh variants/x.so ...   (AB_CASES as in ab_ev.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05ab
L=cloud-haskell-paxos_amd/csrc/libpaxos_batch.so
ARGS=(); for p in 1 2; do ARGS+=($L "$@"); done
AB_CASES=${AB_CASES:-4:16777216:2,4:67108864:1} timeout -k 10 500 python3 -u tools/ab_ev.py "${ARGS[@]}" > gpurun_out/r05ab/ab.txt 2>&1 || { cat gpurun_out/r05ab/ab.txt; exit 1; }
cat gpurun_out/r05ab/ab.txt
