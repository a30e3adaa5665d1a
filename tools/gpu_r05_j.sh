#!/bin/bash
# Round 5 (second session): GPU suite on the current library, then A/B against
# variants/base_r05.so (the session's starting commit), two passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05j
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05j/parity.log 2>&1 || { tail -40 gpurun_out/r05j/parity.log; exit 1; }
tail -2 gpurun_out/r05j/parity.log
L=cloud-haskell-paxos_amd/csrc/libpaxos_batch.so
ARGS=(); for p in 1 2; do ARGS+=(variants/base_r05.so $L "$@"); done
AB_CASES=${AB_CASES:-4:16777216:2,4:67108864:1,3:16777216:2,5:8388608:1} timeout -k 10 500 python3 -u tools/ab_ev.py "${ARGS[@]}" > gpurun_out/r05j/ab.txt 2>&1 || { cat gpurun_out/r05j/ab.txt; exit 1; }
cat gpurun_out/r05j/ab.txt
