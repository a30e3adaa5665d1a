#!/bin/bash
# GPU suite on the current build, then an A/B of the given variants against it
# (AB_CASES, two passes).   bash tools/gpu_r03_c.sh [lib ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r3c
for l in "$@"; do test -f "$l" || { echo "missing $l"; exit 1; }; done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3c/parity.log 2>&1 || { tail -40 gpurun_out/r3c/parity.log; exit 1; }
tail -1 gpurun_out/r3c/parity.log
if [ $# -gt 0 ]; then
  AB_CASES=${AB_CASES:-5:33554432:1,4:8388608:1} timeout -k 10 500 python3 -u tools/ab_ev.py "$@" cloud-haskell-paxos_amd/csrc/libpaxos_batch.so "$@" cloud-haskell-paxos_amd/csrc/libpaxos_batch.so > gpurun_out/r3c/ab.txt 2>&1 || { cat gpurun_out/r3c/ab.txt; exit 1; }
  cat gpurun_out/r3c/ab.txt
fi
