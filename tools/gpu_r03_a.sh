#!/bin/bash
# GPU suite on the current build, then A/B of pool sizes and of residency caps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r3a
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a/parity.log 2>&1 || { tail -40 gpurun_out/r3a/parity.log; exit 1; }
tail -2 gpurun_out/r3a/parity.log
timeout -k 10 300 python3 -u tools/ab_ev.py variants/L3.so variants/L3p22.so variants/L3.so variants/L3p22.so > gpurun_out/r3a/ab.txt 2>&1 || { cat gpurun_out/r3a/ab.txt; exit 1; }
cat gpurun_out/r3a/ab.txt
for b in 9 8; do
  PXB_BLOCKS_PER_CU=$b AB_CASES=4:8388608:1 timeout -k 10 120 python3 -u tools/ab_ev.py variants/L3.so > gpurun_out/r3a/cap$b.txt 2>&1 || exit 1
  echo "blocks/CU cap $b: $(tail -1 gpurun_out/r3a/cap$b.txt)"
done
