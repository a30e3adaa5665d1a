#!/bin/bash
# Round-3 first probe: integer multiply issue costs, VALU peak, baseline
# per-lane-kernel rates (configs 4 at 2^22/2^23, 3, 5) on the current build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/p3
timeout -k 10 120 tools/micro/mul_rate > gpurun_out/p3/mul_rate.txt 2>&1 || exit 1
timeout -k 10 120 tools/micro/valu_peak > gpurun_out/p3/valu_peak.txt 2>&1 || exit 1
PXB_RATES_CONFIGS=4,3,5 PXB_RATES_QUICK=1 timeout -k 10 300 python3 -u tools/cfg_rates.py > gpurun_out/p3/rates.txt 2>&1 || exit 1
cat gpurun_out/p3/*.txt
