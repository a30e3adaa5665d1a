#!/bin/bash
# Fault-free per-lane kernels: GPU parity subset (fault-free, log mode, goldens,
# ff1), then the log-mode workload and a duelling fault-free batch on the
# per-lane kernel and on the general kernel (PXB_NO_FFP=1)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ffp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "ff1 or ffp or log_mode or golden or fault_free or ragged or configs_match" > gpurun_out/ffp/parity.log 2>&1 || { tail -30 gpurun_out/ffp/parity.log; exit 1; }
tail -1 gpurun_out/ffp/parity.log
timeout -k 10 200 python3 -u tools/ffp_rates.py > gpurun_out/ffp/rates.txt 2>&1 || { cat gpurun_out/ffp/rates.txt; exit 1; }
cat gpurun_out/ffp/rates.txt
