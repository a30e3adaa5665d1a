#!/bin/bash
# Round 5: oversubscribed grids for the fault-free per-lane kernels (ff1 config 2, ffp config 6).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05i
L=cloud-haskell-paxos_amd/csrc/libpaxos_batch.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "oversubscription or ff1 or ffp or configs_match or config2 or ragged or work_queue or fault_free or log_mode or golden" > gpurun_out/r05i/pytest.log 2>&1 \
  || { tail -40 gpurun_out/r05i/pytest.log; exit 1; }
tail -2 gpurun_out/r05i/pytest.log
AB_CASES=2:268435456:5,6:4194304:3,6:1048576:3 timeout -k 10 300 python3 -u tools/ab_ev.py variants/base_r05.so $L $L@PXB_FF1_OVERSUB=32,PXB_FFP_OVERSUB=32 $L@PXB_FFP_OVERSUB=4 \
  variants/base_r05.so $L $L@PXB_FF1_OVERSUB=32,PXB_FFP_OVERSUB=32 $L@PXB_FFP_OVERSUB=4 > gpurun_out/r05i/ab.txt 2>&1 || { cat gpurun_out/r05i/ab.txt; exit 1; }
cat gpurun_out/r05i/ab.txt
