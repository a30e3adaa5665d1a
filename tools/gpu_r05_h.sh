#!/bin/bash
# Round 5: fault-free per-lane kernel (config 2): one 2^28 launch per rep, grid of k x the
# resident blocks (PXB_FF1_OVERSUB), against the round's base library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05h
L=cloud-haskell-paxos_amd/csrc/libpaxos_batch.so
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "ff1 or configs_match or config2 or ragged or work_queue or fault_free" > gpurun_out/r05h/pytest.log 2>&1 \
  || { tail -40 gpurun_out/r05h/pytest.log; exit 1; }
tail -2 gpurun_out/r05h/pytest.log
AB_CASES=2:268435456:5 timeout -k 10 300 python3 -u tools/ab_ev.py variants/base_r05.so $L $L@PXB_FF1_OVERSUB=2 $L@PXB_FF1_OVERSUB=4 $L@PXB_FF1_OVERSUB=8 $L@PXB_FF1_OVERSUB=16 \
  variants/base_r05.so $L $L@PXB_FF1_OVERSUB=2 $L@PXB_FF1_OVERSUB=4 $L@PXB_FF1_OVERSUB=8 $L@PXB_FF1_OVERSUB=16 > gpurun_out/r05h/ab.txt 2>&1 || { cat gpurun_out/r05h/ab.txt; exit 1; }
cat gpurun_out/r05h/ab.txt
