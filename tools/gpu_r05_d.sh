#!/bin/bash
# Round 5: tight routing A/B against layout 6 alone + a config-4 parity subset.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05d
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "tight or contiguous or configs_match or golden or north_star or topology_sweep" > gpurun_out/r05d/pytest.log 2>&1 \
  || { tail -40 gpurun_out/r05d/pytest.log; exit 1; }
tail -2 gpurun_out/r05d/pytest.log
L=cloud-haskell-paxos_amd/csrc/libpaxos_batch.so
AB_CASES=${AB_CASES:-4:16777216:2,4:67108864:1} timeout -k 10 300 python3 -u tools/ab_ev.py $L $L@PXB_NO_TIGHT=1 $L $L@PXB_NO_TIGHT=1 \
  > gpurun_out/r05d/ab.txt 2>&1 || { cat gpurun_out/r05d/ab.txt; exit 1; }
cat gpurun_out/r05d/ab.txt
