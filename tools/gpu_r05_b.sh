#!/bin/bash
# Round 5: tight routing (layout 7, 50 words) -- parity subset, A/B against
# layout 6 alone, and the first launch's wave placement (residency check).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05b
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "tight or contiguous or configs_match or golden or north_star or bail_list or topology_sweep" > gpurun_out/r05b/pytest.log 2>&1 \
  || { tail -40 gpurun_out/r05b/pytest.log; exit 1; }
tail -3 gpurun_out/r05b/pytest.log
L=cloud-haskell-paxos_amd/csrc/libpaxos_batch.so
AB_CASES=4:16777216:2,4:67108864:1 timeout -k 10 300 python3 -u tools/ab_ev.py $L $L@PXB_NO_TIGHT=1 $L $L@PXB_NO_TIGHT=1 \
  > gpurun_out/r05b/ab.txt 2>&1 || { cat gpurun_out/r05b/ab.txt; exit 1; }
cat gpurun_out/r05b/ab.txt
timeout -k 10 120 python3 -u tools/ev_wave_times.py variants/v_wt.so 4 8388608 > gpurun_out/r05b/wt_tight.txt 2>&1 || { cat gpurun_out/r05b/wt_tight.txt; exit 1; }
cat gpurun_out/r05b/wt_tight.txt
