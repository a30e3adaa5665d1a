#!/bin/bash
# Round 5: ff1 work queue (config 2, one launch of 2^28 per rep) and the
# broadcast store-back variant (config 4), A/B against the round's base library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05e
L=cloud-haskell-paxos_amd/csrc/libpaxos_batch.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "ff1 or configs_match or golden or config2 or ragged or work_queue or fault_free" > gpurun_out/r05e/pytest.log 2>&1 \
  || { tail -40 gpurun_out/r05e/pytest.log; exit 1; }
tail -2 gpurun_out/r05e/pytest.log
AB_CASES=2:268435456:5 timeout -k 10 300 python3 -u tools/ab_ev.py variants/base_r05.so $L variants/base_r05.so $L > gpurun_out/r05e/ab2.txt 2>&1 || { cat gpurun_out/r05e/ab2.txt; exit 1; }
cat gpurun_out/r05e/ab2.txt
AB_CASES=4:16777216:2,4:67108864:1 timeout -k 10 400 python3 -u tools/ab_ev.py variants/base_r05.so variants/sb1.so variants/base_r05.so variants/sb1.so > gpurun_out/r05e/ab4.txt 2>&1 || { cat gpurun_out/r05e/ab4.txt; exit 1; }
cat gpurun_out/r05e/ab4.txt
