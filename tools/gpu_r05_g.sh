#!/bin/bash
# Round 5: halfword response links on the faulty log-mode shape (75 words, 8 waves per CU) and on
# config 5's two-proposer slim shape (75 words, 8 waves), against the round's base library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05g
L=cloud-haskell-paxos_amd/csrc/libpaxos_batch.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "log or kats or fuzz or random or config5 or split or configs_match or golden or topology" > gpurun_out/r05g/pytest.log 2>&1 || { tail -40 gpurun_out/r05g/pytest.log; exit 1; }
tail -2 gpurun_out/r05g/pytest.log
AB_CASES=7:4194304:2,7:1048576:2,5:33554432:1 timeout -k 10 400 python3 -u tools/ab_ev.py variants/base_r05.so $L variants/base_r05.so $L > gpurun_out/r05g/ab.txt 2>&1 || { cat gpurun_out/r05g/ab.txt; exit 1; }
cat gpurun_out/r05g/ab.txt
