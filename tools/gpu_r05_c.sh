#!/bin/bash
# Round 5: stream-list handover tests + kernel trace of the tight routing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05c
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "failure_after_first or release_in_flight or many_streams or stream_release or run_multi or tight" > gpurun_out/r05c/pytest.log 2>&1 \
  || { tail -40 gpurun_out/r05c/pytest.log; exit 1; }
tail -3 gpurun_out/r05c/pytest.log
bash tools/gpu_r05_trace.sh
