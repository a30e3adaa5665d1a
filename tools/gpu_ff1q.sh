#!/bin/bash
# quick config-2 rate of the fault-free per-lane kernel (+ its parity tests)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ff1q
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "ff1 or configs_match or golden or fault_free or ragged" > gpurun_out/ff1q/parity.log 2>&1 || { tail -30 gpurun_out/ff1q/parity.log; exit 1; }
tail -1 gpurun_out/ff1q/parity.log
timeout -k 10 120 python3 -u bench.py --config 2 --steps 10 --warmup 2 --no-cpu --no-extra > gpurun_out/ff1q/c2.json 2> gpurun_out/ff1q/c2.err || { cat gpurun_out/ff1q/c2.err; exit 1; }
python3 -c "import json; e=json.load(open('gpurun_out/ff1q/c2.json')); print('config 2: %.3f G/s  %.3f ms/step' % (e['value']/1e9, e['ms_per_step']))"
