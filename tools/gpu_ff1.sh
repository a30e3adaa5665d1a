#!/bin/bash
# Fault-free per-lane kernel check: GPU parity suite, then config 2 (the
# headline: 2^26 instances per step) on the per-lane kernel and on the general
# fault-free kernel (PXB_NO_FF1=1), config 1 too.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ff1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ff1/parity.log 2>&1 || { tail -30 gpurun_out/ff1/parity.log; exit 1; }
tail -1 gpurun_out/ff1/parity.log
for mode in ff1 general; do
  if [ $mode = general ]; then export PXB_NO_FF1=1; fi
  for c in 2; do
    timeout -k 10 120 python3 -u bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-extra > gpurun_out/ff1/c${c}_$mode.json 2> gpurun_out/ff1/c${c}_$mode.err || { cat gpurun_out/ff1/c${c}_$mode.err; exit 1; }
    python3 -c "import json; e=json.load(open('gpurun_out/ff1/c${c}_$mode.json')); print('config $c $mode: %.3f G/s  %.3f ms/step' % (e['value']/1e9, e['ms_per_step']))"
  done
done
