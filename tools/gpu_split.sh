#!/bin/bash
# Config-5 split routing check: GPU parity suite, then config 5 at 2^25 with
# the split routing and with the general kernel alone (PXB_NO_SPLIT=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/split
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/split/parity.log 2>&1 || { tail -30 gpurun_out/split/parity.log; exit 1; }
tail -1 gpurun_out/split/parity.log
for mode in split nosplit; do
  if [ $mode = nosplit ]; then export PXB_NO_SPLIT=1; fi
  timeout -k 10 200 python3 -u bench.py --config 5 --instances 33554432 --steps 1 --warmup 1 --no-cpu --no-extra > gpurun_out/split/c5_$mode.json 2> gpurun_out/split/c5_$mode.err || { cat gpurun_out/split/c5_$mode.err; exit 1; }
  python3 -c "import json; e=json.load(open('gpurun_out/split/c5_$mode.json')); print('config 5 $mode: %.2f M/s  %.1f ms/step' % (e['value']/1e6, e['ms_per_step']))"
done
unset PXB_NO_SPLIT
for c in 4 3; do
  timeout -k 10 120 python3 -u bench.py --config $c --instances 4194304 --steps 2 --warmup 1 --no-cpu --no-extra > gpurun_out/split/c$c.json 2> gpurun_out/split/c$c.err || { cat gpurun_out/split/c$c.err; exit 1; }
  python3 -c "import json; e=json.load(open('gpurun_out/split/c$c.json')); print('config $c: %.1f M/s  %.2f ms/step' % (e['value']/1e6, e['ms_per_step']))"
done
