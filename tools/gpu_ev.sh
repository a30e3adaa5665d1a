#!/bin/bash
# Per-lane kernel check on the GPU box: parity suite, then config-4/3/5 rates
# with the per-lane kernel and with the general kernel (PXB_NO_EV=1).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ev_parity.log 2>&1 || { tail -30 gpurun_out/ev_parity.log; exit 1; }
tail -3 gpurun_out/ev_parity.log
for c in 4 3 5; do
  timeout -k 10 120 python -u bench.py --config $c --instances 4194304 --steps 2 --warmup 1 --no-cpu --no-extra > gpurun_out/ev_c$c.json 2> gpurun_out/ev_c$c.err || { cat gpurun_out/ev_c$c.err; exit 1; }
  PXB_NO_EV=1 timeout -k 10 120 python -u bench.py --config $c --instances 4194304 --steps 2 --warmup 1 --no-cpu --no-extra > gpurun_out/gen_c$c.json 2> gpurun_out/gen_c$c.err || { cat gpurun_out/gen_c$c.err; exit 1; }
  python3 -c "import json; e=json.load(open('gpurun_out/ev_c$c.json')); g=json.load(open('gpurun_out/gen_c$c.json')); print('config $c ev %.1f M/s  general %.1f M/s  ms %.2f vs %.2f' % (e['value']/1e6, g['value']/1e6, e['ms_per_step'], g['ms_per_step']))"
done
