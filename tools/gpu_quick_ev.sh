#!/bin/bash
# Quick per-lane-kernel check: GPU parity suite, configs 4/3/5 rates, PMC of config 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q/parity.log 2>&1 || { tail -30 gpurun_out/q/parity.log; exit 1; }
tail -1 gpurun_out/q/parity.log
for c in 4 3 5; do
  timeout -k 10 120 python3 -u bench.py --config $c --instances 4194304 --steps 2 --warmup 1 --no-cpu --no-extra > gpurun_out/q/c$c.json 2> gpurun_out/q/c$c.err || { cat gpurun_out/q/c$c.err; exit 1; }
  python3 -c "import json; e=json.load(open('gpurun_out/q/c$c.json')); print('config $c: %.1f M/s  %.2f ms/step' % (e['value']/1e6, e['ms_per_step']))"
done
cd /tmp && export TMPDIR=/tmp
CNT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $CNT -d $R/gpurun_out/q/pmc4 -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --config 4 --instances 4194304 --steps 2 --warmup 1 > $R/gpurun_out/q/pmc4.log 2>&1 || exit 1
cd $R && python3 tools/pmc_summary.py gpurun_out/q/pmc4 paxos_ev_kernel | cat
