#!/bin/bash
# Occupancy sensitivity of the per-lane kernel: config C at capped blocks per CU, then a PMC pass.
#   bash tools/gpu_occ.sh <config> <instances> <caps...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
C=$1; NI=$2; shift 2
mkdir -p $R/gpurun_out/occ
for cap in "$@"; do
  PXB_BLOCKS_PER_CU=$cap timeout -k 10 120 python3 -u $R/bench.py --config $C --instances $NI --steps 2 --warmup 1 --no-cpu --no-extra > $R/gpurun_out/occ/c${C}_cap$cap.json 2>/dev/null || exit 1
  python3 -c "import json; e=json.load(open('$R/gpurun_out/occ/c${C}_cap$cap.json')); print('config $C cap $cap: %.1f M/s  %.2f ms/step' % (e['value']/1e6, e['ms_per_step']))"
done
cd /tmp && export TMPDIR=/tmp
CNT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $CNT -d $R/gpurun_out/occ/pmc_c$C -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --config $C --instances $NI --steps 2 --warmup 1 > $R/gpurun_out/occ/pmc_c$C.log 2>&1 || exit 1
cd $R && python3 tools/pmc_summary.py gpurun_out/occ/pmc_c$C paxos_ev_kernel
