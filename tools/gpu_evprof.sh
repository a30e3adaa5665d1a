#!/bin/bash
# PMC instruction mix of the per-lane (EV) kernel vs the general kernel on one config.
#   bash tools/gpu_evprof.sh <config> <instances>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
C=${1:-4}; NI=${2:-4194304}
OUT=$R/gpurun_out/evprof_c$C
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CNT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/ev_trace -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --config $C --instances $NI --steps 2 --warmup 1 > $OUT/ev_trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $CNT -d $OUT/ev_valu -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --config $C --instances $NI --steps 2 --warmup 1 > $OUT/ev_valu.log 2>&1 || exit 1
PXB_NO_EV=1 timeout -s KILL 120 rocprofv3 --pmc $CNT -d $OUT/gen_valu -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --config $C --instances $NI --steps 2 --warmup 1 > $OUT/gen_valu.log 2>&1 || exit 1
cd $R
echo "== ev kernel"; python3 tools/pmc_summary.py $OUT/ev_valu paxos_ev_kernel
echo "== general kernel behind ev (bailed ids)"; python3 tools/pmc_summary.py $OUT/ev_valu paxos_batch_kernel
echo "== general kernel alone"; python3 tools/pmc_summary.py $OUT/gen_valu paxos_batch_kernel
grep -h "paxos" $OUT/ev_trace/*/*kernel_stats.csv 2>/dev/null | cut -c1-200 || find $OUT/ev_trace -name "*stats*"
