#!/bin/bash
# PMC pass (issue / wait counters) of the fault-free per-lane kernel on config 2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmcff1
cd /tmp && export TMPDIR=/tmp
CNT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $CNT -d $R/gpurun_out/pmcff1/p1 -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --config 2 --steps 2 --warmup 1 > $R/gpurun_out/pmcff1/p1.log 2>&1 || exit 1
CNT2="SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $CNT2 -d $R/gpurun_out/pmcff1/p2 -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --config 2 --steps 2 --warmup 1 > $R/gpurun_out/pmcff1/p2.log 2>&1 || exit 1
cd $R && python3 tools/pmc_summary.py gpurun_out/pmcff1/p1 paxos_ff1_kernel | cat && python3 tools/pmc_summary.py gpurun_out/pmcff1/p2 paxos_ff1_kernel | cat
