#!/bin/bash
# Extra PMC passes of the config-4 per-lane kernel (instruction cache, issue
# classes).   bash tools/gpu_pmc_ev.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/pmcx
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-extra --config 4 --instances 4194304 --steps 2 --warmup 1"
i=0
for CNT in "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT -d $R/gpurun_out/pmcx/p$i -o pmc --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmcx/p$i.log 2>&1 || { tail -5 $R/gpurun_out/pmcx/p$i.log; exit 1; }
  (cd $R && python3 tools/pmc_summary.py gpurun_out/pmcx/p$i paxos_ev_kernel)
done
