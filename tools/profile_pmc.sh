#!/bin/bash
# PMC passes for the dominant kernel, one rocprofv3 run per counter group
# (gfx950 slot limits: 8 SQ, 4 TCC with FETCH_SIZE=3 / WRITE_SIZE=2).
# Usage on the GPU box:  bash tools/profile_pmc.sh <outdir> [bench args...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; shift
ARGS="$@"
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra $ARGS > $OUT/$name.log 2>&1
}
run inst SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH
run cyc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT
run fetch FETCH_SIZE
run write WRITE_SIZE
echo done
