#!/bin/bash
# One PMC pass (instruction mix) per library: bash tools/pmc_inst.sh outdir lib...
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  name=$(basename $lib .so)
  PXB_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d $OUT/$name -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --steps 4 --warmup 1 > $OUT/$name.log 2>&1 || exit 1
done
