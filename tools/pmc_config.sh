#!/bin/bash
# Instruction-mix / issue PMC pass + kernel trace for one BASELINE config.
#   bash tools/pmc_config.sh <outdir> <config> <instances> [lib.so]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; C=$2; NI=$3
[ -n "$4" ] && export PXB_LIB=$R/$4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --config $C --instances $NI --steps 2 --warmup 1 > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/valu -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --config $C --instances $NI --steps 2 --warmup 1 > $OUT/valu.log 2>&1
python3 $R/tools/valu_roofline.py $OUT $NI $OUT/valu_roofline.json
