#!/bin/bash
# Round profile set for the bench workload: kernel-trace stats + FETCH/WRITE passes.
#   bash tools/profile_round.sh <outdir> [bench args]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-extra "$@" > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --steps 4 --warmup 1 "$@" > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --steps 4 --warmup 1 "$@" > $OUT/write.log 2>&1
# instruction mix / issue (8 SQ counters + 1 GRBM: one pass)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/valu -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --steps 4 --warmup 1 "$@" > $OUT/valu.log 2>&1
echo profile done
