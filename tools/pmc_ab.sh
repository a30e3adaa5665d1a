#!/bin/bash
# Instruction-mix PMC pass per library variant (config 2 bench workload).
#   bash tools/pmc_ab.sh <outdir> lib1.so [lib2.so ...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  name=$(basename $lib .so)
  PXB_LIB=$R/$lib timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d $OUT/$name -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --steps 4 --warmup 1 $BENCH_ARGS > $OUT/$name.log 2>&1 || exit 1
  PXB_LIB=$R/$lib timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES -d $OUT/${name}_b -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --steps 4 --warmup 1 $BENCH_ARGS > $OUT/${name}_b.log 2>&1 || exit 1
  echo "== $name"; python3 $R/tools/pmc_summary.py $OUT/$name; python3 $R/tools/pmc_summary.py $OUT/${name}_b
done
