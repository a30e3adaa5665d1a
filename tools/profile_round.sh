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
echo profile done
