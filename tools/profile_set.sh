#!/bin/bash
# Profile set of one bench workload (rounds 2, 3): kernel-trace stats, one SQ/GRBM
# PMC pass, FETCH_SIZE and WRITE_SIZE passes (each its own run, per the
# MI355X guide), then tools/roofline.py -> <outdir>/step.json (what bench.py
# reads for its roofline).  Runs on the GPU box:
#   bash tools/profile_set.sh <outdir> <config> <instances/step> <steps> <warmup>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; C=$2; NI=$3; S=$4; W=$5
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# (--one-stream: with bench.py's two step streams a launch queued behind another is
# dispatched early and rocprof's duration for it includes the wait for CUs)
ARGS="--no-cpu --no-extra --one-stream --config $C --instances $NI --steps $S --warmup $W"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench.json 2> $OUT/trace.log || { tail -5 $OUT/trace.log; exit 1; }
echo "trace done"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $OUT/valu -o pmc --output-format csv -- python3 $R/bench.py $ARGS > $OUT/valu.log 2>&1 || { tail -5 $OUT/valu.log; exit 1; }
echo "valu done"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o pmc --output-format csv -- python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1 || { tail -5 $OUT/fetch.log; exit 1; }
echo "fetch done"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o pmc --output-format csv -- python3 $R/bench.py $ARGS > $OUT/write.log 2>&1 || { tail -5 $OUT/write.log; exit 1; }
echo "write done"
cd $R && python3 tools/roofline.py $OUT "BASELINE config $C" $(( NI * (S + W) )) $OUT/step.json > /dev/null && echo "step.json written"
