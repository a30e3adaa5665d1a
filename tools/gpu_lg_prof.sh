#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06b; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt20 -o run --output-format csv -- python3 $R/bench.py --config 7 --instances 1048576 --steps 10 --warmup 1 --no-cpu --no-extra > $O/kt20.log 2>&1 || { tail -5 $O/kt20.log; exit 1; }
echo kt20 done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt22 -o run --output-format csv -- python3 $R/bench.py --config 7 --instances 4194304 --steps 3 --warmup 1 --no-cpu --no-extra > $O/kt22.log 2>&1 || { tail -5 $O/kt22.log; exit 1; }
echo kt22 done
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
timeout -s KILL 120 rocprofv3 --pmc $C -d $O/pmc7 -o pmc --output-format csv -- python3 $R/bench.py --config 7 --instances 4194304 --steps 1 --warmup 1 --no-cpu --no-extra --one-stream > $O/pmc7.log 2>&1 || { tail -5 $O/pmc7.log; exit 1; }
echo pmc done
