#!/bin/bash
# bash tools/build_wt.sh [name [extra -D flags...]] -> variants/<name>.so (default v_wt): the whole
# library with -DPXB_WAVE_TIMES (per-wave timelines of the general and per-lane kernels;
# tools/ev_wave_times.py), e.g. tools/build_wt.sh v_wt20 -DPXB_EV_CMP_POOL=20
set -e
R=$(cd $(dirname $0)/.. && pwd)
NAME=${1:-v_wt}
shift || true
mkdir -p $R/variants
cd $R
python3 -c "
import subprocess, sys
sys.path.insert(0, '.')
import __graft_entry__ as g
extra = sys.argv[2:]
objs = g._hip_objects(['-DPXB_WAVE_TIMES'] + extra, '_' + sys.argv[1])
subprocess.run([g.HIPCC, *g.HIPFLAGS, '-shared', '-o', 'variants/%s.so' % sys.argv[1], *objs, '-lrccl'], check=True)
" $NAME "$@"
