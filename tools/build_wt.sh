#!/bin/bash
# bash tools/build_wt.sh -> variants/v_wt.so: the whole library with -DPXB_WAVE_TIMES
# (per-wave timelines of the general and per-lane kernels; tools/ev_wave_times.py)
set -e
R=$(cd $(dirname $0)/.. && pwd)
mkdir -p $R/variants
cd $R
python3 -c "
import subprocess, sys
sys.path.insert(0, '.')
import __graft_entry__ as g
objs = g._hip_objects(['-DPXB_WAVE_TIMES'], '_wt')
subprocess.run([g.HIPCC, *g.HIPFLAGS, '-shared', '-o', 'variants/v_wt.so', *objs, '-lrccl'], check=True)
"
