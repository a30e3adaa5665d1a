#!/bin/bash
# bash tools/build_variant.sh <name> [-D... extra hipcc flags]  -> variants/<name>.so
set -e
R=$(cd $(dirname $0)/.. && pwd)
mkdir -p $R/variants
cd $R
python3 -c "
import sys, subprocess
sys.path.insert(0, '.')
import __graft_entry__ as g
objs = g._hip_objects(tuple(sys.argv[2:]), tag='_' + sys.argv[1])
subprocess.run([g.HIPCC, *g.HIPFLAGS, '-shared', '-o', 'variants/%s.so' % sys.argv[1], *objs, '-lrccl'], check=True)
" "$@"
