#!/bin/bash
# bash tools/build_wire_variant.sh <name> [-D... extra hipcc flags] -> variants/<name>.so
# Rebuilds only the wire codec unit (paxos_wire.hip) with the extra flags and
# links it with the current build's other objects (A/B of wire codec changes).
set -e
R=$(cd $(dirname $0)/.. && pwd)
mkdir -p $R/variants
cd $R
python3 -c "
import os, sys, subprocess
sys.path.insert(0, '.')
import __graft_entry__ as g
g._hip_objects()
o = os.path.join(g.OBJ_DIR, 'paxos_wire_%s.o' % sys.argv[1])
subprocess.run([g.HIPCC, *g.HIPFLAGS, *sys.argv[2:], '-c', '-o', o, os.path.join(g.CSRC, 'paxos_wire.hip')], check=True)
base = [os.path.join(g.OBJ_DIR, n + '.o') for n in
        ['paxos_ev_p%d_%d' % (p, part) for p in (1, 2, 3) for part in (0, 1)] + ['paxos_trace']
        + ['paxos_inst_p%d_l%d' % (p, m) for p in (1, 2, 3) for m in (0, 1)]
        + ['paxos_ff1', 'paxos_ffp', 'paxos_batch', 'paxos_multi']]
subprocess.run([g.HIPCC, *g.HIPFLAGS, '-shared', '-o', 'variants/%s.so' % sys.argv[1], o, *base, '-lrccl'], check=True)
" "$@"
