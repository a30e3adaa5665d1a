#!/bin/bash
# bash tools/build_ev_variant.sh <name> [-D... extra hipcc flags] -> variants/<name>.so
# Rebuilds only the per-lane kernel units (paxos_ev_p1..3 parts 0/1, trace) with the
# extra flags and links them with the current build's other objects: A/B of
# paxos_ev.h changes in a minute instead of a full library build.  EVP1 / EVP2
# / EVP3 (or EVP2_1 etc.: one part) in the environment set one unit's scheduler flags;
# EV_FLAGS_OVERRIDE replaces __graft_entry__.EV_FLAGS for the variant.
set -e
R=$(cd $(dirname $0)/.. && pwd)
mkdir -p $R/variants
cd $R
python3 -c "
import os, sys, subprocess
sys.path.insert(0, '.')
import __graft_entry__ as g
g._hip_objects()                       # the base objects, up to date
tag = '_' + sys.argv[1]
extra = sys.argv[2:]
if os.environ.get('EV_FLAGS_OVERRIDE') is not None:   # replace the per-lane units' LLVM flags
    g.EV_FLAGS = os.environ['EV_FLAGS_OVERRIDE'].split()
procs, objs = [], []
for p in (1, 2, 3):
  for part in (0, 1):
    o = os.path.join(g.OBJ_DIR, 'paxos_ev_p%d_%d%s.o' % (p, part, tag))
    # EVP<p>: flags for that proposer count's units; EVP<p>_<part>: for one unit
    # (part 0: wide / compact / simple-schedule shapes, 1: log-mode and slim);
    # without either, the build's own per-unit flags (__graft_entry__.ev_unit_flags)
    own = g.ev_unit_flags(p, part)
    unit = (os.environ.get('EVP%d_%d' % (p, part)) or os.environ.get('EVP%d' % p) or ' '.join(own)).split()
    procs.append(subprocess.Popen([g.HIPCC, *g.HIPFLAGS, *extra, *g.EV_FLAGS, *unit, '-DPXB_EV_P=%d' % p,
                                   '-DPXB_EV_PART=%d' % part, '-c', '-o', o, os.path.join(g.CSRC, 'paxos_ev.hip')]))
    objs.append(o)
o = os.path.join(g.OBJ_DIR, 'paxos_trace%s.o' % tag)
procs.append(subprocess.Popen([g.HIPCC, *g.HIPFLAGS, *extra, *g.EV_FLAGS, '-c', '-o', o, os.path.join(g.CSRC, 'paxos_trace.hip')]))
objs.append(o)
for pr in procs:
    if pr.wait():
        raise SystemExit('hipcc failed')
base = [os.path.join(g.OBJ_DIR, n + '.o') for n in ['paxos_inst_p%d_l%d' % (p, m) for p in (1, 2, 3) for m in (0, 1)]
        + ['paxos_ff1', 'paxos_ffp', 'paxos_batch', 'paxos_wire', 'paxos_multi']]
subprocess.run([g.HIPCC, *g.HIPFLAGS, '-shared', '-o', 'variants/%s.so' % sys.argv[1], *objs, *base, '-lrccl'], check=True)
" "$@"
