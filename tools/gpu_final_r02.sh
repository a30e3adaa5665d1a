#!/bin/bash
# Round-2 closing pass on one GPU box: the full -m gpu suite, the profile set
# of every bench line (tools/profile_r02.sh: kernel-trace stats, SQ/GRBM,
# FETCH_SIZE and WRITE_SIZE passes -> step.json), copied into profiles/r02_*,
# then the default bench line.  Everything lands under gpurun_out/fin/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/fin
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fin/pytest.log 2>&1 || { tail -30 gpurun_out/fin/pytest.log; exit 1; }
tail -1 gpurun_out/fin/pytest.log
prof() {   # <config> <instances per step> <steps> <warmup>
  timeout -k 10 600 bash tools/profile_r02.sh gpurun_out/fin/config$1 $1 $2 $3 $4 || return 1
  mkdir -p profiles/r02_config$1   # (on the box; copy gpurun_out/fin back into profiles/ afterwards)
  cp gpurun_out/fin/config$1/step.json profiles/r02_config$1/
  cp $(find gpurun_out/fin/config$1/trace -name '*kernel_stats.csv' | head -1) profiles/r02_config$1/kernel_stats.csv
  cp $(find gpurun_out/fin/config$1/valu -name '*counter_collection.csv' | head -1) profiles/r02_config$1/pmc_valu.csv
  cp $(find gpurun_out/fin/config$1/fetch -name '*counter_collection.csv' | head -1) profiles/r02_config$1/pmc_fetch.csv
  cp $(find gpurun_out/fin/config$1/write -name '*counter_collection.csv' | head -1) profiles/r02_config$1/pmc_write.csv
}
prof 2 268435456 2 1 && prof 4 16777216 1 1 && prof 3 16777216 1 1 && prof 5 33554432 1 1 || exit 1
timeout -k 10 600 python3 -u bench.py > gpurun_out/fin/bench.json 2> gpurun_out/fin/bench.err || { tail -20 gpurun_out/fin/bench.err; exit 1; }
cp gpurun_out/fin/bench.json profiles/r02_bench.json
python3 -c "
import json; j=json.load(open('gpurun_out/fin/bench.json'))
print('headline %.4g %s  ms/step %.2f  roofline frac %s' % (j['value'], j['unit'], j['ms_per_step'], j['roofline']['frac']))
ns=j['north_star']; print('north star %.4g inst/s  frac %s' % (ns['instances_per_s'], ns['roofline']['frac']))
for k in ('config3', 'config5'): print(k, '%.4g inst/s' % j['extra'][k]['instances_per_s'], 'frac', j['extra'][k]['roofline']['frac'])
print('cpu', j['cpu_baseline']['value'], j['cpu_baseline']['cores'])"
