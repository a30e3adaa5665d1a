#!/bin/bash
# Round-5 closing pass on one GPU box: the full -m gpu suite, the profile set
# of every bench line (tools/profile_set.sh: kernel-trace stats, SQ/GRBM,
# FETCH_SIZE and WRITE_SIZE passes -> step.json) into profiles/r05_*, then the
# default bench line, which reads those profiles: profile and bench from one box.
# Everything also lands under gpurun_out/fin5/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/fin5
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fin5/pytest.log 2>&1 || { tail -30 gpurun_out/fin5/pytest.log; exit 1; }
tail -1 gpurun_out/fin5/pytest.log
# GPU-vs-oracle fuzz over the per-lane shapes (tests/fuzz_gpu.py)
timeout -k 10 400 python3 -u tests/fuzz_gpu.py 2000 16384 > gpurun_out/fin5/fuzz.txt 2>&1 || { tail -20 gpurun_out/fin5/fuzz.txt; exit 1; }
tail -1 gpurun_out/fin5/fuzz.txt
prof() {   # <config> <instances per step> <steps> <warmup>
  timeout -k 10 600 bash tools/profile_set.sh gpurun_out/fin5/config$1 $1 $2 $3 $4 || return 1
  D=gpurun_out/fin5/prof/r05_config$1; mkdir -p $D
  cp gpurun_out/fin5/config$1/step.json $D/
  cp $(find gpurun_out/fin5/config$1/trace -name '*kernel_stats.csv' | head -1) $D/kernel_stats.csv
  cp $(find gpurun_out/fin5/config$1/valu -name '*counter_collection.csv' | head -1) $D/pmc_valu.csv
  cp $(find gpurun_out/fin5/config$1/fetch -name '*counter_collection.csv' | head -1) $D/pmc_fetch.csv
  cp $(find gpurun_out/fin5/config$1/write -name '*counter_collection.csv' | head -1) $D/pmc_write.csv
  mkdir -p profiles && rm -rf profiles/r05_config$1 && cp -r $D profiles/   # (the bench below reads them)
}
# (two warmup steps and one stream, tools/profile_set.sh: every dispatch of a kernel is the same
# size and runs alone, so rocprof's average duration is the per-launch kernel time)
prof 4 67108864 1 2 && prof 2 268435456 2 2 && prof 3 16777216 1 2 && prof 5 33554432 1 2 && prof 7 4194304 2 2 || exit 1
timeout -k 10 600 python3 -u bench.py > gpurun_out/fin5/bench.json 2> gpurun_out/fin5/bench.err || { tail -20 gpurun_out/fin5/bench.err; exit 1; }
cp gpurun_out/fin5/bench.json gpurun_out/fin5/prof/r05_bench.json
python3 -c "
import json; j=json.load(open('gpurun_out/fin5/bench.json'))
print('headline %.4g %s  ms/step %.2f  roofline frac %s' % (j['value'], j['unit'], j['ms_per_step'], j['roofline']['frac']))
for k, v in j['extra'].items():
    if 'instances_per_s' in v: print(k, '%.4g inst/s' % v['instances_per_s'], 'frac', (v.get('roofline') or {}).get('frac'))
print('cpu', j['cpu_baseline']['value'], j['cpu_baseline']['cores'])"
