#!/bin/bash
# Round-2 GPU pass: full -m gpu suite, the profile sets bench.py's roofline
# reads (config 2 headline step = 64 x 2^20, config 4 north star), then the
# default bench.  Everything lands under gpurun_out/r02/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r02
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02/pytest.log 2>&1 || { tail -30 gpurun_out/r02/pytest.log; exit 1; }
tail -1 gpurun_out/r02/pytest.log
timeout -k 10 600 bash tools/profile_r02.sh gpurun_out/r02/config2 2 67108864 2 1 || exit 1
timeout -k 10 600 bash tools/profile_r02.sh gpurun_out/r02/config4 4 16777216 1 1 || exit 1
mkdir -p profiles/r02_config2 profiles/r02_config4
cp gpurun_out/r02/config2/step.json profiles/r02_config2/ && cp gpurun_out/r02/config4/step.json profiles/r02_config4/
timeout -k 10 400 python -u bench.py > gpurun_out/r02/bench.json 2> gpurun_out/r02/bench.err || { tail -20 gpurun_out/r02/bench.err; exit 1; }
python3 -c "
import json; j=json.load(open('gpurun_out/r02/bench.json'))
print('headline %.3g %s  ms/step %.2f  roofline frac %s' % (j['value'], j['unit'], j['ms_per_step'], j['roofline']['frac']))
ns=j['north_star']; print('north star %.3g inst/s  frac %s' % (ns['instances_per_s'], ns['roofline']['frac']))
print('cpu', j['cpu_baseline']['value'], j['cpu_baseline']['cores'])"
