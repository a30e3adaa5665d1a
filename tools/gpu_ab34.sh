set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ab34
for v in base "$@"; do
  for c in 4 3; do
    if [ $v = base ]; then unset PXB_LIB; else export PXB_LIB=variants/$v.so; fi
    timeout -k 10 200 python3 -u bench.py --config $c --instances 16777216 --steps 2 --warmup 1 --no-cpu --no-extra > gpurun_out/ab34/$v.c$c.json 2> gpurun_out/ab34/$v.c$c.err || { cat gpurun_out/ab34/$v.c$c.err; exit 1; }
    python3 -c "import json; e=json.load(open('gpurun_out/ab34/$v.c$c.json')); print('$v config $c: %.2f M inst/s' % (e['counters']['instances']/e['ms_per_step']/2e3))"
  done
done
