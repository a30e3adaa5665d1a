set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/s25
for v in base s25; do
  if [ $v = base ]; then unset PXB_LIB; else export PXB_LIB=variants/$v.so; fi
  timeout -k 10 200 python3 -u bench.py --config 5 --instances 33554432 --steps 2 --warmup 1 --no-cpu --no-extra > gpurun_out/s25/$v.json 2> gpurun_out/s25/$v.err || { cat gpurun_out/s25/$v.err; exit 1; }
  python3 -c "import json; e=json.load(open('gpurun_out/s25/$v.json')); print('$v config 5 2^25: %.2f M inst/s' % (e['counters']['instances']/e['ms_per_step']/2e3))"
done
