set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/ch
for c in 0 24 22 20; do
  if [ $c != 0 ]; then export PXB_FF1_CHUNK=$c; fi
  timeout -k 10 120 python3 -u bench.py --config 2 --steps 10 --warmup 2 --no-cpu --no-extra > gpurun_out/ch/c$c.json 2> gpurun_out/ch/c$c.err || { cat gpurun_out/ch/c$c.err; exit 1; }
  python3 -c "import json; e=json.load(open('gpurun_out/ch/c$c.json')); print('chunk 2^$c: %.3f G/s  %.3f ms/step' % (e['value']/1e9, e['ms_per_step']))"
done
