set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/c5s
for pass in 1 2; do for ns in 1 2; do
timeout -k 10 200 python3 bench.py --config 5 --instances 33554432 --no-cpu --no-extra --streams $ns --steps 4 --warmup 2 > gpurun_out/c5s/s${ns}_$pass.json 2>gpurun_out/c5s/err.log || exit 1
python3 -c "import json; j=json.load(open('gpurun_out/c5s/s${ns}_$pass.json')); print('streams $ns pass $pass', round(j['value']/1e6,2), 'M/s', round(j['ms_per_step'],1), 'ms')"
done; done
