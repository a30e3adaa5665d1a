set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/kt
cd /tmp && export TMPDIR=/tmp
for NI in 8388608 67108864; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt/n$NI -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-extra --config 4 --instances $NI --steps 2 --warmup 1 > $R/gpurun_out/kt/bench_$NI.json 2> $R/gpurun_out/kt/log_$NI.txt || exit 1
  echo "done $NI"
done
