#!/bin/bash
# The driver's round-end bench command (one GPU), timed, with a one-line summary.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/drv
start=$(date +%s)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv/bench.json 2> gpurun_out/drv/bench.err || { tail -20 gpurun_out/drv/bench.err; exit 1; }
echo "wall $(( $(date +%s) - start )) s"
python3 - <<'PY'
import json
j = json.load(open("gpurun_out/drv/bench.json"))
print("value %.4g ms/step %.2f frac %.3f" % (j["value"], j["ms_per_step"], j["roofline"]["frac"]))
ns = j["north_star"]
print("north star %.4g M/s frac %.3f" % (ns["instances_per_s"] / 1e6, ns["roofline"]["frac"]))
for k, v in j["extra"].items():
    if "instances_per_s" in v:
        print(k, "%.4g M/s" % (v["instances_per_s"] / 1e6))
print("cpu", j["cpu_baseline"]["value"], j["cpu_baseline"]["cores"])
PY
