#!/bin/bash
# GPU suite + a short bench line (no CPU baseline): the routine check after a change.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/chk
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/chk/parity.log 2>&1 || { tail -40 gpurun_out/chk/parity.log; exit 1; }
tail -2 gpurun_out/chk/parity.log
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/chk/bench.json 2> gpurun_out/chk/bench.err || { tail -20 gpurun_out/chk/bench.err; exit 1; }
python3 - <<'PY'
import json
j = json.load(open("gpurun_out/chk/bench.json"))
print("headline %.2f G/s" % (j["value"] / 1e9))
ns = j["north_star"]; print("north star %.2f M/s (%.1f ms)" % (ns["instances_per_s"] / 1e6, ns["ms_per_step"]))
for k, v in j.get("extra", {}).items():
    if "instances_per_s" in v:
        print("%s %.2f M/s%s" % (k, v["instances_per_s"] / 1e6, (" (x%.2f vs general kernel)" % v["speedup_vs_general_kernel"]) if "speedup_vs_general_kernel" in v else ""))
PY
