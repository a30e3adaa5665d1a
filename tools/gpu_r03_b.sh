#!/bin/bash
# GPU suite + short bench on the current build, then an A/B of the variants given.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r3b
for l in "$@"; do test -f "$l" || { echo "missing $l"; exit 1; }; done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3b/parity.log 2>&1 || { tail -40 gpurun_out/r3b/parity.log; exit 1; }
tail -2 gpurun_out/r3b/parity.log
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/r3b/bench.json 2> gpurun_out/r3b/bench.err || { tail -20 gpurun_out/r3b/bench.err; exit 1; }
python3 - <<'PY'
import json
j = json.load(open("gpurun_out/r3b/bench.json"))
print("headline %.2f G/s" % (j["value"] / 1e9))
ns = j["north_star"]; print("north star %.2f M/s (%.1f ms)" % (ns["instances_per_s"] / 1e6, ns["ms_per_step"]))
for k, v in j.get("extra", {}).items():
    if "instances_per_s" in v:
        print("%s %.2f M/s%s" % (k, v["instances_per_s"] / 1e6, (" (x%.2f vs general kernel)" % v["speedup_vs_general_kernel"]) if "speedup_vs_general_kernel" in v else ""))
PY
if [ $# -gt 0 ]; then
  AB_CASES=4:8388608:1,3:4194304:2 timeout -k 10 400 python3 -u tools/ab_ev.py "$@" "$@" > gpurun_out/r3b/ab.txt 2>&1 || { cat gpurun_out/r3b/ab.txt; exit 1; }
  cat gpurun_out/r3b/ab.txt
fi
