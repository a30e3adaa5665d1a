#!/bin/bash
# Round 5 (final code): where the per-lane waves' cycles go (PMC_CONFIG, PMC_N: default config 4 at 2^24);
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r05pmc2
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH"
for tag in tight; do
  if [ $tag = l6 ]; then export PXB_NO_TIGHT=1; else unset PXB_NO_TIGHT; fi
  for pass in 1 2; do
    C=$P1; [ $pass = 2 ] && C=$P2
    timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/r05pmc2/$tag$pass -o pmc --output-format csv -- python3 $R/bench.py --config ${PMC_CONFIG:-4} --instances ${PMC_N:-16777216} --steps 1 --warmup 1 --no-cpu --no-extra --one-stream > $R/gpurun_out/r05pmc2/$tag$pass.log 2>&1 || { tail -5 $R/gpurun_out/r05pmc2/$tag$pass.log; exit 1; }
  done
done
cd $R && python3 - <<'PY'
import csv, glob, collections
for tag in ("tight",):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in (1, 2):
        f = glob.glob("gpurun_out/r05pmc2/%s%d/**/*counter_collection.csv" % (tag, p), recursive=True)[0]
        for r in csv.DictReader(open(f)):
            if "paxos_ev_kernel" in r["Kernel_Name"]:
                agg[r["Kernel_Name"].split("(")[0][-28:]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in agg.items():
        wc = v["SQ_WAVE_CYCLES"]
        print(tag, k, " ".join("%s %.4g" % (n[3:], v[n] / wc if n.startswith(("SQ_WAIT", "SQ_ACTIVE")) else v[n]) for n in sorted(v)))
PY
