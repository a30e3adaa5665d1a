#!/bin/bash
# Round 5: ff1 static share + dynamic tail, A/B by static eighths against the base library (config 2, 2^28 launches).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05f
V=variants/ff1b.so
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "ff1 or configs_match or config2 or ragged or work_queue or fault_free" > gpurun_out/r05f/pytest.log 2>&1 \
  || { tail -40 gpurun_out/r05f/pytest.log; exit 1; }
tail -2 gpurun_out/r05f/pytest.log
AB_CASES=2:268435456:5 timeout -k 10 400 python3 -u tools/ab_ev.py variants/base_r05.so $V $V@PXB_FF1_STATIC_EIGHTHS=8 $V@PXB_FF1_STATIC_EIGHTHS=6 $V@PXB_FF1_STATIC_EIGHTHS=0 \
  variants/base_r05.so $V $V@PXB_FF1_STATIC_EIGHTHS=8 $V@PXB_FF1_STATIC_EIGHTHS=6 $V@PXB_FF1_STATIC_EIGHTHS=0 > gpurun_out/r05f/ab2.txt 2>&1 || { cat gpurun_out/r05f/ab2.txt; exit 1; }
cat gpurun_out/r05f/ab2.txt
# north-star step streams with the tight routing: one vs two (2^26 per step)
for s in 1 2 1 2; do
  timeout -k 10 120 python3 -u bench.py --no-cpu --no-extra --config 4 --steps 4 --warmup 1 --streams $s > gpurun_out/r05f/bench_s$s.json 2> gpurun_out/r05f/bench_s$s.err || { tail -5 gpurun_out/r05f/bench_s$s.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/r05f/bench_s$s.json')); print('streams $s: %.2f M/s, %.1f ms/step' % (j['value']/1e6, j['ms_per_step']))"
done
# flat step end (END_FLAT) against the current library, config 4
L=cloud-haskell-paxos_amd/csrc/libpaxos_batch.so
AB_CASES=4:16777216:2,4:67108864:1 timeout -k 10 400 python3 -u tools/ab_ev.py $L variants/ef1.so $L variants/ef1.so > gpurun_out/r05f/ab4.txt 2>&1 || { cat gpurun_out/r05f/ab4.txt; exit 1; }
cat gpurun_out/r05f/ab4.txt
