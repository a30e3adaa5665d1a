#!/bin/bash
# Round 5, first GPU pass of the tight routing (config 4): parity tests of the
# new routing, an A/B against layout 6 alone (PXB_NO_TIGHT=1), and a kernel
# trace of one 2^26 north-star step.  Output under gpurun_out/r05a/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05a
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "tight or contiguous or configs_match or golden or north_star or bail_list" > gpurun_out/r05a/pytest.log 2>&1 \
  || { tail -40 gpurun_out/r05a/pytest.log; exit 1; }
tail -3 gpurun_out/r05a/pytest.log
AB_PASSES=2 AB_CASES=4:16777216:2,4:67108864:1 timeout -k 10 300 python3 -u tools/ab_ev.py \
  cloud-haskell-paxos_amd/csrc/libpaxos_batch.so cloud-haskell-paxos_amd/csrc/libpaxos_batch.so@PXB_NO_TIGHT=1 \
  cloud-haskell-paxos_amd/csrc/libpaxos_batch.so cloud-haskell-paxos_amd/csrc/libpaxos_batch.so@PXB_NO_TIGHT=1 \
  > gpurun_out/r05a/ab.txt 2>&1 || { cat gpurun_out/r05a/ab.txt; exit 1; }
cat gpurun_out/r05a/ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05a/trace -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu --no-extra --one-stream --config 4 --steps 2 --warmup 1 > $R/gpurun_out/r05a/bench.json \
  2> $R/gpurun_out/r05a/trace.log || { tail -5 $R/gpurun_out/r05a/trace.log; exit 1; }
cat $R/gpurun_out/r05a/bench.json | head -c 600; echo
find $R/gpurun_out/r05a/trace -name '*kernel_stats.csv' -exec cat {} \;
