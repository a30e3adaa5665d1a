#!/bin/bash
# One GPU lease, any sequence of steps (replaces the per-round gpu_r0*_*.sh
# one-offs).  Every step runs under its own time limit; the first failure ends
# the lease (no GPU step runs after a failed, killed or timed-out one).
#
#   bash tools/gpu_lease.sh <tag> <step> [<step> ...]
#
# steps (arguments after ':' separated by ','):
#   tests                      the full -m gpu suite
#   tests:<pytest -k expr>     a subset of it
#   fuzz:<schedules>,<n>[,<seed>[,<kind>+<kind>...]]   tests/fuzz_gpu.py, GPU vs the C oracle
#   bench                      the default bench line (bench.py, CPU baseline and extra included)
#   bench:<bench.py args>      e.g. bench:--no-cpu --no-extra --steps 5  (spaces allowed)
#   ab:<lib.so>+<lib.so>...    tools/ab_ev.py A/B of library variants (AB_CASES, AB_PASSES from the env)
#   prof:<config>,<n>,<steps>,<warmup>[,<round>]   tools/profile_set.sh -> profiles/<round>_config<c>
#   wt:<lib.so>,<config>,<n>   per-wave timelines (tools/ev_wave_times.py, a -DPXB_WAVE_TIMES build)
#   env:<VAR>=<value>          set a library hook (PXB_NO_LG2=1, ...) for the steps after it
#   unenv:<VAR>                unset it again
# Output: gpurun_out/<tag>/ (step logs, bench JSON lines, profiles).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R || exit 1
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
k=0
for step in "$@"; do
  k=$((k + 1))
  name=${step%%:*}
  arg=""; [[ "$step" == *:* ]] && arg=${step#*:}
  echo "== step $k: $step"
  case $name in
    tests)
      if [ -n "$arg" ]; then
        timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$arg" > $O/pytest_$k.log 2>&1
      else
        timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$k.log 2>&1
      fi
      rc=$?; tail -3 $O/pytest_$k.log; [ $rc -eq 0 ] || { tail -40 $O/pytest_$k.log; exit 1; } ;;
    fuzz)
      IFS=, read -r ns ni seed kinds <<< "$arg"
      timeout -k 10 600 python3 -u tests/fuzz_gpu.py $ns $ni $seed ${kinds//+/,} > $O/fuzz_$k.txt 2>&1 || { tail -20 $O/fuzz_$k.txt; exit 1; }
      tail -1 $O/fuzz_$k.txt ;;
    bench)
      timeout -k 10 600 python3 -u bench.py $arg > $O/bench_$k.json 2> $O/bench_$k.err || { tail -20 $O/bench_$k.err; exit 1; }
      python3 tools/bench_summary.py $O/bench_$k.json ;;
    ab)
      libs=${arg//+/ }
      for l in $libs; do test -f "${l%%@*}" || { echo "missing $l"; exit 1; }; done
      LIBS=(); for p in $(seq ${AB_PASSES:-2}); do LIBS+=($libs); done
      AB_CASES=${AB_CASES:-4:8388608:1,3:4194304:2} timeout -k 10 900 python3 -u tools/ab_ev.py "${LIBS[@]}" > $O/ab_$k.txt 2>&1 || { cat $O/ab_$k.txt; exit 1; }
      cat $O/ab_$k.txt ;;
    prof)
      IFS=, read -r c n s w rnd <<< "$arg"; rnd=${rnd:-r06}
      timeout -k 10 900 bash tools/profile_set.sh $O/config$c $c $n $s $w || exit 1
      D=$O/prof/${rnd}_config$c; mkdir -p $D
      cp $O/config$c/step.json $D/
      cp $(find $O/config$c/trace -name '*kernel_stats.csv' | head -1) $D/kernel_stats.csv
      cp $(find $O/config$c/valu -name '*counter_collection.csv' | head -1) $D/pmc_valu.csv
      cp $(find $O/config$c/fetch -name '*counter_collection.csv' | head -1) $D/pmc_fetch.csv
      cp $(find $O/config$c/write -name '*counter_collection.csv' | head -1) $D/pmc_write.csv
      # (bench.py reads profiles/<round>_config<c>: the box's profiles feed the bench line after them)
      mkdir -p profiles && rm -rf profiles/${rnd}_config$c && cp -r $D profiles/ ;;
    wt)
      IFS=, read -r lib c n <<< "$arg"
      timeout -k 10 300 python3 -u tools/ev_wave_times.py $lib $c $n > $O/wt_$k.txt 2>&1 || { tail -20 $O/wt_$k.txt; exit 1; }
      cat $O/wt_$k.txt ;;
    env) export "$arg" ;;
    unenv) unset "$arg" ;;
    *) echo "unknown step $step"; exit 1 ;;
  esac
done
echo "lease $TAG done"
