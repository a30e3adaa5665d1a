#!/bin/bash
# Quick check: GPU parity tests (fast subset or all) + A/B timing of variants.
#   bash tools/gpu_quick.sh <tag> <pytest -k expr or "all"> lib1.so [lib2.so ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; K=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$K" = "all" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
fi
tail -2 $O/pytest.log
timeout -k 10 500 python3 tools/exp.py "$@" > $O/exp.log 2>&1 || { echo "exp failed"; tail $O/exp.log; exit 1; }
cat $O/exp.log
