set -o pipefail
O=gpurun_out/diag5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1 || { echo "pytest failed"; tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
timeout -k 10 400 python3 tools/exp.py variants/prev.so variants/flat.so > $O/exp.log 2>&1
cat $O/exp.log
