set -o pipefail
O=gpurun_out/diag13; mkdir -p $O
PXB_LIB=$PWD/variants/occ24.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "config or topolog" > $O/pt.log 2>&1 || { echo "pytest failed"; tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
timeout -k 10 400 python3 tools/exp.py variants/base.so variants/occ24.so > $O/exp.log 2>&1
cat $O/exp.log
