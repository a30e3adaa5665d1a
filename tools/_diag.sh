set -o pipefail
O=gpurun_out/diag2; mkdir -p $O
for v in m2; do
  PXB_LIB=$PWD/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "config or topolog or golden or edge or log or multi" > $O/pt_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 $O/pt_$v.log; exit 1; }
  tail -1 $O/pt_$v.log
done
timeout -k 10 400 python3 tools/exp.py variants/mall1.so variants/m2.so > $O/exp.log 2>&1
cat $O/exp.log
