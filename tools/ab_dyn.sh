set -o pipefail
mkdir -p gpurun_out/dyn
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dyn/pytest.log 2>&1 || { tail -30 gpurun_out/dyn/pytest.log; exit 1; }
tail -2 gpurun_out/dyn/pytest.log
timeout -k 10 300 python -u tools/cfg_rates.py > gpurun_out/dyn/new.txt 2>&1 || { cat gpurun_out/dyn/new.txt; exit 1; }
cat gpurun_out/dyn/new.txt
timeout -k 10 300 python -u tools/cfg_rates.py variants/static.so > gpurun_out/dyn/static.txt 2>&1 || { cat gpurun_out/dyn/static.txt; exit 1; }
cat gpurun_out/dyn/static.txt
