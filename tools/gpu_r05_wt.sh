set -o pipefail
mkdir -p gpurun_out/r05wt
timeout -k 10 120 python3 -u tools/ev_wave_times.py variants/v_wt.so 4 8388608 > gpurun_out/r05wt/tight.txt 2>&1 && \
PXB_NO_TIGHT=1 timeout -k 10 120 python3 -u tools/ev_wave_times.py variants/v_wt.so 4 8388608 > gpurun_out/r05wt/l6.txt 2>&1
cat gpurun_out/r05wt/tight.txt gpurun_out/r05wt/l6.txt
