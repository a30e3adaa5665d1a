set -e
echo "nproc=$(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"
cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cpu.max"; cat /proc/cpuinfo | grep "model name" | head -1
rocm-smi --showclocks 2>/dev/null | head -20 || true
timeout -k 10 300 bash tools/pmc_config.sh gpurun_out/r02_base_c4 4 16777216
echo done
