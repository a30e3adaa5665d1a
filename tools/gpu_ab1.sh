set -o pipefail
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out/ab1
timeout -k 10 120 tools/micro/mul_rate > gpurun_out/ab1/mul_rate.txt 2>&1 || exit 1
AB_CASES=4:8388608:1,3:4194304:2 timeout -k 10 500 python3 -u tools/ab_ev.py variants/base.so variants/ilp2.so variants/maxilp2.so variants/base.so variants/ilp2.so variants/maxilp2.so > gpurun_out/ab1/ab.txt 2>&1 || { cat gpurun_out/ab1/ab.txt; exit 1; }
cat gpurun_out/ab1/mul_rate.txt gpurun_out/ab1/ab.txt
