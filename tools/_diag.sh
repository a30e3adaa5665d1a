set -o pipefail
O=$PWD/gpurun_out/diag12; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_wire.py tests/test_abi.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1 || { echo "pytest failed"; tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 $R/tools/wire_ab.py cloud-haskell-paxos_amd/csrc/libpaxos_batch.so > $O/log 2>&1
cat $O/log | grep -v amdgpu.ids
