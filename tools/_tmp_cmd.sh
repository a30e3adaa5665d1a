set -o pipefail
cd $GRAFT_REPO_ROOT
for v in st_v4b st_v5b; do echo "== $v"; PXB_LIB=$GRAFT_REPO_ROOT/variants/$v.so timeout -k 10 200 python3 tools/stamps.py 2>&1 | grep -v amdgpu.ids || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/avail.txt 2>&1 || true
grep -i -E "icache|ifetch|SQC_" $GRAFT_REPO_ROOT/gpurun_out/avail.txt | head -40
