for cap in 0 16 20 24; do echo "== cap $cap"; PXB_BLOCKS_PER_CU=$cap timeout -k 10 200 python3 tools/exp.py variants/multi2.so 2>&1 | grep -v amdgpu.ids | cut -c1-120 || exit 1; done
