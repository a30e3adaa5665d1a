for v in "$@"; do echo "== $v"; timeout -k 10 300 python3 tools/cfg_rates.py variants/$v.so 2>&1 | grep -v amdgpu.ids | cut -c1-130 || exit 1; done
