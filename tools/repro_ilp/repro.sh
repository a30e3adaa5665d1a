#!/bin/bash
# Compile one per-lane kernel shape with the flag set that crashes the
# compiler, then with each ingredient removed.  Prints one line per build.
# Found with ROCm 7.2.0 (hipcc / clang-22, gfx950); see DESIGN.md §3.
cd "$(dirname "$0")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
BASE="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -phi-node-folding-threshold=16 -mllvm -two-entry-phi-node-folding-threshold=64 -mllvm -amdgpu-atomic-optimizer-strategy=None -c -o /tmp/repro_ilp.o one_unit.hip"
ILP="-mllvm -amdgpu-sched-strategy=iterative-ilp"
$HIPCC --version 2>/dev/null | grep -m1 -i "clang version"
run() {
  if $HIPCC $BASE $2 > /tmp/repro_ilp.log 2>&1; then echo "$1: ok"
  elif grep -q "Segmentation fault" /tmp/repro_ilp.log; then
    echo "$1: COMPILER SEGFAULT ($(grep -m1 -o "Running pass '[^']*' on function '[^']*'" /tmp/repro_ilp.log))"
  else echo "$1: error (see /tmp/repro_ilp.log)"; fi
}
run "iterative-ilp + asm v_bfi_b32 (the library's form)" "$ILP"
run "iterative-ilp + bitop3 builtin selects" "$ILP -DPXB_EV_BITOP3_BFI"
run "default scheduler + asm v_bfi_b32" ""
