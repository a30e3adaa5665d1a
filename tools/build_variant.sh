#!/bin/bash
# bash tools/build_variant.sh <name> [-D... extra hipcc flags]  -> variants/<name>.so
set -e
R=$(cd $(dirname $0)/.. && pwd)
name=$1; shift
mkdir -p $R/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-pass-failed "$@" -shared \
  -o $R/variants/$name.so $R/cloud-haskell-paxos_amd/csrc/paxos_batch.hip $R/cloud-haskell-paxos_amd/csrc/paxos_multi.cpp -lrccl
