#!/bin/bash
# Profile sets (tools/profile_r02.sh) for the bench line's config-3 and
# config-5 entries, copied into profiles/r02_config{3,5}/ on the box (and
# back through gpurun_out/r02x/).   bash tools/gpu_prof_extra.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r02x
timeout -k 10 600 bash tools/profile_r02.sh gpurun_out/r02x/config3 3 16777216 1 1 || exit 1
timeout -k 10 600 bash tools/profile_r02.sh gpurun_out/r02x/config5 5 16777216 1 1 || exit 1
