#!/bin/bash
# round-4: WPT tile block sizes (JWV_WPT_NT bit 0: 512-thread reverse, bit 1: 1024-thread forward)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_ab_multi.sh wpt 2 "wpt_config4_shape or wpt_large or wpt_batch" "JWV_WPT_NT=0" "JWV_WPT_NT=1" "JWV_WPT_NT=2" > gpurun_out/r04i_ab.txt 2>&1 || { cat gpurun_out/r04i_ab.txt; exit 1; }
cat gpurun_out/r04i_ab.txt
