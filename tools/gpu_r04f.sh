#!/bin/bash
# round-4: stream geometries A/B (MODWT forward; WPT forward/reverse 512 x 4096)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_ab_multi.sh modwt 2 "modwt" "JWV_MODWT_FSTREAM=0" "JWV_MODWT_FSTREAM=2" "JWV_MODWT_FSTREAM=3" "JWV_MODWT_FSTREAM=4" > gpurun_out/r04f_ab.txt 2>&1 || { cat gpurun_out/r04f_ab.txt; exit 1; }
cat gpurun_out/r04f_ab.txt
bash tools/gpu_ab_multi.sh wpt 2 "wpt_config4_shape or wpt_large or wpt_batch" "JWV_WPT_FSTREAM=0" "JWV_WPT_FSTREAM=4 JWV_WPT_RSTREAM=4" > gpurun_out/r04f_abw.txt 2>&1 || { cat gpurun_out/r04f_abw.txt; exit 1; }
cat gpurun_out/r04f_abw.txt
