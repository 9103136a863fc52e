#!/bin/bash
# round-4: streamed MODWT inverse (JWV_MODWT_STREAM=1: 256 x 512, =2: 512 x 1024)
# and forward (JWV_MODWT_FSTREAM=1: 256 x 1024, =2: 512 x 1024): parity + A/B
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_ab_multi.sh modwt 2 "modwt" "JWV_MODWT_STREAM=0" "JWV_MODWT_STREAM=1" "JWV_MODWT_STREAM=2" "JWV_MODWT_FSTREAM=1" "JWV_MODWT_FSTREAM=2" > gpurun_out/r04e_ab.txt 2>&1 || { cat gpurun_out/r04e_ab.txt; exit 1; }
cat gpurun_out/r04e_ab.txt
bash tools/gpu_ab_multi.sh wpt 2 "wpt_config4_shape or wpt_large or wpt_batch" "JWV_WPT_FSTREAM=0" "JWV_WPT_FSTREAM=1" "JWV_WPT_FSTREAM=2" "JWV_WPT_FSTREAM=3" > gpurun_out/r04e_abw.txt 2>&1 || { cat gpurun_out/r04e_abw.txt; exit 1; }
cat gpurun_out/r04e_abw.txt
bash tools/gpu_ab_multi.sh wpt 2 "wpt_config4_shape or wpt_large or wpt_batch" "JWV_WPT_RSTREAM=0" "JWV_WPT_RSTREAM=1" "JWV_WPT_RSTREAM=2" "JWV_WPT_RSTREAM=3" > gpurun_out/r04e_abr.txt 2>&1 || { cat gpurun_out/r04e_abr.txt; exit 1; }
cat gpurun_out/r04e_abr.txt
