#!/bin/bash
# round-4 measurements: full GPU suite (cleaned library), MODWT pipe A/B,
# kernel stats, WPT pad (parity + A/B)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T="timeout -k 10"
$T 120 tools/diag/fp64_rate > gpurun_out/r04a_fp64_rate.txt 2>&1 || { cat gpurun_out/r04a_fp64_rate.txt; exit 1; }
cat gpurun_out/r04a_fp64_rate.txt
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04a_tests.txt 2>&1 || { tail -40 gpurun_out/r04a_tests.txt; exit 1; }
tail -2 gpurun_out/r04a_tests.txt
bash tools/gpu_ab_wl.sh modwt "JWV_MODWT_PIPE=0" "JWV_MODWT_PIPE=3" 3 "modwt" > gpurun_out/r04a_pipe.txt 2>&1 || { cat gpurun_out/r04a_pipe.txt; exit 1; }
cat gpurun_out/r04a_pipe.txt
JWV_MODWT_PIPE=3 bash tools/gpu_kstats.sh r04a_ks_modwt modwt > gpurun_out/r04a_ks_modwt.txt 2>&1 || { cat gpurun_out/r04a_ks_modwt.txt; exit 1; }
cat gpurun_out/r04a_ks_modwt.txt
bash tools/gpu_ab_wl.sh wpt "JWV_WPT_PAD=0" "JWV_WPT_PAD=1" 2 "wpt_config4 or wpt_large" > gpurun_out/r04a_pad.txt 2>&1 || { cat gpurun_out/r04a_pad.txt; exit 1; }
cat gpurun_out/r04a_pad.txt
bash tools/gpu_ab_wl.sh fwt2d "JWV_FWT16=0" "JWV_FWT16=1" 2 "fwt2d or 3d or axis_columns or parallel_transform" > gpurun_out/r04a_fwt16.txt 2>&1 || { cat gpurun_out/r04a_fwt16.txt; exit 1; }
cat gpurun_out/r04a_fwt16.txt
