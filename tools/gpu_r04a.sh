#!/bin/bash
# round-4 measurements: parity of the touched paths, MODWT pipe A/B + stats,
# WPT pad A/B, C16 column slabs A/B
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "wpt or fwt2d or 3d or modwt or jni or rowcap or fwt_large or fwt_batch or decompose or aed or parallel" > gpurun_out/r04b_tests.txt 2>&1
rc=$?; tail -4 gpurun_out/r04b_tests.txt
# assertion failures (rc 1) do not stop the measurements; a crash, abort or timeout does
[ $rc -le 1 ] || exit 1
bash tools/gpu_ab_wl.sh modwt "JWV_MODWT_PIPE=0" "JWV_MODWT_PIPE=3" 3 "modwt" > gpurun_out/r04b_pipe.txt 2>&1 || { cat gpurun_out/r04b_pipe.txt; exit 1; }
cat gpurun_out/r04b_pipe.txt
JWV_MODWT_PIPE=3 bash tools/gpu_kstats.sh r04b_ks_modwt modwt > gpurun_out/r04b_ks_modwt.txt 2>&1 || { cat gpurun_out/r04b_ks_modwt.txt; exit 1; }
cat gpurun_out/r04b_ks_modwt.txt
bash tools/gpu_ab_wl.sh wpt "JWV_WPT_PAD=0" "JWV_WPT_PAD=1" 2 "wpt_config4 or wpt_large" > gpurun_out/r04b_pad.txt 2>&1 || { cat gpurun_out/r04b_pad.txt; exit 1; }
cat gpurun_out/r04b_pad.txt
bash tools/gpu_ab_wl.sh fwt2d "JWV_FWT16=0" "JWV_FWT16=1" 2 "fwt2d or 3d or axis_columns" > gpurun_out/r04b_fwt16.txt 2>&1 || { cat gpurun_out/r04b_fwt16.txt; exit 1; }
cat gpurun_out/r04b_fwt16.txt
