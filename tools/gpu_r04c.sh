#!/bin/bash
# round-4: MODWT inverse W prefetch depth A/B (parity under both, rocprof stats of D = 2)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_ab_wl.sh modwt "JWV_MODWT_D2=0" "JWV_MODWT_D2=1" 3 "modwt" > gpurun_out/r04c_d2.txt 2>&1 || { cat gpurun_out/r04c_d2.txt; exit 1; }
cat gpurun_out/r04c_d2.txt
JWV_MODWT_D2=1 bash tools/gpu_kstats.sh r04c_ks_modwt modwt > gpurun_out/r04c_ks_modwt.txt 2>&1 || { cat gpurun_out/r04c_ks_modwt.txt; exit 1; }
cat gpurun_out/r04c_ks_modwt.txt
