#!/bin/bash
# round-4: resident column passes, 16-column blocks vs XCD-paired half slabs (JWV_COLW=8)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_ab_multi.sh fwt2d 2 "2d or 3d or axis" "JWV_COLW=16" "JWV_COLW=8" > gpurun_out/r04h_ab.txt 2>&1 || { cat gpurun_out/r04h_ab.txt; exit 1; }
cat gpurun_out/r04h_ab.txt
JWV_COLW=8 bash tools/gpu_kstats.sh r04h_ks8 fwt2d > gpurun_out/r04h_ks8.txt 2>&1 || { cat gpurun_out/r04h_ks8.txt; exit 3; }
head -9 gpurun_out/r04h_ks8.txt
