#!/bin/bash
# round-4: config-3 row reverse tile geometry (JWV_REV1G)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_ab_multi.sh fwt2d 2 "fwt2d or fwt_large or fwt_batch or 2d" "JWV_REV1G=0" "JWV_REV1G=1" "JWV_REV1G=2" "JWV_REV1G=3" > gpurun_out/r04k_ab.txt 2>&1 || { cat gpurun_out/r04k_ab.txt; exit 1; }
cat gpurun_out/r04k_ab.txt
