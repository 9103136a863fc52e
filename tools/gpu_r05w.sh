#!/bin/bash
# round 5: config-3 forward column tile rows 512 (2 blocks/CU) vs 256 (3 blocks/CU, 38% halo)
set -o pipefail
mkdir -p gpurun_out
JWAVE_AMD_LIB=jwave_amd/lib/ab_t256.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "fwt2d or fwt3d or parallel" > gpurun_out/r05w_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05w_parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh fwt2d 4 jwave_amd/lib/ab_t512.so jwave_amd/lib/ab_t256.so 2>&1 | tee gpurun_out/r05w_ab.txt
