#!/bin/bash
# round 5: config-3 forward column tile 16-column (78 KB) vs 8-column (40 KB) slabs
set -o pipefail
mkdir -p gpurun_out
JWAVE_AMD_LIB=jwave_amd/lib/ab_f8.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "fwt2d or fwt3d or parallel" > gpurun_out/r05w2_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05w2_parity.log; [ $rc -eq 0 ] || exit $rc
JWAVE_AMD_LIB=jwave_amd/lib/ab_h16.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "fwt2d or fwt3d or parallel" > gpurun_out/r05w2_parity_h16.log 2>&1 || exit 1; tail -1 gpurun_out/r05w2_parity_h16.log; bash tools/gpu_ab_libs.sh fwt2d 4 jwave_amd/lib/ab_f16.so jwave_amd/lib/ab_f8.so jwave_amd/lib/ab_h16.so 2>&1 | tee gpurun_out/r05w2_ab.txt
