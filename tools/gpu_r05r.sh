#!/bin/bash
# round 5: array-head pairs of the couple reverse tiles from LDS-staged taps (no register-select rotation)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "fwt" > gpurun_out/r05r_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05r_parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh fwt2d 3 jwave_amd/lib/ab_revold.so jwave_amd/lib/ab_revtl.so jwave_amd/lib/ab_small_nolin.so jwave_amd/lib/ab_small_lin.so 2>&1 | tee gpurun_out/r05r_ab.txt
