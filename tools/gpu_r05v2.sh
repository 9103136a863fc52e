#!/bin/bash
# round 5: WPT forward 8192-sample tiles with 640 threads (5 waves/SIMD at 2 blocks/CU) vs 512
set -o pipefail
mkdir -p gpurun_out
JWAVE_AMD_LIB=jwave_amd/lib/ab_fnt640.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "wpt" > gpurun_out/r05v2_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05v2_parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh wpt 4 jwave_amd/lib/ab_fnt512.so jwave_amd/lib/ab_fnt640.so 2>&1 | tee gpurun_out/r05v2_ab.txt
