#!/bin/bash
# round 5: MODWT inverse without the barrier before the final level's global stores
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "modwt or signed_zeros" > gpurun_out/r05y4_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05y4_parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh modwt 4 jwave_amd/lib/ab_mb1.so jwave_amd/lib/ab_mb0.so 2>&1 | tee gpurun_out/r05y4_ab.txt
