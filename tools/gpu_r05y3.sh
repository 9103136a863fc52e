#!/bin/bash
# round 5: MODWT forward stream V below the top level without the +0.0 start (JWV_MOD_NZS)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "modwt or signed_zeros" > gpurun_out/r05y3_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05y3_parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh modwt 4 jwave_amd/lib/ab_fz0.so jwave_amd/lib/ab_fz1.so 2>&1 | tee gpurun_out/r05y3_ab.txt
