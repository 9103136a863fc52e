#!/bin/bash
# round 5: WPT LDS-only levels without the +0.0 start (ZS), signed-zero parity, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "wpt" > gpurun_out/r05p_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05p_parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh wpt 3 jwave_amd/lib/ab_wptzs.so jwave_amd/lib/ab_wptnzs.so 2>&1 | tee gpurun_out/r05p_ab.txt
