#!/bin/bash
# round 5: WPT slot division unsigned + unpredicated reverse couple stores
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "wpt" > gpurun_out/r05o_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05o_parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh wpt 3 jwave_amd/lib/ab_wptold.so jwave_amd/lib/ab_wptnew.so 2>&1 | tee gpurun_out/r05o_ab.txt
