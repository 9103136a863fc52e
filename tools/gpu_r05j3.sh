#!/bin/bash
# round 5: WPT forward pipe group 4 (reverse 2) vs the default (2, 2)
set -o pipefail
mkdir -p gpurun_out
JWAVE_AMD_LIB=jwave_amd/lib/ab_p42.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "wpt" > gpurun_out/r05j3_parity.log 2>&1 || { tail -5 gpurun_out/r05j3_parity.log; exit 1; }
tail -1 gpurun_out/r05j3_parity.log
bash tools/gpu_ab_libs.sh wpt 5 jwave_amd/lib/ab_p22.so jwave_amd/lib/ab_p42.so 2>&1 | tee gpurun_out/r05j3_ab.txt
