#!/bin/bash
# round 5: row reverse resident cap 1024 (default) vs 512
set -o pipefail
mkdir -p gpurun_out
JWAVE_AMD_LIB=jwave_amd/lib/ab_rt512.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "fwt2d or fwt3d or parallel or rows_chunked or wpt2d" > gpurun_out/r05q4_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05q4_parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh fwt2d 4 jwave_amd/lib/ab_rt1024.so jwave_amd/lib/ab_rt512.so 2>&1 | tee gpurun_out/r05q4_ab.txt
