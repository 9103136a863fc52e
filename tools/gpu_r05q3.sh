#!/bin/bash
# round 5: reverse tiles level 0 as couples (default) vs one pair per lane (JWV_REV_COUPLE0=0)
set -o pipefail
mkdir -p gpurun_out
JWAVE_AMD_LIB=jwave_amd/lib/ab_c00.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "fwt2d or fwt3d or parallel or rows_chunked or wpt2d" > gpurun_out/r05q3_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05q3_parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh fwt2d 4 jwave_amd/lib/ab_c01.so jwave_amd/lib/ab_c00.so 2>&1 | tee gpurun_out/r05q3_ab.txt
