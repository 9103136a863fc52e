#!/bin/bash
# round 5: forward resident column tails with one wave per column (fwt_fwd_col16) vs block per 8-column slab
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "fwt2d or fwt3d or parallel or rows_chunked or wpt2d" > gpurun_out/r05q2_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05q2_parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh fwt2d 4 jwave_amd/lib/ab_fc0.so jwave_amd/lib/ab_fc1.so 2>&1 | tee gpurun_out/r05q2_ab.txt
