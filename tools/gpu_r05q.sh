#!/bin/bash
# round 5: two rows per wave in the deep levels of the wave-per-row tails (config 3)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "fwt2d or rowcap or batch or rows_chunked or fwt3d or wpt2d or parallel" > gpurun_out/r05q_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05q_parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh fwt2d 3 jwave_amd/lib/ab_nopair.so jwave_amd/lib/ab_pair.so 2>&1 | tee gpurun_out/r05q_ab.txt
