#!/bin/bash
# round 5: WPT pipe groups re-checked on the closing kernels: (F,R) = (2,2) default, (4,4), (2,4)
set -o pipefail
mkdir -p gpurun_out
for v in p44 p24; do
  JWAVE_AMD_LIB=jwave_amd/lib/ab_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k "wpt" > gpurun_out/r05j2_parity_$v.log 2>&1 || { tail -5 gpurun_out/r05j2_parity_$v.log; exit 1; }
  tail -1 gpurun_out/r05j2_parity_$v.log
done
bash tools/gpu_ab_libs.sh wpt 3 jwave_amd/lib/ab_p22.so jwave_amd/lib/ab_p44.so jwave_amd/lib/ab_p24.so 2>&1 | tee gpurun_out/r05j2_ab.txt
