#!/bin/bash
# round 5: MODWT inverse geometry: 512 x 2048 (default) vs 1024 x 2048 vs 1024 x 4096
set -o pipefail
mkdir -p gpurun_out
for v in inv1024 inv1024t4; do
  JWAVE_AMD_LIB=jwave_amd/lib/ab_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k "modwt" > gpurun_out/r05x2_parity_$v.log 2>&1 || { tail -5 gpurun_out/r05x2_parity_$v.log; exit 1; }
  tail -1 gpurun_out/r05x2_parity_$v.log
done
bash tools/gpu_ab_libs.sh modwt 3 jwave_amd/lib/ab_inv512.so jwave_amd/lib/ab_inv1024.so jwave_amd/lib/ab_inv1024t4.so 2>&1 | tee gpurun_out/r05x2_ab.txt
