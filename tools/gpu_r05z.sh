#!/bin/bash
# round 5: config-2 fused forward tail geometry: 2048-sample units x 512 threads (default) vs 1024 x 512 vs 1024 x 256
set -o pipefail
mkdir -p gpurun_out
for v in tb1024 tb1024n256; do
  JWAVE_AMD_LIB=jwave_amd/lib/ab_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k "fwt_large or config2 or fwt1d or plan or tail or epoch" > gpurun_out/r05z_parity_$v.log 2>&1 || { tail -5 gpurun_out/r05z_parity_$v.log; exit 1; }
  tail -1 gpurun_out/r05z_parity_$v.log
done
bash tools/gpu_ab_libs.sh fwt1d 5 jwave_amd/lib/ab_tb2048.so jwave_amd/lib/ab_tb1024.so jwave_amd/lib/ab_tb1024n256.so 2>&1 | tee gpurun_out/r05z_ab.txt
