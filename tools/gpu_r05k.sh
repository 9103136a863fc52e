#!/bin/bash
# round 5: MODWT sums with the products of G taps issued ahead of their adds
# (inverse run form JWV_MODINV_PIPE, streamed forward JWV_MODFWD_PIPE; m00 =
# the round-4 forms).  Parity of the MODWT cases per build, then config 5 A/B.
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
O=gpurun_out/r05k; mkdir -p $O
L=jwave_amd/lib
for v in ab_i2f2 ab_i2f0 ab_i0f2 ab_i4f4; do
  JWAVE_AMD_LIB=$L/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "modwt" > $O/pytest_$v.log 2>&1 || { echo "parity $v failed"; grep -E "FAILED|Error" $O/pytest_$v.log | head; exit 1; }
  tail -1 $O/pytest_$v.log
done
bash tools/gpu_ab_libs.sh modwt 3 $L/ab_m00.so $L/ab_i2f2.so $L/ab_i2f0.so $L/ab_i0f2.so $L/ab_i4f4.so
