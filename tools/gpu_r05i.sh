#!/bin/bash
# round 5: SGPR-limited residency of the config-3 row tiles (L = 16 taps in
# SGPRs): amdgpu_waves_per_eu 7 / 8 on the forward row tile (f7, f8) and 7 on
# the reverse (r7).  Parity of the 2-D / row-cap cases with every build, then
# config 3 A/B.
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
O=gpurun_out/r05i; mkdir -p $O
L=jwave_amd/lib
for v in f7 f8 f7r7 f8r7; do
  JWAVE_AMD_LIB=$L/ab_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fwt2d or rowcap or batch_rowcap" > $O/pytest_$v.log 2>&1 || { echo "parity $v failed"; grep -E "FAILED|Error" $O/pytest_$v.log | head; exit 1; }
  tail -1 $O/pytest_$v.log
done
bash tools/gpu_ab_libs.sh fwt2d 3 $L/libjwave_hip.so $L/ab_f7.so $L/ab_f8.so $L/ab_f7r7.so $L/ab_f8r7.so
