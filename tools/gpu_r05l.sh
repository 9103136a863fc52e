#!/bin/bash
# round 5: the FWT tiles' couples with products issued ahead of their adds
# (JWV_FWT_FPIPE / JWV_FWT_RPIPE; fp00 = off) -- parity of the FWT cases per
# build, config 3 and config 2 A/B -- after the MODWT A/B (gpu_r05k.sh)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
bash tools/gpu_r05k.sh || exit 1
O=gpurun_out/r05l; mkdir -p $O
L=jwave_amd/lib
for v in ab_fp22 ab_fp20; do
  JWAVE_AMD_LIB=$L/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fwt2d or rowcap or config2 or fwt_large or chain or axis or 3d" > $O/pytest_$v.log 2>&1 || { echo "parity $v failed"; grep -E "FAILED|Error" $O/pytest_$v.log | head; exit 1; }
  tail -1 $O/pytest_$v.log
done
bash tools/gpu_ab_libs.sh fwt2d 3 $L/ab_fp00.so $L/ab_fp22.so $L/ab_fp20.so
bash tools/gpu_ab_libs.sh fwt1d 3 $L/ab_fp00.so $L/ab_fp22.so $L/ab_fp20.so
