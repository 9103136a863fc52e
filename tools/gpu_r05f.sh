#!/bin/bash
# round 5: MODWT inverse with the W taps from global memory (no W window in
# LDS) -- parity of every MODWT case with the default build (WG, 512 x 2048),
# then config 5 A/B: base (W windows in LDS) / WG 512x2048 / WG 512x4096 /
# WG 1024x4096 / WG 256x2048
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
mkdir -p gpurun_out/r05f
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "modwt" > gpurun_out/r05f/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r05f/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/r05f/pytest.log | head -20; exit 1; }
L=jwave_amd/lib
for v in t4k t4k1k t2k256; do
  JWAVE_AMD_LIB=$L/ab_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "modwt_config5 or modwt_chunked or modwt_deep" > gpurun_out/r05f/pytest_$v.log 2>&1 || { echo "parity $v failed"; grep -E "FAILED|Error" gpurun_out/r05f/pytest_$v.log | head; exit 1; }
  tail -1 gpurun_out/r05f/pytest_$v.log
done
bash tools/gpu_ab_libs.sh modwt 3 $L/ab_base.so $L/libjwave_hip.so $L/ab_t4k.so $L/ab_t4k1k.so $L/ab_t2k256.so
