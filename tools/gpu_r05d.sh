#!/bin/bash
# round 5: fused row tails (fwt_fwd_tile1r / fwt_rev_tile1h) -- parity of the
# row-pass cases, then config 3 A/B: no fusion / forward only / both
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
mkdir -p gpurun_out/r05d
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fwt2d or rowcap or batch" > gpurun_out/r05d/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r05d/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/r05d/pytest.log | head -20; exit 1; }
L=jwave_amd/lib
bash tools/gpu_ab_libs.sh fwt2d 3 $L/ab_nofuse.so $L/ab_m00.so $L/libjwave_hip.so $L/ab_m22.so
