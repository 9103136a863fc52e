#!/bin/bash
# round 5: ramped staging chunks for the pageable host entries
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "host_entry or reentr or aed or decompose" tests/test_jni_shim.py tests/test_multi.py > gpurun_out/r05s_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05s_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3 4; do for L in ab_ramp0 ab_ramp1; do
  timeout -k 10 120 python tools/host_entry_ab.py jwave_amd/lib/$L.so 5 || exit 1
done; done 2>&1 | tee gpurun_out/r05s_ab.txt
