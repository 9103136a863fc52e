#!/bin/bash
# round 6: multi-device 2-D / MODWT batch entries (device 0 listed several times) + JNI shim on GPU
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
O=gpurun_out/${1:-r06d}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_multi.py tests/test_jni_shim.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; exit $rc
